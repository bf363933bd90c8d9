#!/bin/bash
# One GPU session: parity tests, benches of every workload, rocprofv3 kernel trace of the headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for w in c2 c3 c4 c5 crc e2e; do
  timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/prof_c2.log 2>&1 || { echo "rocprof failed"; tail $O/prof_c2.log; exit 1; }
find $O/prof_c2 -name '*stats*' | head
