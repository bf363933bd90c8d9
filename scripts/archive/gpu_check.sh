#!/bin/bash
# One GPU session: parity tests, benches of every workload, rocprofv3 kernel trace + PMC traffic of C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for w in ${WORKLOADS:-c1 c2 c3 c3r c4 c5 crc verify e2e queue}; do
  timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
[ -n "$NOPROF" ] && exit 0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/prof_c2.log 2>&1 || { echo "rocprof failed"; tail $O/prof_c2.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --stats -d $O/pmc_c2_$ctr -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_c2_$ctr.log 2>&1 || { echo "pmc $ctr failed"; exit 1; }
done
echo prof done
