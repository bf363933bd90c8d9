#!/bin/bash
# Round evidence in one GPU session: parity tests, then per workload a bench line, a rocprofv3 kernel-trace
# summary and separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md rocprofv3 section).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/full
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for w in ${WORKLOADS:-c2 c3 c3r c4 c5 crc verify e2e host queue}; do
  timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
[ -n "$NOPROF" ] && exit 0
export TMPDIR=/tmp
cd /tmp
for w in ${PROF_WORKLOADS:-c2 c3 c3r c4 c5 crc verify}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 10 --warmup 3 --no-cpu > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --stats -d $O/pmc_${w}_$ctr -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu > $O/pmc_${w}_$ctr.log 2>&1 || { echo "pmc $w $ctr failed"; exit 1; }
  done
  echo "profiled $w"
done
echo full done
