#!/bin/bash
# Round 2: parity suite, C5 end to end, C4 on its block-major layout, the other side workloads, and a 2-rank
# rehearsal of the self-spawning --gpus launcher on one device.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for w in ${WORKLOADS:-c5 c4 c4s c5dev c3r c3 crc verify}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 3 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
OZEC_BENCH_SAME_DEVICE=1 OZEC_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --stripes 1024 --e2e-stripes 1024 > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -30 $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.json
