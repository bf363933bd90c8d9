#!/bin/bash
# Round-2 evidence on one MI355X: the whole GPU suite, smoke(), the default bench line, every workload's line (live
# PMC traffic where bench.py takes it), rocprofv3 kernel stats of the main kernels, and a 2-rank rehearsal of the
# multi-rank launcher on the one device.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
grep -v amdgpu.ids $O/smoke.log
t0=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
echo "default bench: $(( $(date +%s) - t0 )) s"
for w in ${WORKLOADS:-c1 c3 c3r c3r_host c4 c5dev crc verify queue host stream}; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  echo "bench $w ok"
done
timeout -k 10 300 python bench.py --workload c3 --erased 1,4,10,13 > $O/bench_c3_mixed.json 2> $O/bench_c3_mixed.err || { echo "c3 mixed failed"; exit 1; }
timeout -k 10 300 python bench.py --workload c3r --erased 1,4,10,13 > $O/bench_c3r_mixed.json 2> $O/bench_c3r_mixed.err || { echo "c3r mixed failed"; exit 1; }
OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --stripes 1024 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -20 $O/bench_2rank.err; exit 1; }
echo "2-rank ok"
export TMPDIR=/tmp
cd /tmp
for w in ${PROF_WORKLOADS:-c2 c3 c3r c5dev crc}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 10 --warmup 10 --no-cpu --no-pmc --no-e2e > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  echo "profiled $w"
done
echo final done
