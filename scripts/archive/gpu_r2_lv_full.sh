#!/bin/bash
# Round-2 evidence for the streamed-input fused kernel: whole GPU suite, smoke, bench lines of the fused
# workloads (live PMC traffic included), rocprofv3 kernel stats of the same commands.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r2lv; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/pytest_gpu.log
[ -n "$NOTEST" ] || timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
[ -n "$NOTEST" ] || grep -v amdgpu.ids $O/smoke.log
for w in ${WORKLOADS:-c5dev c3r c5 queue}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  cut -c1-600 $O/bench_$w.json
done
export TMPDIR=/tmp
cd /tmp
for w in ${PROF_WORKLOADS:-c5dev c3r}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 10 --warmup 3 --no-cpu --no-pmc > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  echo "profiled $w"
done
