#!/bin/bash
# Evidence for the nibble-table fused kernel as default: whole GPU suite, smoke, bench lines of the fused workloads
# (live PMC traffic), rocprofv3 kernel stats of C3r / C5dev.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/nbfinal; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
grep -v amdgpu.ids $O/smoke.log
fi
for w in ${WORKLOADS:-c3r c5dev c5 c3r_host queue}; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  echo "bench $w ok"
done
timeout -k 10 300 python bench.py --workload c3r --erased 1,4,10,13 > $O/bench_c3r_mixed.json 2> $O/bench_c3r_mixed.err || { echo "c3r mixed failed"; exit 1; }
export TMPDIR=/tmp
cd /tmp
for w in ${PROF_WORKLOADS:-c3r c5dev}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 10 --warmup 10 --no-cpu --no-pmc --no-e2e > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  echo "profiled $w"
done
echo final done
