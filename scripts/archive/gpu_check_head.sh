#!/bin/bash
# Whole-tree check on the GPU box: GPU parity suite, smoke(), default bench line (N=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/head; mkdir -p $O
if [ -z "$BENCH_ONLY" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
grep -v amdgpu.ids $O/smoke.log
fi
t0=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail -30 $O/bench_default.err; exit 1; }
echo "default bench wall: $(( $(date +%s) - t0 )) s"
cat $O/bench_default.json
