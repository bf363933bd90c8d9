#!/bin/bash
# Round 2 check: GPU parity suite, then the default bench line (c2 + C5 e2e leg + live PMC traffic + CPU baselines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r2a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
