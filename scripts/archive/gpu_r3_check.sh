#!/bin/bash
# Round 3: the GPU suite (or a -k subset), then optional bench workloads; every step time-limited, stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3check}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
if [ -z "$NOTEST" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for w in $WORKLOADS; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --workload $w $BENCH_ARGS > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
  echo "bench $w ok"
done
echo check done
