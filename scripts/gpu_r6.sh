#!/bin/bash
# Round-6 GPU session steps: OUT=gpurun_out/<tag>; each GPU step under its own time limit, chained with && so that a
# failed or faulting step ends the call (nothing further touches the GPU).
#   scripts/gpu_r6.sh <tag> probe suite smoke bench ...
set -o pipefail
tag=$1
shift
OUT=gpurun_out/$tag
mkdir -p "$OUT"
step() { echo "[gpu_r6 $(date +%H:%M:%S)] $*" | tee -a "$OUT/steps.log"; }
run() {
  local what=$1
  case $what in
    probe)
      step probe
      timeout -k 10 120 python -u scripts/lock_probe.py > "$OUT/lock_probe.out" 2>&1 ;;
    suite)
      step "pytest -m gpu"
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke)
      step smoke
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      step "bench default"
      OZEC_BENCH_FULL=$OUT/bench_full.json timeout -k 10 900 python -u bench.py > "$OUT/bench.json" \
        2> "$OUT/bench.err" ;;
    percall)
      step "percall probe"
      { timeout -k 10 120 scripts/percall_probe 1048576 200 && timeout -k 10 120 scripts/percall_probe 65536 500; } \
        > "$OUT/percall.json" 2> "$OUT/percall.err" ;;
    d2h)
      step "d2h probe"
      timeout -k 10 120 scripts/d2h_probe > "$OUT/d2h.json" 2> "$OUT/d2h.err" ;;
    engines)
      step "stream engine probe"
      { timeout -k 10 120 scripts/stream_engine_probe 8 && HSA_ENABLE_SDMA=0 timeout -k 10 120 scripts/stream_engine_probe 8; } \
        > "$OUT/engines.json" 2> "$OUT/engines.err" ;;
    jni)
      step "bench jni rows"
      timeout -k 10 300 python -u bench.py --workload jni > "$OUT/jni.json" 2> "$OUT/jni.err" ;;
    *)
      step "unknown step $what"
      return 2 ;;
  esac
  local rc=$?
  step "$what rc=$rc"
  return $rc
}
for s in "$@"; do
  run "$s" || exit $?
done
step done
