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
    pipeline)
      step "pipeline probe"
      timeout -k 10 200 scripts/pipeline_probe 1048576 200 > "$OUT/pipeline.json" 2> "$OUT/pipeline.err" ;;
    fusedab)
      step "fused vs unfused A/B (WIDE, XOR TAIL)"
      timeout -k 10 400 python -u scripts/fused_ab_r6.py > "$OUT/fused_ab.json" 2> "$OUT/fused_ab.err" ;;
    d2h)
      step "d2h probe"
      timeout -k 10 120 scripts/d2h_probe > "$OUT/d2h.json" 2> "$OUT/d2h.err" ;;
    engines)
      step "stream engine probe"
      { timeout -k 10 120 scripts/stream_engine_probe ${ENGINE_STREAMS:-8} ${ENGINE_HOW:-0} && HSA_ENABLE_SDMA=0 \
          timeout -k 10 120 scripts/stream_engine_probe ${ENGINE_STREAMS:-8} ${ENGINE_HOW:-0}; } \
        > "$OUT/engines.json" 2> "$OUT/engines.err" ;;
    prof)  # rocprofv3 kernel statistics of the headline and of every leg with the bench's own warm-up and steps
      step "rocprof c2 + legs"
      (cd /tmp && export TMPDIR=/tmp) && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run \
        --output-format csv -- python3 bench.py --workload c2 --no-cpu --no-pmc --no-e2e --no-legs --no-jni \
        > "$OUT/prof_c2.log" 2>&1 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_legs" -o run \
        --output-format csv -- python3 bench.py --workload legs --no-cpu --no-pmc > "$OUT/prof_legs.log" 2>&1 ;;
    rehearse)  # the driver's N = 2 launch (torchrun, two ranks) on one GPU: two gloo ranks on device 0, default line
      step "rehearse N=2"
      OZEC_BENCH_SAME_DEVICE=1 OZEC_DIST_BACKEND=gloo OZEC_BENCH_FULL=$OUT/bench_2rank_full.json timeout -k 10 900 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
        bench.py --gpus 2 --steps 5 --warmup 3 > "$OUT/bench_2rank.json" 2> "$OUT/bench_2rank.err" ;;
    jni)
      step "bench jni rows"
      timeout -k 10 300 python -u bench.py --workload jni > "$OUT/jni.json" 2> "$OUT/jni.err" ;;
    jnisweep)
      # the JNI heap-array forms (OZEC_JNI_HEAP auto / cb / arena) x libozec tunings (JNI_TUNES, one OZEC_TUNE each)
      step "jni sweep"
      gcc -O2 -I tests/native/mockjni -I include jni/ozec_jni.c jni/ozec_marshal.c tests/native/mockjni/mockjni.c \
        tests/native/jni_percall.c -L ozone_amd/lib -lozec -lpthread \
        -Wl,--wrap=ozec_encode,--wrap=ozec_decode,--wrap=ozec_crc_update,--wrap=ozec_checksum_windows \
        -Wl,--wrap=ozec_encode_cb,--wrap=ozec_decode_cb,--wrap=ozec_host_alloc,--wrap=ozec_host_free \
        -Wl,-rpath,"$PWD/ozone_amd/lib" -o "$OUT/jni_percall" || return 1
      local specs="" m c t
      for m in encode decode; do for c in 65536 1048576; do for t in 1 4 16; do specs="$specs $m:6:3:$c:$t"; done; done; done
      for heap in ${JNI_HEAPS:-auto cb arena}; do
        for tune in ${JNI_TUNES:-host_zero_copy=48 host_zero_copy=0}; do
          echo "# heap=$heap tune=$tune" >> "$OUT/jnisweep.json"
          OZEC_JNI_HEAP=$heap OZEC_TUNE=$tune timeout -k 10 120 "$OUT/jni_percall" 0.5 ${JNI_SPECS:-$specs} \
            >> "$OUT/jnisweep.json" 2>> "$OUT/jnisweep.err" || return 1
        done
      done ;;
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
