#!/bin/bash
# Round-5 GPU call: the fault probe's log phase, the whole GPU suite + smoke, the default bench line (C2 headline, every
# device-resident leg with rocprof + PMC, C5 e2e multi-process and in-process, JNI per-call rows, CPU baseline), then
# the probe's deterministic phase last (the one step that may fault).  Every GPU step has its own time limit; the
# chain stops at the first failure.
#   OUT=gpurun_out/r5a STEPS="probe tests bench fixed" scripts/gpu_r5.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r5}
STEPS=${STEPS:-probe tests bench fixed}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "[gpu_r5 $(date +%T)] $name" | tee -a "$OUT/steps.log" >&2
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[gpu_r5 $(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log" >&2
  return $rc
}
for s in $STEPS; do
  case $s in
    probe)
      for n in 65536 262144; do
        run "probe log $n" 150 env AMD_LOG_LEVEL=4 python -u scripts/fault_probe.py log $n \
          > "$OUT/probe_log_$n.out" 2> "$OUT/probe_log_$n.err" || exit 1
        gzip -f "$OUT/probe_log_$n.err"
      done ;;
    tests)
      run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 2; }
      tail -3 "$OUT/pytest_gpu.log"
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 3 ;;
    bench)
      run bench 900 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 4; } ;;
    jni)
      run jni 300 python -u bench.py --workload jni > "$OUT/bench_jni.json" 2> "$OUT/bench_jni.err" || exit 5 ;;
    rehearse)  # the N = 2 path on one GPU: two gloo ranks on device 0, C2 + C5 multi-process + in-process legs
      run rehearse 600 env OZEC_BENCH_SAME_DEVICE=1 OZEC_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 5 \
        --warmup 2 --no-legs --no-jni > "$OUT/bench_2rank.json" 2> "$OUT/bench_2rank.err" || { tail -20 "$OUT/bench_2rank.err"; exit 9; } ;;
    prof)  # rocprofv3 kernel statistics of the headline and of every leg with the bench's own warm-up and steps
      run "prof c2" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- python3 bench.py \
        --workload c2 --no-cpu --no-pmc --no-e2e --no-legs --no-jni > "$OUT/prof_c2.log" 2>&1 || exit 10
      run "prof legs" 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_legs" -o run --output-format csv -- python3 \
        bench.py --workload legs --no-cpu --no-pmc > "$OUT/prof_legs.log" 2>&1 || exit 11 ;;
    duplex)  # A/B of the duplex column chunks of pinned per-call coding (host_duplex), same process order each way
      i=0
      for t in 0 524288 0 524288; do
        i=$((i + 1))
        run "jni duplex=$t" 300 python -u bench.py --workload jni --tune host_duplex=$t > "$OUT/jni_duplex_${t}_$i.json" \
          2>> "$OUT/duplex.err" || exit 12
        run "host pinned duplex=$t" 300 python -u bench.py --workload host --host-pinned --threads 1 --steps 5 \
          --warmup 2 --tune host_duplex=$t > "$OUT/host_pinned_duplex_${t}_$i.json" 2>> "$OUT/duplex.err" || exit 13
      done ;;
    g6)  # same-process A/B of the 6-bit CRC groups (G6 variants 210-213) against the shipped 5-bit ones
      run "ab c3r" 300 python -u scripts/ab.py c3r crc_variant ${C3R:-0,177,210} ${ROUNDS:-6} > "$OUT/ab_c3r.log" 2>&1 \
        || { tail -20 "$OUT/ab_c3r.log"; exit 14; }
      run "ab c5dev" 300 python -u scripts/ab.py c5dev crc_variant ${C5:-0,171,211,212} ${ROUNDS:-6} \
        > "$OUT/ab_c5dev.log" 2>&1 || { tail -20 "$OUT/ab_c5dev.log"; exit 15; }
      run "ab c3" 300 python -u scripts/ab.py c3 crc_variant ${C3:-0,177,210} ${ROUNDS:-6} > "$OUT/ab_c3.log" 2>&1 \
        || { tail -20 "$OUT/ab_c3.log"; exit 16; } ;;
    ua)  # 16-B buffer loads / stores at unaligned byte offsets: bytes, bandwidth, the range edge (odd-length cells)
      [ -x scripts/unaligned_probe ] || { echo "scripts/unaligned_probe not built" >&2; exit 17; }
      run "unaligned probe" 120 scripts/unaligned_probe > "$OUT/unaligned_probe.json" 2> "$OUT/unaligned_probe.err" || exit 17 ;;
    abprev)  # the device-resident legs on the previous build (ab/libozec_prev.so) and this one, alternated
      for i in 1 2; do
        run "legs prev $i" 300 env OZEC_LIB_OVERRIDE=ab/libozec_prev.so python -u bench.py --workload legs --no-cpu \
          --no-pmc > "$OUT/legs_prev_$i.json" 2>> "$OUT/abprev.err" || exit 18
        run "legs new $i" 300 python -u bench.py --workload legs --no-cpu --no-pmc > "$OUT/legs_new_$i.json" \
          2>> "$OUT/abprev.err" || exit 19
      done ;;
    small)  # per-call time of small fused batches: fused kernel vs unfused kernels (fused_min_units)
      run "small batches" 400 python -u scripts/small_batch_ab.py ${ROUNDS:-5} > "$OUT/small_batch_ab.json" \
        2> "$OUT/small_batch_ab.err" || { tail -20 "$OUT/small_batch_ab.err"; exit 20; } ;;
    sq)  # SQ counters of each leg's dominant kernel, two passes (scripts/final_sq_summary.py writes sq_summary.json)
      P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
      P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
      for wl in ${SQ_WORKLOADS:-c3r c5dev c3 crc c4 c2}; do
        for p in 1 2; do
          eval PM=\$P$p
          run "sq $wl p$p" 120 rocprofv3 --pmc $PM --kernel-trace -d "$OUT/sq_${wl}_p$p" -o run --output-format csv -- \
            python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e --no-legs --no-jni \
            > "$OUT/sq_${wl}_p$p.log" 2>&1 || { tail -5 "$OUT/sq_${wl}_p$p.log"; exit 22; }
        done
      done
      python3 scripts/final_sq_summary.py "$OUT" > "$OUT/sq_summary.log" 2>&1 || exit 23 ;;
    recab)  # fused reconstruction A/B of rs-6-3 / rs-3-2 shapes (scripts/ab_single_erasure.py, VARIANTS)
      run "rec ab" 300 env SHAPES=all VARIANTS=${VARIANTS:-0,231} python -u scripts/ab_single_erasure.py ${ROUNDS:-6} \
        > "$OUT/ab_rec.log" 2>&1 || { tail -20 "$OUT/ab_rec.log"; exit 24; } ;;
    abcrc)  # same-process A/Bs of the streaming CRC kernel: compute (batched trees) and verify (run check)
      run "ab crc" 300 python -u scripts/ab.py crc crc_variant ${CRC:-0,28,29} ${ROUNDS:-6} > "$OUT/ab_crc.log" 2>&1 \
        || { tail -20 "$OUT/ab_crc.log"; exit 25; }
      run "ab verify" 300 python -u scripts/ab.py verify crc_variant ${VERIFY:-0,24} ${ROUNDS:-6} > "$OUT/ab_verify.log" \
        2>&1 || { tail -20 "$OUT/ab_verify.log"; exit 26; } ;;
    oddshapes)  # XOR / generic RS coding at odd byte offsets: previous build (byte kernel) vs this one (BUF kernels)
      run "odd shapes prev" 300 env OZEC_LIB_OVERRIDE=ab/libozec_prev.so python -u scripts/odd_shapes_ab.py prev \
        > "$OUT/odd_shapes_prev.json" 2> "$OUT/odd_shapes.err" || exit 27
      run "odd shapes new" 300 python -u scripts/odd_shapes_ab.py new > "$OUT/odd_shapes_new.json" \
        2>> "$OUT/odd_shapes.err" || exit 28 ;;
    oddbpc)  # CRC windows of any length / at odd offsets: previous build (byte kernel) vs this one (per-window kernel)
      run "odd bpc prev" 300 env OZEC_LIB_OVERRIDE=ab/libozec_prev.so python -u scripts/odd_bpc_ab.py prev \
        > "$OUT/odd_bpc_prev.json" 2> "$OUT/odd_bpc.err" || exit 29
      run "odd bpc new" 300 python -u scripts/odd_bpc_ab.py new > "$OUT/odd_bpc_new.json" 2>> "$OUT/odd_bpc.err" || exit 30 ;;
    wide)  # coding with units 2 GiB or more apart: previous build (typed / byte kernels) vs this one (WIDE)
      run "wide prev" 300 env OZEC_LIB_OVERRIDE=ab/libozec_prev.so python -u scripts/wide_ab.py prev \
        > "$OUT/wide_prev.json" 2> "$OUT/wide.err" || exit 31
      run "wide new" 300 python -u scripts/wide_ab.py new > "$OUT/wide_new.json" 2>> "$OUT/wide.err" || exit 32 ;;
    tail)
      run tail 300 python -u bench.py --workload tail > "$OUT/bench_tail.json" 2> "$OUT/bench_tail.err" || exit 6 ;;
    tailnp)  # the same with the host batches' device unit pitch = the cell length (host_pitch16=0)
      run "tail pitch=len" 300 python -u bench.py --workload tail --tune host_pitch16=0 > "$OUT/bench_tail_np.json" \
        2> "$OUT/bench_tail_np.err" || exit 21 ;;
    heap)
      for n in 65536 262144; do
        run "probe heap $n" 150 env AMD_LOG_LEVEL=4 python -u scripts/fault_probe.py heap $n \
          > "$OUT/probe_heap_$n.out" 2> "$OUT/probe_heap_$n.err"
        rc=$?
        gzip -f "$OUT/probe_heap_$n.err"
        [ $rc -eq 0 ] || exit 8
      done ;;
    fixed)
      for n in 65536 262144; do
        run "probe fixed $n" 150 env AMD_LOG_LEVEL=4 python -u scripts/fault_probe.py fixed $n \
          > "$OUT/probe_fixed_$n.out" 2> "$OUT/probe_fixed_$n.err"
        rc=$?
        gzip -f "$OUT/probe_fixed_$n.err"
        [ $rc -eq 0 ] || exit 7
      done ;;
  esac
done
echo "[gpu_r5 $(date +%T)] done" | tee -a "$OUT/steps.log"
