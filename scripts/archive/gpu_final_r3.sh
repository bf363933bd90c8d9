#!/bin/bash
# Round-3 evidence on one MI355X, in three calls (each under gpurun's 20-minute limit):
#   PHASE=a  the whole GPU suite, smoke(), the default bench line, a 2-rank rehearsal with per-rank arrays;
#   PHASE=b  every workload's line (live PMC traffic and rocprof clocks where bench.py takes them);
#   PHASE=c  the mixed erasure sets, the per-call host encode at T threads, rocprofv3 kernel stats of the main kernels
#            with the bench's own warmup/steps, SQ counter passes of the fused defaults.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3final}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
if [ "${PHASE:-a}" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
  grep -v amdgpu.ids $O/smoke.log
  t0=$(date +%s)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
  echo "default bench: $(( $(date +%s) - t0 )) s"
  OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --stripes 1024 --e2e-stripes 2048 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -20 $O/bench_2rank.err; exit 1; }
  echo "2-rank ok"
  exit 0
fi
if [ "${PHASE}" = b ]; then
for w in ${WORKLOADS:-c1 c3 c3r c3r_host c4 c5dev crc verify queue queue_pageable host stream}; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  echo "bench $w ok"
done
echo workloads done
exit 0
fi
if [ -n "$CTESTS" ]; then  # the GPU tests of the host-buffer paths (staging copies), before the lines
  timeout -k 10 600 python -u -m pytest $CTESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_host_paths.log 2>&1 || { echo "host-path tests failed"; tail -30 $O/pytest_host_paths.log; exit 1; }
  tail -1 $O/pytest_host_paths.log
fi
for w in ${CWORKLOADS:-crc verify}; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
done
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant 0,150,102,62,173 6 > $O/ab_c3r_defaults.log 2>&1 || { tail $O/ab_c3r_defaults.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant 0,167,163,87,174 6 > $O/ab_c5dev_defaults.log 2>&1 || { tail $O/ab_c5dev_defaults.log; exit 1; }
grep -h '"wl"' $O/ab_c3r_defaults.log $O/ab_c5dev_defaults.log
timeout -k 10 300 python bench.py --workload c3 --erased 1,4,10,13 > $O/bench_c3_mixed.json 2> $O/bench_c3_mixed.err || { echo "c3 mixed failed"; exit 1; }
timeout -k 10 300 python bench.py --workload c3r --erased 1,4,10,13 > $O/bench_c3r_mixed.json 2> $O/bench_c3r_mixed.err || { echo "c3r mixed failed"; exit 1; }
for t in 4 8 16; do
  timeout -k 10 300 python bench.py --workload host --threads $t --no-cpu > $O/bench_host_t$t.json 2> $O/bench_host_t$t.err || { echo "host T=$t failed"; exit 1; }
done
# staging copies with plain memcpy (copy_stream=0) beside the default streaming stores
for t in 1 16; do
  timeout -k 10 300 python bench.py --workload host --threads $t --no-cpu --tune copy_stream=0 > $O/bench_host_t${t}_memcpy.json 2> $O/bench_host_t${t}_memcpy.err || { echo "host memcpy T=$t failed"; exit 1; }
done
timeout -k 10 300 python bench.py --workload queue_pageable --no-cpu --tune copy_stream=0 > $O/bench_queue_pageable_memcpy.json 2> $O/bench_queue_pageable_memcpy.err || { echo "queue_pageable memcpy failed"; exit 1; }
echo "mixed + host T ok"
export TMPDIR=/tmp
cd /tmp
for w in ${PROF_WORKLOADS:-c2 c3 c3r c5dev crc}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --no-cpu --no-pmc --no-e2e > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  echo "profiled $w"
done
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"
for wl in c3r c5dev; do
  for p in 1 2; do
    eval PM=\$P$p
    timeout -k 5 120 rocprofv3 --pmc $PM --kernel-trace -d $O/sq_${wl}_p$p -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e > $O/sq_${wl}_p$p.log 2>&1 || { echo "pmc $wl $p failed"; tail -5 $O/sq_${wl}_p$p.log; exit 1; }
  done
done
echo final done
