#!/bin/bash
# C4 reconciliation: the bench line and the same-process A/B of the XOR fused kernel in ONE call,
# then SQ / clock counters of C4 beside C2 (same read:write byte mix), one --pmc pass per counter group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=$R/gpurun_out/${OUT:-r4c4}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c4 --no-cpu --no-pmc > $O/bench_c4_$i.json 2> $O/bench_c4_$i.err || { tail $O/bench_c4_$i.err; exit 1; }
  timeout -k 10 300 python -u scripts/ab.py c4 crc_variant 0,4,5,2,3,20 ${ROUNDS:-5} > $O/ab_c4_$i.log 2>&1 || { tail -20 $O/ab_c4_$i.log; exit 1; }
done
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_c4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
grep -h median_ms $O/ab_c4_*.log
cd /tmp
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for wl in c4 c2; do
  for p in 1 2; do
    eval PM=\$P$p
    timeout -k 5 120 rocprofv3 --pmc $PM --kernel-trace -d $O/sq_${wl}_p$p -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 5 --warmup 5 --no-cpu --no-pmc --no-e2e --no-fused > $O/sq_${wl}_p$p.log 2>&1 || { echo "pmc $wl $p failed"; tail -5 $O/sq_${wl}_p$p.log; exit 1; }
  done
done
echo c4 done
