#!/bin/bash
# SQ issue / wait / LDS counters and the effective clock of the fused kernels' current defaults, one rocprofv3
# --pmc pass per counter set (each within the per-block limits: 8 SQ, 2 GRBM).  Usage: W="c5dev c3r" bash ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sqpmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 5 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
for w in ${W:-c5dev c3r}; do
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_WAVES" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -k 5 120 rocprofv3 --pmc $ctrs --kernel-trace -d $O/${w}_p$i -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu --no-pmc $EXTRA > $O/${w}_p$i.log 2>&1 || { echo "pmc $w pass $i failed"; tail -5 $O/${w}_p$i.log; }
  done
done
echo done
