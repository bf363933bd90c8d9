#!/bin/bash
# SQ counter passes (LDS pipe, VALU issue, waits) of the nibble-table kernel beside the streamed-input kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/nbsq; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"
for spec in ${SPECS:-c3r:0 c3r:62 c5dev:0 c5dev:61}; do
  wl=${spec%%:*}; v=${spec##*:}
  for p in 1 2; do
    eval PM=\$P$p
    timeout -k 5 120 rocprofv3 --pmc $PM --kernel-trace -d $O/${wl}_v${v}_p$p -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e --tune crc_variant=$v > $O/${wl}_v${v}_p$p.log 2>&1 || { echo "pmc $wl $v $p failed"; tail -5 $O/${wl}_v${v}_p$p.log; exit 1; }
  done
done
echo done
