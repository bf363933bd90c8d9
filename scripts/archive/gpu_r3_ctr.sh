#!/bin/bash
# Round 3: instruction-fetch, issue and LDS counters of the shipped nibble-kernel defaults (one --pmc pass per group).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3ctr}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU"
P2="GRBM_GUI_ACTIVE SQC_ICACHE_MISSES SQC_ICACHE_HITS"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_ANY"
P4="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
for spec in ${SPECS:-c3r:0 c5dev:0}; do
  wl=${spec%%:*}; v=${spec##*:}
  for p in ${PASSES:-1 2 3 4}; do
    eval PM=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $PM --kernel-trace -d $O/${wl}_v${v}_p$p -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e --tune crc_variant=$v > $O/${wl}_v${v}_p$p.log 2>&1 || { echo "pmc $wl $v $p failed"; tail -5 $O/${wl}_v${v}_p$p.log; exit 1; }
    echo "ok $wl $v $p"
  done
done
