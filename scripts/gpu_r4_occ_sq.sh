#!/bin/bash
# SQ counters of the rs-10-4 nibble kernel at 16 / 20 / 28 resident waves per CU: the default 177
# beside the half-dword-fence probes 199 (16-wave workgroups), 197 (two 10-wave), 200 (two 14-wave); one --pmc pass
# per counter group, each under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r4occ}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P3="GRBM_GUI_ACTIVE SQC_ICACHE_MISSES SQC_ICACHE_HITS"
P4="GRBM_GUI_ACTIVE SQ_WAVES SQ_IFETCH SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
for v in ${VARIANTS:-0 199 197 200}; do
  for p in 1 2 3 4; do
    eval PM=\$P$p
    timeout -k 5 120 rocprofv3 --pmc $PM --kernel-trace -d $O/sq_v${v}_p$p -o run --output-format csv -- python3 $R/bench.py --workload c3r --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e --no-fused --tune crc_variant=$v > $O/sq_v${v}_p$p.log 2>&1 || { echo "pmc v$v p$p failed"; tail -5 $O/sq_v${v}_p$p.log; exit 1; }
  done
  echo "variant $v done"
done
echo occ done
