#!/bin/bash
# SQ issue / wait breakdown and effective clock of the fused encode+CRC kernel (one PMC pass per counter set)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc5
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
W=${W:-c5}
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_WAVES"; do
  i=$((i+1))
  timeout -k 5 90 rocprofv3 --pmc $ctrs --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --no-cpu $EXTRA > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
