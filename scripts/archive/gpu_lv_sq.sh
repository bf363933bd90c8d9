#!/bin/bash
# Streamed-input fused kernel: effective clock and SQ issue/wait breakdown (one rocprofv3 --pmc pass per kernel),
# plus an A/B of random vs all-zero data (data-dependent power/clock).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/lvsq; mkdir -p $O
for wl in c5dev c3r; do
  timeout -k 10 200 python -u scripts/ab.py $wl crc_variant ${VARIANTS:-49,0} 3 > $O/ab_rand_$wl.log 2>&1 || { tail $O/ab_rand_$wl.log; exit 1; }
  grep '"wl"' $O/ab_rand_$wl.log
done
ZERO=1 timeout -k 10 200 python -u scripts/ab.py c5dev crc_variant ${VARIANTS:-49,0} 3 > $O/ab_zero_c5dev.log 2>&1 || { tail $O/ab_zero_c5dev.log; exit 1; }
grep '"wl"' $O/ab_zero_c5dev.log | sed 's/^/zero-data /'
export TMPDIR=/tmp
cd /tmp
for wl in c5dev c3r; do
  for v in $(echo ${VARIANTS:-49,0} | tr , ' '); do
    timeout -k 5 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --kernel-trace -d $O/${wl}_v$v -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e --tune crc_variant=$v > $O/${wl}_v$v.log 2>&1 || { echo "pmc $wl $v failed"; tail -5 $O/${wl}_v$v.log; exit 1; }
  done
done
echo done
