#!/bin/bash
# CRC32C / verify streaming kernel: run length per wave (crc_run) and grid A/B on the bench shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/crcrun; mkdir -p $O
for wl in crc verify; do
  timeout -k 10 300 python -u scripts/ab.py $wl crc_run ${RUNS:-262144,65536,131072,524288,1048576,32768} 5 > $O/ab_$wl.log 2>&1 || { tail -20 $O/ab_$wl.log; exit 1; }
  grep '"wl"' $O/ab_$wl.log
done
