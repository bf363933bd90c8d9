#!/bin/bash
# Streaming CRC kernel: (D, ring) variants, random vs all-zero data (clock / power sensitivity).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/crcab; mkdir -p $O
timeout -k 10 300 python -u scripts/ab.py crc crc_variant ${VARIANTS:-0,20,21,23,24} 5 > $O/ab_rand.log 2>&1 || { tail -20 $O/ab_rand.log; exit 1; }
grep '"wl"' $O/ab_rand.log
ZERO=1 timeout -k 10 300 python -u scripts/ab.py crc crc_variant 0 5 > $O/ab_zero.log 2>&1 || { tail -20 $O/ab_zero.log; exit 1; }
grep '"wl"' $O/ab_zero.log | sed 's/^/zero-data /'
