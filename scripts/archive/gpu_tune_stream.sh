#!/bin/bash
# Interleaved A/B (scripts/tune_crc.py) of the streaming kernels over grid sizes: a persistent grid (0) gives
# each wave a long run of windows; larger grids give shorter runs and dispatch-order locality.
set -o pipefail
O=gpurun_out/tune2
mkdir -p $O
C5VARIANTS=-1 C4VARIANTS=${C4V:-0,13} CRCVARIANTS=${CRCV:-0,13} GRIDS=${GRIDS:-0,4096,16384,65536} timeout -k 10 500 python scripts/tune_crc.py ${ROUNDS:-3} > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -v amdgpu.ids $O/tune.log
