#!/bin/bash
# Round 3: grid-size sweeps (windows per wave) of nibble-kernel geometries on C3r / C5dev, one process per geometry.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$PWD:$PWD/tests/golden
O=gpurun_out/r3grid; mkdir -p $O
for spec in ${SPECS:-c3r:62 c3r:77 c3r:78 c5dev:87 c5dev:79 c5dev:68}; do
  wl=${spec%%:*}; v=${spec##*:}
  FIX=crc_variant=$v timeout -k 10 200 python -u scripts/ab.py $wl crc_grid ${GRIDS:-0,8192,4096,2048} ${ROUNDS:-3} > $O/${wl}_v$v.log 2>&1 || { tail $O/${wl}_v$v.log; exit 1; }
  grep '"wl"' $O/${wl}_v$v.log
done
