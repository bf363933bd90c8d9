#!/bin/bash
# Round 3: free register shifts (XO) in the streaming CRC kernel (crc_variant 25-27): parity, then same-process A/Bs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3crcxo}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "stream_runs_cross_cells or checksum" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/ab.py crc crc_variant 0,25,26,27 ${ROUNDS:-6} > $O/ab_crc.log 2>&1 || { tail $O/ab_crc.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py verify crc_variant 0,25,26,27 ${ROUNDS:-6} > $O/ab_verify.log 2>&1 || { tail $O/ab_verify.log; exit 1; }
grep -h '"wl"' $O/ab_crc.log $O/ab_verify.log
