#!/bin/bash
# Round 3: free register shifts (XO) in the XOR codec's per-window fused kernel (crc_variant 4 / 5): parity, then
# same-process A/Bs on C4 (block-major 256 MiB blocks).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3c4xo}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_next.py -k "xor" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/ab.py c4 crc_variant 0,4,5 ${ROUNDS:-6} > $O/ab_c4.log 2>&1 || { tail $O/ab_c4.log; exit 1; }
grep -h '"wl"' $O/ab_c4.log
