#!/bin/bash
# Nibble-table kernel: parity of its variants (tests -k nibble/variants/reconstruct) and same-process A/Bs on C3r / C5dev.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$PWD:$PWD/tests/golden
O=gpurun_out/nb; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_next.py -k "nibble or variants or reconstruct_crc_batch" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
timeout -k 10 200 python -u scripts/ab.py c3r crc_variant ${C3R:-0,62} ${ROUNDS:-5} > $O/ab_c3r.log 2>&1 || { tail $O/ab_c3r.log; exit 1; }
timeout -k 10 200 python -u scripts/ab.py c5dev crc_variant ${C5:-0,61} ${ROUNDS:-5} > $O/ab_c5dev.log 2>&1 || { tail $O/ab_c5dev.log; exit 1; }
grep '"wl"' $O/ab_c3r.log $O/ab_c5dev.log
