#!/bin/bash
# Streamed-input fused kernel (fused.hip): fused parity tests, then interleaved A/B against the per-window kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/lv; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_next.py -m gpu -x -q -k "encode_crc or reconstruct" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
for wl in ${WLS:-c5dev c3r}; do
  timeout -k 10 300 python -u scripts/ab.py $wl crc_variant ${VARIANTS:-49,0,51,52,53,54,55,56,57,58} 3 > $O/ab_$wl.log 2>&1 || { tail -20 $O/ab_$wl.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$wl.log
done
