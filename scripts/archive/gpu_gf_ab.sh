#!/bin/bash
# Coding-kernel variants (gf_variant): parity tests of the coding path, then interleaved A/B on C3 and C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/gfab; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variant or decode or encode" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/pytest.log
for wl in ${WLS:-c3 c2}; do
  timeout -k 10 300 python -u scripts/ab.py $wl gf_variant ${VARIANTS:-0,11,12,13} 5 > $O/ab_$wl.log 2>&1 || { tail -20 $O/ab_$wl.log; exit 1; }
  grep -E '"wl"|false' $O/ab_$wl.log
done
