#!/bin/bash
# What one more VALU instruction per step costs the fused kernels (variants 40 / 41 add 64 / 192 independent
# v_xor_b32 per wave-step): if the kernel is VALU-issue-bound, time grows by the pad's issue cost.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/valupad
mkdir -p $O
for rep in 1 2; do
  for w in ${WLS:-c5dev c3r}; do
    for v in ${VARS:-0 40 41}; do
      timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu --no-pmc --tune crc_variant=$v > $O/${w}_${v}_$rep.json 2>$O/err.log || { echo "$w $v failed"; tail $O/err.log; exit 1; }
      python -c "import json;d=json.load(open('$O/${w}_${v}_$rep.json'));print('$w', $v, d['roofline']['kernel_ms'])"
    done
  done
done
