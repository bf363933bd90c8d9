#!/bin/bash
# Interleaved A/B of fused reconstruction (C3r) kernel variants: occupancy (waves per SIMD) vs D.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/abc3r
mkdir -p $O
for r in 1 2; do
  for v in ${VARIANTS:-0 11 15 16}; do
    for w in ${WORKLOADS:-c3r}; do
      timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu --tune crc_variant=$v > $O/${w}_v${v}_$r.json 2> $O/${w}_v${v}_$r.err || { tail $O/${w}_v${v}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" $O/${w}_v${v}_$r.json $w $v $r
    done
  done
done
