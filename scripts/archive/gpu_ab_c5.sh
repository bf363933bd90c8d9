#!/bin/bash
# Variant parity, then interleaved A/B of C5 fused kernel variants (crc_variant).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/abc5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variants_vs_oracle" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_variants.log 2>&1 || { tail -30 $O/pytest_variants.log; exit 1; }
tail -1 $O/pytest_variants.log
for r in 1 2; do
  for v in ${VARIANTS:-0 15 16}; do
    timeout -k 10 120 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu --tune crc_variant=$v > $O/c5_v${v}_$r.json 2> $O/c5_v${v}_$r.err || { tail $O/c5_v${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', sys.argv[2], sys.argv[3], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" $O/c5_v${v}_$r.json $v $r
  done
done
