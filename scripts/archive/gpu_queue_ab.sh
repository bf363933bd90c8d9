#!/bin/bash
# A/B of the stripe-queue ring depth (queue_batches) on pinned and pageable cells.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for w in ${WLS:-queue}; do
for nb in ${NBS:-3 4 6 8}; do
  timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu --tune queue_batches=$nb > $O/qab_${w}_$nb.json 2> $O/qab_${w}_$nb.err || { echo "bench $w $nb failed"; tail $O/qab_${w}_$nb.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['pcie']['value_frac_of_duplex_h2d'])" $O/qab_${w}_$nb.json $w $nb
done
done
