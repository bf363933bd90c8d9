#!/bin/bash
# Round 3: stripe-queue batch sizes, and the per-call host encode at T threads under staging knobs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r3host; mkdir -p $O
for b in ${QB:-16 32 64}; do
  timeout -k 10 300 python bench.py --workload queue --queue-batch $b --no-cpu > $O/queue_b$b.json 2> $O/queue_b$b.err || { tail $O/queue_b$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/queue_b$b.json')); print('queue batch $b', d['value'], d['pcie']['value_frac_of_duplex_h2d'])"
done
for t in ${TS:-8 16}; do for ct in ${CTS:-7 15}; do for ch in ${CHS:-4194304 262144}; do for sl in ${SLS:-8 16}; do
  f=$O/host_t${t}_ct${ct}_ch${ch}_sl${sl}.json
  timeout -k 10 300 python bench.py --workload host --threads $t --stripes 256 --no-cpu --tune copy_threads=$ct --tune host_chunk=$ch --tune host_slots=$sl > $f 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('host T=$t ct=$ct ch=$ch slots=$sl', d['value'], d['pcie']['value_frac_of_duplex_h2d'])"
done; done; done; done
