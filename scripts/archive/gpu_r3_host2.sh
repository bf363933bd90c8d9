#!/bin/bash
# Round 3: per-call host encode (1 MiB cells) at T threads vs the staging chunk size; 2-rank rehearsal with per-rank arrays.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r3host2; mkdir -p $O
for t in ${TS:-1 4 16}; do for ch in ${CHS:-4194304 1048576 524288 262144 131072}; do
  f=$O/host_t${t}_ch${ch}.json
  timeout -k 10 300 python bench.py --workload host --threads $t --stripes 256 --no-cpu --tune host_chunk=$ch > $f 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('host T=$t ch=$ch', d['value'], d['pcie']['value_frac_of_duplex_h2d'])"
done; done
if [ -z "$NO2RANK" ]; then
OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --stripes 1024 --e2e-stripes 2048 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -20 $O/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank.json')); print('2rank', d['value'], d['n_ranks'], d['per_rank'], d['e2e'].get('per_rank'))"
fi
