#!/bin/bash
# 2-rank rehearsal of bench.py's own launcher on one device (gloo for the control collectives), stdout checked to
# be exactly one JSON line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r2rank; mkdir -p $O
OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --stripes 1024 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -20 $O/bench_2rank.err; exit 1; }
python -c "import json,sys; L=[l for l in open(sys.argv[1]) if l.strip()]; assert len(L)==1, L; d=json.loads(L[0]); print('one JSON line:', d['n_gpus'], d['n_ranks'], d['value'], d['e2e']['value'], d['e2e']['stripes_per_gpu'])" $O/bench_2rank.json
