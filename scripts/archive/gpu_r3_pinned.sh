#!/bin/bash
# Round 3: per-call host path with pinned caller buffers (DMA in place) -- its tests and the other host-buffer tests,
# the per-call stream line with the pinned rows, and a 4-rank rehearsal of the bench on one GPU (gloo, per-rank arrays).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3pinned}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 600 python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_path or checksum" tests/test_gpu_e2e.py tests/test_stripe_queue.py tests/test_jni_glue.py tests/test_jni_marshal.py tests/test_host_abi.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --workload stream > $O/bench_stream.json 2> $O/bench_stream.err || { echo "stream failed"; tail $O/bench_stream.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_stream.json'))['calls']; print({k: v for k, v in d.items() if k.startswith('encode')})"
OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 400 python bench.py --gpus 4 --stripes 512 --e2e-stripes 1024 --no-cpu > $O/bench_4rank.json 2> $O/bench_4rank.err || { echo "4-rank failed"; tail -20 $O/bench_4rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_4rank.json')); print('4rank', d['value'], d['n_gpus'], d['n_ranks'], d['per_rank'], d['e2e'].get('per_rank'))"
