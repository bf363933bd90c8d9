#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python bench.py --workload c3r --steps 10 --warmup 3 > $O/bench_c3r.json 2>$O/bench_c3r.err || { echo c3r failed; tail $O/bench_c3r.err; exit 1; }
cat $O/bench_c3r.json
OZEC_DIST_BACKEND=gloo OZEC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --stripes 512 > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo 2rank failed; tail -20 $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.json
PADS=0,256,4096,65536 timeout -k 10 500 python scripts/tune_layout.py 3 > $O/tune_layout.log 2>&1 || { echo layout failed; tail $O/tune_layout.log; exit 1; }
grep -v amdgpu.ids $O/tune_layout.log
