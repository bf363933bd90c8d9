# host-buffer paths: parity of the staged pipeline / stripe queue, then throughput at 1/4/8/16 caller threads
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_rawcoder_api.py tests/test_stripe_queue.py tests/test_coder_benchmark.py -q -m gpu -k "host or concurrent or golden or queue or benchmark" > gpurun_out/host_test.log 2>&1
for T in 1 4 8 16; do
  timeout -k 10 180 python bench.py --workload host --threads $T --stripes 128 --steps 5 --warmup 2 --cpu-seconds 1 >> gpurun_out/host_bench.log 2>&1
done
for w in queue queue_pageable; do
  timeout -k 10 180 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu >> gpurun_out/host_bench.log 2>&1
done
