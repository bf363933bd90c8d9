#!/bin/bash
# GPU parity suite, then default vs round-1 (crc_variant=1) bench lines for the fused / CRC workloads.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/ab/pytest_gpu.log
for w in ${WORKLOADS:-c5 c4 c3r crc}; do
  for v in 0 1; do
    timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu --tune crc_variant=$v > gpurun_out/ab/bench_${w}_v$v.json 2> gpurun_out/ab/bench_${w}_v$v.err || { tail gpurun_out/ab/bench_${w}_v$v.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" gpurun_out/ab/bench_${w}_v$v.json $w $v
  done
done
