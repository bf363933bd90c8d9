#!/bin/bash
# GPU parity suite, interleaved A/B of the CRC kernel variants (per-window vs streaming), bench lines of the
# CRC compute and verify workloads.
set -o pipefail
O=gpurun_out/stream
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
CRCVARIANTS=${CRCVARIANTS:-0,13,11,20,21,23,24} C5VARIANTS=0 GRIDS=0 timeout -k 10 300 python scripts/tune_crc.py 5 > $O/tune_stream.log 2>&1 || { tail -20 $O/tune_stream.log; exit 1; }
grep -v amdgpu.ids $O/tune_stream.log
for w in crc verify; do
  for v in 0 13; do
    timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu --tune crc_variant=$v > $O/bench_${w}_v$v.json 2> $O/bench_${w}_v$v.err || { tail $O/bench_${w}_v$v.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" $O/bench_${w}_v$v.json $w $v
  done
done
