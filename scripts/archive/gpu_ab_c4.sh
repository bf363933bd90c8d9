#!/bin/bash
# GPU parity suite, then the fused XOR encode + CRC workload (C4) per kernel variant, interleaved twice:
# 0 = streaming default, 20 / 21 = streaming with a 2 / 4-step ring, 13 = per-window kernel.
set -o pipefail
O=gpurun_out/c4ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  for v in ${VARIANTS:-0 20 21 13}; do
    timeout -k 10 240 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu --tune crc_variant=$v > $O/bench_c4_v${v}_r$r.json 2> $O/bench_c4_v${v}_r$r.err || { tail $O/bench_c4_v${v}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" $O/bench_c4_v${v}_r$r.json $v
  done
done
