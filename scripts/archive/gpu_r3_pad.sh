#!/bin/bash
# Round 3: which pipe sets the nibble kernel's time -- marginal cost of 64 / 192 more VALU (140/141, 144/145) or
# 16 / 48 more LDS reads (142/143, 146/147) per wave-step -- and the per-call host encode at T threads with the
# adaptive staging chunk; then the reconstruction tests through the new rs-10-x default (102).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r3pad; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_next.py tests/test_gpu_e2e.py -k "${TESTK:-reconstruct or c3r or nibble or 14}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant ${C3R:-62,0,140,141,142,143} ${ROUNDS:-5} > $O/ab_c3r.log 2>&1 || { tail $O/ab_c3r.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant ${C5:-0,144,145,146,147} ${ROUNDS:-5} > $O/ab_c5dev.log 2>&1 || { tail $O/ab_c5dev.log; exit 1; }
grep '"wl"' $O/ab_c3r.log $O/ab_c5dev.log
for t in ${TS:-1 4 8 16}; do
  f=$O/host_t$t.json
  timeout -k 10 300 python bench.py --workload host --threads $t --stripes 256 --no-cpu > $f 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('host T=$t', d['value'], d['pcie']['value_frac_of_duplex_h2d'])"
done
