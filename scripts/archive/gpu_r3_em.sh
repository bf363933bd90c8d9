#!/bin/bash
# Round 3: lane-parallel emit of the window CRCs (EM, variants 170-174) -- parity tests of the new variants, then
# same-process A/Bs against the XO defaults (150 rs-10-x, 167 rs-6-x).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3em}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "${KSEL:-17}" \
  tests/test_gpu_parity.py::test_encode_crc_nibble_kernel_vs_oracle tests/test_gpu_parity.py::test_encode_crc_rs63_variants_vs_oracle \
  tests/test_gpu_parity.py::test_encode_crc_other_shapes_variants_vs_oracle tests/test_gpu_next.py::test_reconstruct_crc_batch \
  > $O/pytest_em.log 2>&1 || { tail -30 $O/pytest_em.log; exit 1; }
tail -2 $O/pytest_em.log
fi
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant ${C3R:-150,170,173} ${ROUNDS:-5} > $O/ab_c3r.log 2>&1 || { tail $O/ab_c3r.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant ${C5:-167,171,172,174} ${ROUNDS:-5} > $O/ab_c5dev.log 2>&1 || { tail $O/ab_c5dev.log; exit 1; }
grep -h '"wl"\|false' $O/ab_c3r.log $O/ab_c5dev.log
