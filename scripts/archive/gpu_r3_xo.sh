#!/bin/bash
# Round 3: free output-register shifts (XO, variants 150-158) -- bit-exact vs the default, then same-process A/Bs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3xo}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant ${C3R:-0,150,151,154,158} ${ROUNDS:-5} > $O/ab_c3r.log 2>&1 || { tail $O/ab_c3r.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant ${C5:-0,152,151,153,154,155,156,157} ${ROUNDS:-5} > $O/ab_c5dev.log 2>&1 || { tail $O/ab_c5dev.log; exit 1; }
grep -h '"wl"\|false' $O/ab_c3r.log $O/ab_c5dev.log
