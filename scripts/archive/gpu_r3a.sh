set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/r3a; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant 62,0,130,131,133,135,140,141,142,143 4 > $O/ab_c3r.log 2>&1 || { tail $O/ab_c3r.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant 0,100,132,134,144,145,146,147 4 > $O/ab_c5dev.log 2>&1 || { tail $O/ab_c5dev.log; exit 1; }
grep '"wl"' $O/ab_c3r.log $O/ab_c5dev.log
