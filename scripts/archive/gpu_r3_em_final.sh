#!/bin/bash
# Round 3, after the lane-parallel emit (EM) became the fused default: the fused workloads' lines, the defaults A/B,
# rocprofv3 kernel stats with the bench's own warmup/steps and the SQ counter passes of the new defaults.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3emfin}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
for w in c3r c5dev; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
done
timeout -k 10 300 python bench.py --workload c3r --erased 1,4,10,13 > $O/bench_c3r_mixed.json 2> $O/bench_c3r_mixed.err || { echo "c3r mixed failed"; exit 1; }
echo lines ok
timeout -k 10 300 python -u scripts/ab.py c3r crc_variant 0,170,150,102,173 6 > $O/ab_c3r_defaults.log 2>&1 || { tail $O/ab_c3r_defaults.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py c5dev crc_variant 0,167,163,87,174 6 > $O/ab_c5dev_defaults.log 2>&1 || { tail $O/ab_c5dev_defaults.log; exit 1; }
grep -h '"wl"' $O/ab_c3r_defaults.log $O/ab_c5dev_defaults.log
export TMPDIR=/tmp
cd /tmp
for w in c3r c5dev; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --no-cpu --no-pmc --no-e2e > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail $O/prof_$w.log; exit 1; }
  echo "profiled $w"
done
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"
for wl in c3r c5dev; do
  for p in 1 2; do
    eval PM=\$P$p
    timeout -k 5 120 rocprofv3 --pmc $PM --kernel-trace -d $O/sq_${wl}_p$p -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-pmc --no-e2e > $O/sq_${wl}_p$p.log 2>&1 || { echo "pmc $wl $p failed"; tail -5 $O/sq_${wl}_p$p.log; exit 1; }
  done
done
echo final done
