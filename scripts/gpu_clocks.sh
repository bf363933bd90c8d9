#!/bin/bash
# Shader clock and board power while each main kernel runs back to back (read-only rocm-smi samples every 0.5 s
# beside a long bench.py run), to put a measured clock under the "power-limited clock" reading of the SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r4clk}; mkdir -p $O
for spec in ${SPECS:-c2:2000 c5dev:2000 c3r:2400 crc:8000 c4:6000}; do
  w=${spec%%:*}; n=${spec#*:}
  timeout -k 10 240 python bench.py --workload $w --steps $n --warmup 20 --no-cpu --no-pmc --no-e2e --no-fused > $O/bench_$w.json 2> $O/bench_$w.err &
  pid=$!
  : > $O/smi_$w.log
  while kill -0 $pid 2> /dev/null; do
    { date +%s.%N; timeout -k 2 5 rocm-smi --showuse --showclocks --showpower --json 2> /dev/null; echo; } >> $O/smi_$w.log
    sleep 0.5
  done
  wait $pid || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  echo "sampled $w: $(grep -c '^[0-9]' $O/smi_$w.log) samples"
done
echo clocks done
