#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes (separate runs) of one workload's bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/traffic
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
W=${W:-c5}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 10 --warmup 3 --no-cpu > $O/prof_$W.log 2>&1 || { echo "rocprof failed"; tail $O/prof_$W.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --stats -d $O/pmc_${W}_$ctr -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu > $O/pmc_${W}_$ctr.log 2>&1 || { echo "pmc $ctr failed"; exit 1; }
done
tail -1 $O/prof_$W.log
echo traffic done
