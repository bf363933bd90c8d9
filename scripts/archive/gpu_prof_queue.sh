#!/bin/bash
# Kernel + memory-copy trace of the stripe-queue bench (no PMC counters in this run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_queue -o run --output-format csv -- python3 $R/bench.py --workload ${W:-queue} --steps 3 --warmup 1 --no-cpu > $O/prof_queue.log 2>&1 || { echo "rocprof failed"; tail $O/prof_queue.log; exit 1; }
tail -2 $O/prof_queue.log
find $O/prof_queue -name "*.csv" | head
