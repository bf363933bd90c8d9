#!/bin/bash
# Round 3: staging copies with streaming stores (copy_stream 0 memcpy / 1 both ways / 2 into staging only),
# same-process A/Bs of the per-call host encode at 1 and 16 threads and of the pageable stripe queue.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3copy}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
STRIPES=128 THREADS=1 timeout -k 10 300 python -u scripts/ab.py host copy_stream -1,0,1 ${ROUNDS:-5} > $O/ab_host_t1.log 2>&1 || { tail $O/ab_host_t1.log; exit 1; }
STRIPES=256 THREADS=16 timeout -k 10 300 python -u scripts/ab.py host copy_stream -1,0,1 ${ROUNDS:-5} > $O/ab_host_t16.log 2>&1 || { tail $O/ab_host_t16.log; exit 1; }
timeout -k 10 300 python -u scripts/ab.py queue_pageable copy_stream -1,0,1 ${ROUNDS:-5} > $O/ab_queue_pageable.log 2>&1 || { tail $O/ab_queue_pageable.log; exit 1; }
grep -h '"wl"' $O/ab_*.log
