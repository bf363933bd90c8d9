#!/bin/bash
# PMC passes (separate runs, --kernel-trace/--stats only, as MI355X_MICROARCH.md's rocprofv3 section asks).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
for w in ${WORKLOADS:-c2 c5}; do
  for ctr in FETCH_SIZE WRITE_SIZE "$SQSET"; do
    [ -z "$ctr" ] && continue
    tag=$(echo $ctr | tr ' ' '_' | cut -c1-40)
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --stats -d $O/${w}_$tag -o run --output-format csv -- \
      python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu > $O/${w}_$tag.log 2>&1 || { echo "pmc $w $ctr failed"; tail $O/${w}_$tag.log; exit 1; }
  done
done
echo pmc done
