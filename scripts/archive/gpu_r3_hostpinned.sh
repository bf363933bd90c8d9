#!/bin/bash
# Round 3: per-call host encode from pinned caller cells (DMA in place) at 1 / 4 / 16 threads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/${OUT:-r3hostpinned}; mkdir -p $O
export PYTHONPATH=$R:$R/tests/golden
for t in 1 4 16; do
  timeout -k 10 300 python bench.py --workload host --host-pinned --threads $t --stripes 256 --no-cpu > $O/bench_host_pinned_t$t.json 2> $O/bench_host_pinned_t$t.err || { echo "T=$t failed"; tail $O/bench_host_pinned_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_host_pinned_t$t.json')); print('pinned T=$t', d['value'], d['pcie']['value_frac_of_duplex_h2d'])"
done
