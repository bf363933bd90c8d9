#!/bin/bash
# Round 4 GPU evidence: GPU parity suite + smoke, then the default bench line (C2 headline + fused legs + C5 e2e +
# PMC passes + CPU baseline), then any extra bench workloads in $EXTRA.  Every GPU step under its own time limit,
# chained so that the first failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${OUT:-r4}; mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
  python - $O/bench_default.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rf = d["roofline"]
print("C2", d["value"], rf["frac"], rf.get("frac_rocprof_avg"), rf.get("traffic"))
for l in d.get("fused", []):
    print("fused", l.get("workload", l)[:60], l.get("kernel_ms"), l.get("frac"), l.get("frac_rocprof_avg"), l.get("pmc", {}).get("traffic_over_algorithmic"), l.get("verified"))
e = d.get("e2e", {})
print("e2e", e.get("value"), e.get("error"))
PY
fi
# interleaved same-process A/Bs: AB="c3r:0,170,191 c5dev:0,171,189" (ROUNDS each)
for spec in $AB; do
  w=${spec%%:*}; v=${spec#*:}
  timeout -k 10 300 python -u scripts/ab.py $w crc_variant $v ${ROUNDS:-5} > $O/ab_$w.log 2>&1 || { tail -20 $O/ab_$w.log; exit 1; }
  grep median_ms $O/ab_$w.log
done
for w in $EXTRA; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['roofline']['frac'], d['roofline'].get('frac_rocprof_avg'), d['roofline'].get('traffic'))"
done
