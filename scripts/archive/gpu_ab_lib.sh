#!/bin/bash
# Interleaved A/B of two builds of libozec.so (ozone_amd/lib/libozec_a.so vs libozec_b.so): GPU parity suite on B,
# then bench lines of each workload for A, B, A, B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/ablib
mkdir -p $O
L=ozone_amd/lib
cp $L/libozec_b.so $L/libozec.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_b.log 2>&1 || { tail -30 $O/pytest_gpu_b.log; exit 1; }
tail -1 $O/pytest_gpu_b.log
for r in 1 2; do
  for v in a b; do
    cp $L/libozec_$v.so $L/libozec.so
    for w in ${WORKLOADS:-c5 c3r crc}; do
      timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail $O/${w}_${v}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" $O/${w}_${v}_$r.json $w $v $r
    done
  done
done
