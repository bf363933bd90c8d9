#!/bin/bash
# Run the host-buffer C ABI paths on the GPU with libozec's host code under ASan + UBSan (host instrumentation only;
# built here by scripts/build_gpu_host_asan.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/asan; mkdir -p $O
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:log_path=$O/asan UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1:log_path=$O/ubsan \
  timeout -k 10 300 tests/native/bin/gpu_host_asan > $O/run.log 2>&1
rc=$?
cat $O/run.log | grep -v amdgpu.ids
ls $O/asan* $O/ubsan* 2>/dev/null && head -60 $O/asan* $O/ubsan* 2>/dev/null
exit $rc
