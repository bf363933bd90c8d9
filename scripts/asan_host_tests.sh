#!/bin/bash
# Host tests of the C ABI against the ASan + UBSan build of libozec (make -C ozone_amd/csrc asan-host).
R=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:log_path=${ASAN_LOG:-/tmp/ozec_asan} \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1:log_path=${ASAN_LOG:-/tmp/ozec_asan} \
OZEC_LIB_OVERRIDE=$R/build/asan/libozec.so exec python -m pytest "$R"/tests/test_host_abi.py "$R"/tests/test_jni_marshal.py \
  "$R"/tests/test_stripe_queue.py "$R"/tests/test_composite_crc.py "$R"/tests/test_rawcoder_api.py "$R"/tests/test_host_api.py \
  "$R"/tests/test_jni_glue.py -m "not gpu" -q -p no:cacheprovider "$@"
