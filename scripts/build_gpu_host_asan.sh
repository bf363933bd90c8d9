#!/bin/bash
# Build tests/native/bin/gpu_host_asan: the host-buffer C ABI paths driver linked against libozec's host objects
# built with ASan + UBSan (make asan-host) and the regular kernel objects.  The ASan runtime is linked into the
# executable (no preloading).  Run it on the GPU box with scripts/gpu_host_asan.sh.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$R/ozone_amd/csrc" ARCH=gfx950 all asan-host
mkdir -p "$R/tests/native/bin"
gcc -O1 -g -std=gnu11 -fPIC -c "$R/oracle/ozec_oracle.c" -o "$R/build/asan/oracle.o"
CXX=/opt/rocm/lib/llvm/bin/clang++
$CXX -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -c "$R/tests/native/gpu_host_asan.cpp" \
  -o "$R/build/asan/gpu_host_asan.o"
$CXX -fsanitize=address,undefined -o "$R/tests/native/bin/gpu_host_asan" "$R/build/asan/gpu_host_asan.o" \
  "$R"/build/asan/{gf256,crc_host,capi,stripe_queue,copy_pool,numa}.o "$R/build/obj/kernels.o" "$R"/build/obj/fused*.o \
  "$R/build/asan/oracle.o" -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib
echo built "$R/tests/native/bin/gpu_host_asan"
