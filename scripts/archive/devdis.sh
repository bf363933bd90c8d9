#!/bin/bash
# Device-only compile of one HIP source for gfx950 and its disassembly (kernel ISA study): devdis.sh src.hip out.dis [extra flags]
set -e
src=$1; out=$2; shift 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c -o /tmp/devdis.co "$src" "$@"
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn /tmp/devdis.co > "$out"
