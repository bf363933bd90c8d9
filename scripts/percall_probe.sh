#!/bin/bash
# build scripts/percall_probe (host code + libozec; no kernels of its own)
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 scripts/percall_probe.cpp -Lozone_amd/lib -lozec \
  -Wl,-rpath,'$ORIGIN/../ozone_amd/lib' -o scripts/percall_probe
