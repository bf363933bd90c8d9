#!/bin/bash
# build the round-6 host-path probes (host code + libozec; no kernels of their own): percall_probe, pipeline_probe,
# d2h_probe, stream_engine_probe
set -e
cd "$(dirname "$0")/.."
for p in percall_probe pipeline_probe d2h_probe stream_engine_probe; do
  /opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 scripts/$p.cpp -Lozone_amd/lib -lozec \
    -Wl,-rpath,'$ORIGIN/../ozone_amd/lib' -o scripts/$p
done
