#!/bin/bash
# Round 3, last call: the host-memory reconstruction, stripe queue and C4 lines on the final build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=r3last PHASE=b WORKLOADS="c3r_host queue c4" bash scripts/gpu_final_r3.sh
