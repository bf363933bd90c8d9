#!/bin/bash
# Round 3: instruction-cache counters of the XO defaults against the wide step-group variants (is the unrolled
# loop's size what makes D = 2 (rs-10-4) / D = 4 (rs-6-3) slower?)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
SPECS="c3r:150 c3r:163 c5dev:167 c5dev:160" PASSES="2" bash scripts/gpu_r3_ifetch.sh
