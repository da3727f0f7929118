#!/bin/bash
# Round 4: phase clocks of the config-2 weave, fused and separate kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_wprof
mkdir -p $out
CW_TREE_PROF=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-h2d --no-cpu > $out/fused.json 2> $out/fused.err || { tail -5 $out/fused.err; exit 1; }
grep phases $out/fused.err | tail -3
true


