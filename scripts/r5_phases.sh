#!/bin/bash
# Round 5: phase clocks of the config-2 weave (CW_TREE_PROF): the fused
# kernel's front/tree/tour per document, and the separate kernels' sub-phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_phases
mkdir -p $out
B="python3 bench.py --config 2 --steps 1 --warmup 1 --no-cpu --no-refresh"
CW_TREE_PROF=1 timeout -k 10 300 $B > $out/fused.json 2> $out/fused.err || { echo "fused failed"; tail -5 $out/fused.err; exit 1; }
CW_FUSED=0 CW_TREE_PROF=1 timeout -k 10 300 $B > $out/sep.json 2> $out/sep.err || { echo "sep failed"; tail -5 $out/sep.err; exit 1; }
grep -h "phases" $out/fused.err $out/sep.err | sort | uniq -c | head -20
