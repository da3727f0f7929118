#!/bin/bash
# Round 4: walk block geometry at 2e9 nodes (one generation, variants in one process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_walk2e9
mkdir -p $out
V='[{}, {"CW_WALK_THREADS":"256", "CW_WALK_SPAN":"256"}, {"CW_WALK_THREADS":"1024", "CW_WALK_SPAN":"1024"}, {"CW_WALK_SPAN":"2048"}]'
timeout -k 10 1100 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 2000000000 --rounds 2 > $out/sweep.txt 2> $out/sweep.err || { tail -5 $out/sweep.err; exit 1; }
cut -c1-260 $out/sweep.txt
