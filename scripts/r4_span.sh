#!/bin/bash
# Round 4: walkers per walk block (the state-machine walk refills lanes inside a block).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_span
mkdir -p $out
V='[{}, {"CW_WALK_SPAN":"4096"}, {"CW_WALK_SPAN":"16384"}, {"CW_WALK_SPAN":"65536"}]'
timeout -k 10 400 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 67108864 --rounds 3 --check > $out/sweep26.txt 2> $out/sweep26.err || { tail -5 $out/sweep26.err; exit 1; }
cut -c1-200 $out/sweep26.txt
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 268435456 --rounds 2 --check > $out/sweep28.txt 2> $out/sweep28.err || { tail -5 $out/sweep28.err; exit 1; }
cut -c1-200 $out/sweep28.txt
