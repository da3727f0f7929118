#!/bin/bash
# Round 5: where the in-kernel yarns' 3.7 ms go (timing only): the yarn-fused
# kernel with its yarn work skipped (CW_YARN_SKIP, outputs not checked), with
# yarns, and without yarns asked for.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_b
mkdir -p $out
timeout -k 10 400 python -u scripts/sweep.py '[{}, {"CW_YARN_SKIP":"1"}]' --rounds 3 --yarns > $out/yskip.txt 2> $out/yskip.err || { tail -5 $out/yskip.err; exit 1; }
cut -c1-200 $out/yskip.txt
timeout -k 10 400 python -u scripts/sweep.py '[{}]' --rounds 3 > $out/noyarn.txt 2> $out/noyarn.err || { tail -5 $out/noyarn.err; exit 1; }
cut -c1-200 $out/noyarn.txt
