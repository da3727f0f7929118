#!/bin/bash
# Round 5 (timing only, outputs not checked): what bounds k_yarn_doc -- its id
# and rank reads (1), its input-index reads (2), its yarn writes (4) switched off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_e
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep.py '[{}, {"CW_YARN_EXP":"64"}, {"CW_YARN_EXP":"7"}, {"CW_YARN_EXP":"8"}, {"CW_YARN_EXP":"72"}, {"CW_YARN_EXP":"39"}, {"CW_YARN_EXP":"23"}]' --rounds 3 --yarns > $out/y.txt 2> $out/y.err || { tail -5 $out/y.err; exit 1; }
cut -c1-200 $out/y.txt
