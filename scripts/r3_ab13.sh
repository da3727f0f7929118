#!/bin/bash
# Round 3: the small fused-kernel choices re-checked with more interleaved
# rounds (the run-to-run spread is 0.1-0.2 ms): direct list heads (CW_TL_MODE
# 4 vs 0) and 16 front-end ids in flight (CW_FRONT_U 1 vs 0).
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab13
mkdir -p $O
timeout -k 10 900 python -u scripts/sweep.py '[{},{"CW_TL_MODE":"0"},{"CW_FRONT_U":"0"},{"CW_TL_MODE":"0","CW_FRONT_U":"0"}]' --rounds 6 --check > $O/sweep.log 2>&1
grep -i "variant\|identical\|differ" $O/sweep.log | head -20
