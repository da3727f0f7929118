#!/bin/bash
# Round 3: the fused kernel's front-end loads in flight (CW_FRONT_U: 0 = 4/4/4
# items a thread in the directory/rank/input-index passes, 1 = 16/4/16,
# 2 = 32/4/32, 3 = 8/4/8): parity of the deepest, A/B of all.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab8
mkdir -p $O
CW_FRONT_U=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bench_batch or golden or edge or config" > $O/pytest.log 2>&1
echo "parity (FRONT_U 2) ok"; tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/sweep.py '[{},{"CW_FRONT_U":"1"},{"CW_FRONT_U":"2"},{"CW_FRONT_U":"3"}]' --rounds 3 --check > $O/sweep.log 2>&1
grep -i "variant\|identical\|differ" $O/sweep.log | head -20
