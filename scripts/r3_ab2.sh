#!/bin/bash
# Round 3: the fused per-document weave (k_weave_doc, the default) vs the three
# kernels (CW_FUSED=0): parity of both, then an A/B in one process.
#   bash scripts/r3_ab2.sh -> gpurun_out/ab2/
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "parity ok"
timeout -k 10 500 python -u scripts/sweep.py '[{"CW_FUSED":"0"},{"CW_FUSED":"1"}]' --rounds 3 --check > $O/sweep.log 2>&1
grep -i "variant\|identical\|differ" $O/sweep.log | head -20
