#!/bin/bash
# Round 4: effective parents from the fused kernel's front end (CW_FRONT_EFF) -- parity, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_eff
mkdir -p $out
CW_FRONT_EFF=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
V='[{}, {"CW_FRONT_EFF":"1"}, {}, {"CW_FRONT_EFF":"1"}]'
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 10000 --nodes 50000 --rounds 4 --check > $out/sweep.txt 2> $out/sweep.err || { tail -5 $out/sweep.err; exit 1; }
cut -c1-200 $out/sweep.txt
