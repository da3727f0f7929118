#!/bin/bash
# Round 4: one-pass directory build, digit order, walk reverted -- tests, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_gdb
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_parity.py tests/test_gpu_exact.py -k "giant or linked or ranked or walk or large_list or continuation" -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
V='[{}, {"CW_GLOCAL":"0"}]'
timeout -k 10 400 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 67108864 --rounds 3 --check > $out/sweep26.txt 2> $out/sweep26.err || { tail -5 $out/sweep26.err; exit 1; }
cut -c1-300 $out/sweep26.txt
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 600000000 --rounds 2 --check > $out/sweep6e8.txt 2> $out/sweep6e8.err || { tail -5 $out/sweep6e8.err; exit 1; }
cut -c1-300 $out/sweep6e8.txt
