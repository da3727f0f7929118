#!/bin/bash
# Round 4: k_gsib galloping search; radix digit width A/B on the giant path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_giant2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_parity.py -k "giant or linked or ranked" -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
V='[{}, {"CW_MAX_DIGIT":"8"}, {"CW_MAX_DIGIT":"10"}]'
timeout -k 10 400 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 67108864 --rounds 3 --check > $out/sweep26.txt 2> $out/sweep26.err || { tail -5 $out/sweep26.err; exit 1; }
cat $out/sweep26.txt | cut -c1-400
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 1 --nodes 268435456 --rounds 2 --check > $out/sweep28.txt 2> $out/sweep28.err || { tail -5 $out/sweep28.err; exit 1; }
cat $out/sweep28.txt | cut -c1-400
