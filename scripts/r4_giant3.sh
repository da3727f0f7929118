#!/bin/bash
# Round 4: the walk as a per-lane state machine -- giant tests, then config 5 timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_giant3
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_parity.py tests/test_gpu_exact.py -k "giant or linked or ranked or walk or large_list" -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 400 python3 -u scripts/sweep.py '[{}]' --docs 1 --nodes 67108864 --rounds 3 > $out/sweep26.txt 2> $out/sweep26.err || { tail -5 $out/sweep26.err; exit 1; }
cut -c1-300 $out/sweep26.txt
timeout -k 10 600 python3 -u scripts/sweep.py '[{}]' --docs 1 --nodes 268435456 --rounds 2 > $out/sweep28.txt 2> $out/sweep28.err || { tail -5 $out/sweep28.err; exit 1; }
cut -c1-300 $out/sweep28.txt
timeout -k 10 400 python3 -u scripts/sweep.py '[{}]' --docs 10000 --nodes 50000 --rounds 3 > $out/sweepc2.txt 2> $out/sweepc2.err || { tail -5 $out/sweepc2.err; exit 1; }
cut -c1-300 $out/sweepc2.txt
