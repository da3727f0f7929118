#!/bin/bash
# Round 4: the fused tour with sublist slots (CW_TOUR_SLOTS) -- parity, then A/B on config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_tslots
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
V='[{}, {"CW_TOUR_SLOTS":"0"}, {}, {"CW_TOUR_SLOTS":"0"}]'
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 10000 --nodes 50000 --rounds 4 --check > $out/sweep.txt 2> $out/sweep.err || { tail -5 $out/sweep.err; exit 1; }
cut -c1-200 $out/sweep.txt
CW_TREE_PROF=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-h2d --no-cpu --no-refresh > $out/prof.json 2> $out/prof.err || { tail -5 $out/prof.err; exit 1; }
grep phases $out/prof.err | tail -2
