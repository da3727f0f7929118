#!/bin/bash
# Round 4: config 5 at full size -- the bit-exact test, then the 2e9-node bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_c5full
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_giant_full.py -x -v --timeout 560 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 1000 python3 -u bench.py --config 5 --giant 2000000000 --steps 2 --warmup 1 --no-h2d --no-cpu \
  > $out/c5full.json 2> $out/c5full.err || { tail -5 $out/c5full.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c5full.json')); print(d['ms_per_step']); print(d['kernels_ms_per_step'])"
