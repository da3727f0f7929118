#!/bin/bash
# Round 5: 32-entry walk slots at 2e9 nodes (the slot rule now sizes by device
# memory): the config-5 line at full size, then the full-size bit-exact test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_cap
mkdir -p $out
timeout -k 10 600 python3 bench.py --config 5 --giant 2000000001 --steps 2 --warmup 1 --no-cpu --no-refresh > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['hbm_used_gib'], d['kernels_ms_per_step'])"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_giant_full.py > $out/pytest.log 2>&1 || { echo "test failed"; tail -20 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
