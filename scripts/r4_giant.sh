#!/bin/bash
# Round 4: giant-path changes -- its tests, then config 5 timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_giant
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_giant.py tests/test_gpu_exact.py -k "giant or linked or ranked or large_list" -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 3 --no-h2d --no-cpu > $out/c5.json 2> $out/c5.err || { tail -5 $out/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c5.json')); print(d['ms_per_step']); print(d['kernels_ms_per_step'])"
timeout -k 10 300 python3 bench.py --config 1 --steps 20 --warmup 3 --no-h2d --no-cpu > $out/c1.json 2> $out/c1.err || { tail -5 $out/c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c1.json')); print('config1', d['ms_per_step'])"
CW_TREE_PROF=1 timeout -k 10 300 python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $out/c4prof.json 2> $out/c4prof.err || { tail -5 $out/c4prof.err; exit 1; }
grep "map pack phases" $out/c4prof.err | tail -2
