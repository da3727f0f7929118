#!/bin/bash
# Round 4: the map pack -- its tests, config 4 bench and phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_maps
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_mirror.py tests/test_base.py -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu --check > $out/c4.json 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c4.json')); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms_per_step'], d['check'])"
CW_TREE_PROF=1 timeout -k 10 300 python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $out/c4prof.json 2> $out/c4prof.err || { tail -5 $out/c4prof.err; exit 1; }
grep "map pack phases" $out/c4prof.err | tail -1
