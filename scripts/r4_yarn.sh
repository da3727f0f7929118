#!/bin/bash
# Round 4: yarn ids from the front end's directory -- parity tests, then the config-2 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_yarn
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_stream.py tests/test_gpu_mirror.py tests/test_gpu_merge.py -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-h2d --no-cpu > $out/c2.json 2> $out/c2.err || { tail -5 $out/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c2.json')); print(d['ms_per_step'], d['kernels_ms_per_step']); r=d.get('refresh_caches') or {}; print('refresh', r.get('ms_per_step'), r.get('kernels_ms_per_step'))"
