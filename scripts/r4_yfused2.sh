#!/bin/bash
# Round 4: yarns inside the fused kernel -- yarn parity, headline A/B against the measured build's code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_yfused2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_stream.py tests/test_gpu_mirror.py tests/test_gpu_merge.py tests/test_gpu_exact.py tests/test_gpu_k32.py -x -q --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
V='[{}, {"CW_YARN_FUSED":"0"}, {}, {"CW_YARN_FUSED":"0"}]'
timeout -k 10 600 python3 -u scripts/sweep.py "$V" --docs 10000 --nodes 50000 --rounds 4 --check > $out/sweep.txt 2> $out/sweep.err || { tail -5 $out/sweep.err; exit 1; }
cut -c1-160 $out/sweep.txt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-h2d --no-cpu > $out/c2.json 2> $out/c2.err || { tail -5 $out/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c2.json')); print(d['ms_per_step'], d['kernels_ms_per_step']); r=d.get('refresh_caches') or {}; print('refresh', r.get('ms_per_step'), r.get('kernels_ms_per_step'))"
