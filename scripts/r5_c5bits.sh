#!/bin/bash
# Round 5: the giant path sorting by the ids' real width (33 of the declared 35
# bits at 2e9 nodes): this build against LIB_BASE on the full config-5 list
# (input generated once, cached), two alternations, then the full-size
# bit-exact test on this build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_c5bits
mkdir -p $out
B="python3 bench.py --config 5 --giant 2000000001 --cache /tmp/c5cache --steps 2 --warmup 1 --no-cpu --no-refresh"
for rep in 1 2; do
  for lib in cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so; do
    CW_LIB="$PWD/$lib" timeout -k 10 900 $B > $out/b.json 2> $out/b.err || { echo "bench failed"; tail -5 $out/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b.json')); k=d['kernels_ms_per_step']; print('$lib', round(d['ms_per_step'], 2), {x: k.get(x) for x in ('idsort_scatter', 'idsort_hist', 'idsort_scan', 'index', 'join', 'or_reduce')})"
    cp $out/b.json $out/$(basename $lib .so)_$rep.json
  done
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_giant_full.py > $out/pytest.log 2>&1 || { echo "test failed"; tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
