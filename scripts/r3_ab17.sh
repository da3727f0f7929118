#!/bin/bash
# Round 3: radix histogram with all of a thread's key loads issued first, A/B at config 5 (6.7e7 nodes).
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab17
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "giant" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so; do
    CW_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --config 5 --no-cpu > $O/c5.json 2> $O/c5.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], round(d['ms_per_step'],3), {a: round(b,3) for a, b in k.items() if 'hist' in a or 'scan' in a})" $O/c5.json "$lib"
  done
done
