#!/bin/bash
# Round 3: k_tree_l with direct list heads for in-tile parents (CW_TL_MODE=4)
# inside the fused weave: parity and A/B; config 4 with the final map defaults.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab7
mkdir -p $O
CW_TL_MODE=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "parity (TL_MODE 4) ok"; tail -1 $O/pytest.log
timeout -k 10 500 python -u scripts/sweep.py '[{},{"CW_TL_MODE":"4"}]' --rounds 3 --check > $O/sweep.log 2>&1
grep -i "variant\|identical\|differ" $O/sweep.log | head -20
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --check > $O/c4check.json 2> $O/c4check.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('config 4', round(d['ms_per_step'],4), round(d['value']/1e9,2), d.get('kernel_sum_ms_per_step'), d.get('check'))" $O/c4check.json
