#!/bin/bash
# Round 3: k_map_pack pack size with the round-3 map defaults: CW_MAP_PACK
# 0 = auto (512 nodes / 128 threads when every collection fits), 1 = 1024 /
# 256, 3 = 2048 / 512 (the round-2 default); parity and a checked run of auto.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab14
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_mirror.py tests/test_base.py -x -q --timeout 200 --timeout-method thread > $O/pytest_maps.log 2>&1
echo "maps (auto) ok"; tail -1 $O/pytest_maps.log
for rep in 1 2; do
  for m in 0 1 3; do
    CW_MAP_PACK=$m timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu > $O/c4_$m.$rep.json 2> $O/c4.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4), d.get('kernel_sum_ms_per_step'))" $O/c4_$m.$rep.json
  done
done
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --check > $O/c4check.json 2> $O/c4check.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('auto check', d.get('check'), round(d['value']/1e9,2))" $O/c4check.json
