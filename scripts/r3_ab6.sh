#!/bin/bash
# Round 3: k_map_pack defaults (id directory, relaxed look-back, directory
# join) with and without early element loads; the fused weave's phase clocks.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_mirror.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread -k "not full_size_line" > $O/pytest_maps.log 2>&1
echo "maps ok"; tail -1 $O/pytest_maps.log
for rep in 1 2; do
  for e in 0 1; do
    CW_MAP_EARLY=$e timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu > $O/c4_$e.$rep.json 2> $O/c4.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4), d.get('kernel_sum_ms_per_step'))" $O/c4_$e.$rep.json
  done
done
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --check > $O/c4check.json 2> $O/c4check.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('check', d.get('check'), d['value']/1e9)" $O/c4check.json
CW_TREE_PROF=1 timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4p.json 2> $O/c4p.err
grep 'map pack phases' $O/c4p.err | tail -1
timeout -k 10 300 python -u scripts/sweep.py '[{"CW_TREE_PROF":"1"},{"CW_TREE_PROF":"1","CW_FUSED":"0"}]' --rounds 1 > $O/sweep_prof.log 2>&1
grep "phases" $O/sweep_prof.log | head -12
