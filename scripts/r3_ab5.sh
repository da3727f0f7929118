#!/bin/bash
# Round 3: k_map_pack -- early element loads (this build vs the previous,
# cause_amd/libcauseweave_base.so), relaxed look-back atomics (CW_MAP_RELAXED),
# the id directory as the cause join (CW_MAP_DIRJOIN); parity of the variants.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab5
mkdir -p $O
CW_MAP_RELAXED=1 CW_MAP_DIRJOIN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_mirror.py -x -q --timeout 200 --timeout-method thread > $O/pytest_maps.log 2>&1
echo "maps ok (relaxed + dirjoin)"; tail -1 $O/pytest_maps.log
for rep in 1 2; do
  for v in "base 0 0" "new 0 0" "new 1 0" "new 0 1" "new 1 1"; do
    set -- $v
    lib=$PWD/cause_amd/libcauseweave.so; [ $1 = base ] && lib=$PWD/cause_amd/libcauseweave_base.so
    CW_LIB=$lib CW_MAP_RELAXED=$2 CW_MAP_DIRJOIN=$3 timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu > $O/c4_$1_$2_$3.$rep.json 2> $O/c4.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4), d.get('kernel_sum_ms_per_step'))" $O/c4_$1_$2_$3.$rep.json
  done
done
CW_MAP_RELAXED=1 CW_MAP_DIRJOIN=1 timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --check > $O/c4check.json 2> $O/c4check.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('check', d.get('check'))" $O/c4check.json
for v in "0 0" "1 1"; do
  set -- $v
  CW_TREE_PROF=1 CW_MAP_RELAXED=$1 CW_MAP_DIRJOIN=$2 timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4p.json 2> $O/c4p.err
  echo "relaxed=$1 dirjoin=$2"; grep 'map pack phases' $O/c4p.err | tail -1
done
