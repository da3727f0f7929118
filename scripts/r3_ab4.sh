#!/bin/bash
# Round 3: u16 tree tables and links inside k_weave_doc (this build) vs the
# previous build (cause_amd/libcauseweave_base.so), and k_map_pack's id
# directory (CW_MAP_DIR) and four-window look-back (CW_MAP_LBW): parity, A/B.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_giant.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "parity ok"; tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_mirror.py -x -q --timeout 200 --timeout-method thread > $O/pytest_maps.log 2>&1
echo "maps ok"; tail -1 $O/pytest_maps.log
bash scripts/ab.sh cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so > $O/ab.log 2>&1
cat $O/ab.log
for rep in 1 2; do
  for v in "0 1" "1 1" "1 4" "0 4"; do
    set -- $v
    CW_MAP_DIR=$1 CW_MAP_LBW=$2 timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu > $O/c4_$1_$2.$rep.json 2> $O/c4.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4), d.get('kernel_sum_ms_per_step'))" $O/c4_$1_$2.$rep.json
  done
done
CW_MAP_DIR=1 CW_MAP_LBW=4 timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --check > $O/c4check.json 2> $O/c4check.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('check', d.get('check'))" $O/c4check.json
for v in "0 1" "1 4"; do
  set -- $v
  CW_TREE_PROF=1 CW_MAP_DIR=$1 CW_MAP_LBW=$2 timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $O/c4p.json 2> $O/c4p.err
  echo "dir=$1 lbw=$2"; grep 'map pack phases' $O/c4p.err | tail -1
done
