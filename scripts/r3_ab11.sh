#!/bin/bash
# Round 3: the giant join gathering cause | kind << 56 as one word (CW_GPACK):
# parity of the giant path, config 5 at 6.7e7 and 2e9 nodes with and without.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab11
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_giant.py tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "giant parity ok"; tail -1 $O/pytest.log
for rep in 1 2; do
  for g in 0 1; do
    CW_GPACK=$g timeout -k 10 300 python bench.py --config 5 --no-cpu > $O/c5_$g.$rep.json 2> $O/c5.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],3), k.get('join'), k.get('gpack'))" $O/c5_$g.$rep.json
  done
done
for g in 0 1; do
  CW_GPACK=$g timeout -k 10 600 python bench.py --config 5 --giant 2000000001 --steps 2 --warmup 1 --no-cpu > $O/c5full_$g.json 2> $O/c5full.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],3), k.get('join'), k.get('gpack'))" $O/c5full_$g.json
done
