#!/bin/bash
# Round 3: the giant path's launch knobs at config 5 (6.7e7 nodes): walk
# threads, splitter block (CW_LOG2K), slot capacity (CW_LOG2CAP), radix digit.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab15
mkdir -p $O
for v in "X=0" "CW_WALK_THREADS=256" "CW_WALK_THREADS=1024" "CW_LOG2K=4" "CW_LOG2CAP=6" "CW_MAX_DIGIT=10" "X=1"; do
  env $v timeout -k 10 300 python bench.py --config 5 --no-cpu > $O/c5.json 2> $O/c5.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], round(d['ms_per_step'],3), {a: round(b,2) for a, b in sorted(k.items(), key=lambda x: -x[1])[:6]})" $O/c5.json "$v"
done
