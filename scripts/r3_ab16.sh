#!/bin/bash
# Round 3: splitter block size of the giant path (CW_LOG2K) at 6.7e7 and 2.7e8 nodes.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab16
mkdir -p $O
run() {
  local g=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config 5 --giant $g --no-cpu --check > $O/c5.json 2> $O/c5.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], round(d['ms_per_step'],3), d.get('check'), {a: round(b,2) for a, b in sorted(k.items(), key=lambda x: -x[1])[:7]})" $O/c5.json "$g $*"
}
for v in "X=0" "CW_LOG2K=4" "CW_LOG2K=5" "CW_LOG2K=4 CW_LOG2CAP=6" "CW_LOG2K=5 CW_LOG2CAP=6"; do run 67108864 $v; done
for v in "X=0" "CW_LOG2K=4" "CW_LOG2K=5"; do run 268435456 $v; done
