#!/bin/bash
# Round 4: the 2.7e8-node config-5 variants of r3_ab16.sh, each
# with --check (the oracle check under bench.py's heartbeat), to completion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r4_ab16
mkdir -p $O
run() {
  local g=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config 5 --giant $g --no-cpu --no-refresh --steps 3 --warmup 1 --check > $O/c5_$g.json 2> $O/c5_$g.err || { echo "run $g $* failed"; tail -5 $O/c5_$g.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels_ms_per_step',{}); print(sys.argv[2], round(d['ms_per_step'],3), d.get('check'), {a: round(b,2) for a, b in sorted(k.items(), key=lambda x: -x[1])[:6]})" $O/c5_$g.json "$g $*" | tee -a $O/summary.txt
}
for v in "X=0" "CW_GIANT_LOG2K=3" "CW_GIANT_LOG2K=5"; do run 268435456 $v || exit 1; done
