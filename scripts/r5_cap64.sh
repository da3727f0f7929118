#!/bin/bash
# Round 5: 64-entry walk slots (CW_GIANT_LOG2CAP=6) against the default 32 on one
# giant list (GIANT nodes, input cached once), two alternations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_cap64
mkdir -p $out
G=${GIANT:-536870912}
B="python3 bench.py --config 5 --giant $G --cache /tmp/c5cache --steps 3 --warmup 1 --no-cpu --no-refresh"
for rep in 1 2; do
  for cap in 5 6; do
    CW_GIANT_LOG2CAP=$cap timeout -k 10 900 $B > $out/b$cap.json 2> $out/b$cap.err || { echo "bench failed"; tail -5 $out/b$cap.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b$cap.json')); k=d['kernels_ms_per_step']; print('cap', 1 << $cap, round(d['ms_per_step'], 2), {x: k[x] for x in ('walk', 'rank', 'emit')}, d['hbm_used_gib'])"
  done
done
