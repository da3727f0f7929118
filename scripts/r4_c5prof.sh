#!/bin/bash
# Round 4: the walk at 2e9 nodes -- chase calibration up to 64 GiB, then the
# config-5 list with the walk's step/chase counters (CW_TREE_PROF).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_c5prof
mkdir -p $out
timeout -k 10 200 ./scripts/calib_chase > $out/chase.txt || exit 1
tail -4 $out/chase.txt
CW_TREE_PROF=1 timeout -k 10 1000 python3 -u bench.py --config 5 --giant 2000000000 --steps 1 --warmup 1 --no-h2d --no-cpu \
  > $out/c5full.json 2> $out/c5full.err || { tail -5 $out/c5full.err; exit 1; }
grep "walk profile" $out/c5full.err | tail -1
python3 -c "import json; d=json.load(open('$out/c5full.json')); print(d['ms_per_step']); print(d['kernels_ms_per_step'])"
