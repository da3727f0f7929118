#!/bin/bash
# config 5 through the distributed entry on one rank: the tree on rank 0
# (cw_weave_ranked) vs rank by rank (dist.hip + cw_weave_linked)
set -e
O=gpurun_out/c5d
mkdir -p $O
G=${GIANT:-67108864}
for t in root dist; do
  timeout -k 10 600 python -u bench.py --config 5 --dist --tree $t --giant $G --no-cpu --steps 3 --warmup 1 \
    > $O/$t.json 2> $O/$t.err
done
