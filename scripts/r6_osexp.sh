#!/bin/bash
# onesweep pass timing experiments at 2e8 keys (wrong results): geometry 4
# (8 ranged chains): 0 full, 2 no look-back, 8 one look-back window, 4 no write-out
mkdir -p gpurun_out
for e in 0 2 8 4; do
  CW_OS_EXP=$e GEOMS=${CW_ONESWEEP:-4} timeout -k 10 120 python -u scripts/sort_bench.py 200000000 35 3 > gpurun_out/osexp_$e.log 2>&1 || exit 1
done
echo done
