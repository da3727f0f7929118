#!/bin/bash
# Round 5: HBM bytes per phase of the config-2 weave -- the separate kernels
# (CW_FUSED=0: k_front, k_tree_l, k_tour) under FETCH_SIZE / WRITE_SIZE passes,
# and the fused kernel beside them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
out=gpurun_out/r5_sep_pmc
rm -rf $out; mkdir -p $out
B="python3 $R/bench.py --config 2 --steps 1 --warmup 0 --no-cpu --no-refresh"
for pass in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && CW_FUSED=0 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $R/$out/sep/pmc_$pass -o run -- $B > $R/$out/sep_$pass.log 2>&1) || { echo "sep $pass failed"; exit 1; }
  (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $R/$out/fused/pmc_$pass -o run -- $B > $R/$out/fused_$pass.log 2>&1) || { echo "fused $pass failed"; exit 1; }
  echo "pmc $pass ok"
done
python3 scripts/pmc_summary.py $out/sep > $out/sep_table.txt 2>&1 || true
python3 scripts/pmc_summary.py $out/fused > $out/fused_table.txt 2>&1 || true
cat $out/sep_table.txt $out/fused_table.txt
