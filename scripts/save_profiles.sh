#!/bin/bash
# Copy a gpu_measure.sh run's summaries from gpurun_out/ into profiles/ (tracked):
#   bash scripts/save_profiles.sh r03_v1
set -e
tag="$1"; [ -n "$tag" ] || { echo "usage: $0 TAG"; exit 2; }
O=gpurun_out
[ -f $O/bench.log ] && grep '^{' $O/bench.log | tail -1 > profiles/${tag}_bench.json
ks=$(find $O/prof -name '*kernel_stats.csv' | head -1)
[ -n "$ks" ] && cp "$ks" profiles/${tag}_kernel_stats.csv
[ -f $O/pmc_table.txt ] && cp $O/pmc_table.txt profiles/${tag}_pmc_table.txt
[ -f $O/pmc_table_config4.txt ] && cp $O/pmc_table_config4.txt profiles/${tag}_pmc_table_config4.txt
[ -f $O/pmc_sq_table.txt ] && cp $O/pmc_sq_table.txt profiles/${tag}_pmc_sq_table.txt
[ -f $O/pytest_gpu.log ] && tail -3 $O/pytest_gpu.log > profiles/${tag}_pytest_gpu.log
[ -f $O/pmc_traffic.json ] && cp $O/pmc_traffic.json profiles/pmc_traffic.json
ls profiles/${tag}_*
