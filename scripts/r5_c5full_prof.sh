#!/bin/bash
# Round 5: rocprofv3 kernel-trace summary of the full config-5 bench line (2e9
# nodes) on the final build, beside the line's HIP-event kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
out=gpurun_out/r5_c5full_prof
mkdir -p $out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 1100 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof -o run -- python3 $R/bench.py --config 5 --giant 2000000001 --steps 2 --warmup 1 --no-cpu --no-refresh > $R/$out/bench.json 2> $R/$out/bench.err) || { echo "prof failed"; tail -5 $out/bench.err; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $out/kernel_stats.csv
head -6 $out/kernel_stats.csv | cut -c1-160
