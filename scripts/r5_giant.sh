#!/bin/bash
# Round 5: why the giant path's walk slows down per node with size (VERDICT r4
# next #4).  Config 5 at 2^29 nodes (input generated once, cached for the
# profiler passes): the bench line, the kernel trace, and PMC passes for the
# HBM bytes (FETCH_SIZE, WRITE_SIZE), L2 hits and misses, and the address
# translation counters the box lists ($XLAT, one pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
out=gpurun_out/r5_giant
mkdir -p $out
G=${GIANT:-536870912}
B="python3 $R/bench.py --config 5 --giant $G --cache /tmp/c5cache --steps 2 --warmup 1 --no-cpu --no-refresh"
timeout -k 10 600 $B > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['kernels_ms_per_step'])"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof -o run -- $B > $R/$out/prof.log 2>&1) || { echo "prof failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${XLAT:+"$XLAT"}; do
  tag=$(echo $pass | tr ' ' '_')
  (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $R/$out/pmc_$tag -o run -- $B > $R/$out/pmc_$tag.log 2>&1) || { echo "pmc $pass failed"; exit 1; }
  echo "pmc $pass ok"
done
python3 scripts/pmc_summary.py $out > $out/pmc_table.txt 2>&1 || true
head -40 $out/pmc_table.txt
