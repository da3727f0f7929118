#!/bin/bash
# Counters of the giant path (config 5 at 6.7e7 nodes): FETCH_SIZE and
# WRITE_SIZE (HBM bytes per launch, gfx950 FETCH x2), SQ wave states and the
# L2 hit/miss / EA requests, each pass its own run; then the kernel-trace stats.
#   bash scripts/r4_pmc.sh <tag> [bench args, default --config 5]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
tag=${1:-r04}
shift
args="${*:---config 5}"
out=gpurun_out/pmc_$tag
mkdir -p $out
passes=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
for pass in "${passes[@]}"; do
  t=$(echo $pass | tr ' ' '_' | cut -c1-40)
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass \
     --output-format csv -d "$R/$out/pmc_$t" -o run -- \
     python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu --no-h2d $args > "$R/$out/pmc_$t.log" 2>&1) \
     || { echo "pass $pass failed"; tail -5 "$R/$out/pmc_$t.log"; exit 1; }
  echo "pass $pass ok"
done
python3 scripts/pmc_summary.py $out > $out/pmc_table.txt && cat $out/pmc_table.txt | cut -c1-200
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/$out/stats" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-h2d $args \
   > "$R/$out/bench_prof.log" 2>&1) || { echo "stats run failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-h2d $args > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); print(d['kernels_ms_per_step'])"
