#!/bin/bash
# Round-4 final, part A: smoke, PMC traffic (FETCH/WRITE) for configs 2, 4, 5
# (build-tagged, accumulated in gpurun_out/pmc_traffic.json) and one SQ pass each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
out=gpurun_out/r4_final
rm -rf $out
mkdir -p $out
timeout -k 10 300 python -u __graft_entry__.py smoke > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
echo "smoke ok"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
for cfg in 2 4 5; do
  d=$out/pmc_c$cfg
  mkdir -p $d
  for pass in FETCH_SIZE WRITE_SIZE "$SQ"; do
    t=$(echo $pass | tr ' ' '_' | cut -c1-40)
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $pass \
       --output-format csv -d "$R/$d/pmc_$t" -o run -- \
       python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu --no-h2d --no-refresh --config $cfg > "$R/$d/pmc_$t.log" 2>&1) \
       || { echo "config $cfg pass $pass failed"; tail -5 "$R/$d/pmc_$t.log"; exit 1; }
    echo "config $cfg pass $t ok"
  done
  python3 scripts/pmc_summary.py $d > $d/pmc_table.txt || exit 1
  python3 scripts/pmc_traffic.py $d $out/pmc_traffic.json --workload config$cfg >> $out/pmc_traffic.txt || exit 1
  rm -rf $d/pmc_*/
done
cat $out/pmc_traffic.txt | head -60
echo "part A ok"
