#!/bin/bash
# Round-end measurement, config 5 (after gpu_final.sh on the same build, with its
# profiles/pmc_traffic.json copied back), in two calls:
#   bash scripts/gpu_final_c5.sh scaled   PMC FETCH/WRITE at the scaled default
#                                         (2^26 nodes), the config-5 and config-1 lines
#   bash scripts/gpu_final_c5.sh full     the same at BASELINE's 2,000,000,001 nodes
#                                         (input generated once into /tmp/c5cache)
# Each extends gpurun_out/pmc_traffic.json (and profiles/ on the box) with its workload.
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
O=gpurun_out/c5
mkdir -p $O
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
pmc() {  # $1 = dir, $2 = seconds, rest = bench args
  local dir=$1 lim=$2; shift 2
  mkdir -p "$R/$dir"
  for pass in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 $lim rocprofv3 --kernel-trace --pmc $pass \
      --output-format csv -d "$R/$dir/pmc_$pass" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu --no-refresh --check-docs 0 "$@" > "$R/$dir/pmc_$pass.log" 2>&1)
    echo "pmc $dir $pass ok"
  done
}
case "$1" in
  scaled)
    pmc $O/pmc26 300 --config 5
    python scripts/pmc_summary.py $O/pmc26 > $O/pmc_table_config5.txt
    python scripts/pmc_traffic.py $O/pmc26 gpurun_out/pmc_traffic.json --workload config5
    rm -rf $O/pmc26/pmc_*
    cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json  # (the lines below read it)
    timeout -k 10 300 python bench.py --config 5 > $O/c5.json 2> $O/c5.err
    timeout -k 10 300 python bench.py --config 1 > $O/c1.json 2> $O/c1.err
    echo "scaled ok" ;;
  full)
    pmc $O/pmcfull 900 --config 5 --giant 2000000001 --cache /tmp/c5cache
    python scripts/pmc_summary.py $O/pmcfull > $O/pmc_table_config5full.txt
    python scripts/pmc_traffic.py $O/pmcfull gpurun_out/pmc_traffic.json --workload config5full
    rm -rf $O/pmcfull/pmc_*
    cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json  # (the lines below read it)
    timeout -k 10 600 python bench.py --config 5 --giant 2000000001 --cache /tmp/c5cache --steps 2 --warmup 1 > $O/c5full.json 2> $O/c5full.err
    timeout -k 10 300 python bench.py --config 5 > $O/c5.json 2> $O/c5.err
    echo "full ok" ;;
  *) echo "usage: $0 scaled|full"; exit 2 ;;
esac
