#!/bin/bash
# Round measurement on the GPU box: PMC traffic passes (config 2
# and config 4, tagged with the library's build id), the bench line (reads the
# fresh traffic), and the kernel-trace profile of the bench.  Parity tests run
# after the counter passes (one of them checks the traffic of this build).
#   bash scripts/gpu_measure.sh
#     -> gpurun_out/{pytest_gpu.log, pmc_*, pmc_table*.txt, pmc_traffic.json, bench.log, prof/}
# Copy gpurun_out/pmc_traffic.json to profiles/ afterwards (on this host).
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_* gpurun_out/pmc4
bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_table.txt
python scripts/pmc_traffic.py gpurun_out gpurun_out/pmc_traffic.json --workload config2 > gpurun_out/pmc_traffic.txt
PMC_DIR=gpurun_out/pmc4 PMC_BENCH_ARGS="--config 4" bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out/pmc4 > gpurun_out/pmc_table_config4.txt
python scripts/pmc_traffic.py gpurun_out/pmc4 gpurun_out/pmc_traffic.json --workload config4 >> gpurun_out/pmc_traffic.txt
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc4/pmc_FETCH_SIZE gpurun_out/pmc4/pmc_WRITE_SIZE
# the tests after the counters: the N = 2 line test expects this build's traffic
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  echo "tests ok"
fi
bash scripts/gpu_check.sh bench prof
echo "measure ok"
