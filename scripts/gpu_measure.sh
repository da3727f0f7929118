#!/bin/bash
# Round measurement on the GPU box: parity tests, PMC traffic passes, the bench
# line (reads the fresh traffic), and the kernel-trace profile of the bench.
#   bash scripts/gpu_measure.sh   -> gpurun_out/{pytest_gpu.log, pmc_*, pmc_traffic.json, bench.log, prof/}
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_*
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  echo "tests ok"
fi
bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_table.txt
python scripts/pmc_traffic.py gpurun_out gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.txt
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
bash scripts/gpu_check.sh bench prof
echo "measure ok"
