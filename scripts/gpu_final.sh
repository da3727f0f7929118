#!/bin/bash
# Round-end measurement on the GPU box: smoke, every GPU test, PMC traffic and SQ
# counters, the bench line (reads the fresh traffic), rocprof kernel stats, the
# config 3/4 lines.  Each step has its own time limit; the first failure ends it.
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
bash scripts/gpu_check.sh smoke
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "tests ok"
bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_table.txt
python scripts/pmc_traffic.py gpurun_out gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.txt
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
PMC_PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_sq_table.txt
bash scripts/gpu_check.sh bench prof
bash scripts/gpu_configs.sh c3 c4
echo "final ok"
