#!/bin/bash
# Round-end measurement on the GPU box: smoke, every GPU test, PMC traffic
# (config 2 + config 4, build-tagged), the bench line (reads the fresh traffic),
# rocprof kernel stats, SQ counters, the config 3/4 lines.  Each step has its own
# time limit; the first failure ends it.
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
bash scripts/gpu_check.sh smoke
bash scripts/gpu_measure.sh
PMC_PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" PMC_DIR=gpurun_out/pmcsq bash scripts/gpu_check.sh pmc
python scripts/pmc_summary.py gpurun_out/pmcsq > gpurun_out/pmc_sq_table.txt
rm -rf gpurun_out/pmcsq/pmc_SQ*
bash scripts/gpu_configs.sh c3 c4
echo "final ok"
