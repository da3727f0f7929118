#!/bin/bash
# GPU-box perf round: list parity tests, a sweep of variants, optional PMC passes.
#   SWEEP='[{}]' PMC_PASSES='FETCH_SIZE;WRITE_SIZE' bash scripts/gpu_perf.sh
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
DEFAULT_SWEEP='[{}]'
SWEEP="${SWEEP:-$DEFAULT_SWEEP}"
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/sweep.py "$SWEEP" --check > gpurun_out/sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "$PMC_PASSES" ]; then
  rm -rf gpurun_out/pmc_*
  bash scripts/gpu_check.sh pmc; rc=$?
  echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_table.txt 2>&1
fi
