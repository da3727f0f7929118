#!/bin/bash
# A/B on one box: libcauseweave_base.so vs libcauseweave.so (config-2 weave, then
# with yarns), then the list parity tests of the new build
mkdir -p gpurun_out
timeout -k 10 500 bash scripts/ab.sh cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so '[{}]' > gpurun_out/ab.log 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 500 bash scripts/ab.sh cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so '[{}]' --yarns > gpurun_out/ab_y.log 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/parity.log 2>&1 || { echo "parity failed"; exit 1; }
echo done
