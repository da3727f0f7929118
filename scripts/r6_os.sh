#!/bin/bash
# Round 6 GPU batch: the onesweep sort's tests and A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_onesweep.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/os_tests.log 2>&1 || { echo "os tests failed"; exit 1; }
GEOMS=4 timeout -k 10 300 python -u scripts/sort_bench.py 200000000 35 3 > gpurun_out/os_bench_2e8.log 2>&1 || exit 1
GEOMS=4 timeout -k 10 400 python -u scripts/sort_bench.py 2000000001 35 2 > gpurun_out/os_bench_2e9.log 2>&1 || exit 1
CW_ONESWEEP=4 bash scripts/r6_osexp.sh
echo done
