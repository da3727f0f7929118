#!/bin/bash
# onesweep sort on the GPU: its unit tests, the giant-path test that failed with
# the first cut, then the sort A/B at 2e8 and 2e9 random 35-bit keys
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_onesweep.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/os_tests.log 2>&1 || { echo "os tests failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread -k "giant_document_corrupted" \
  > gpurun_out/os_exact.log 2>&1 || { echo "exact failed"; exit 1; }
GEOMS=0,1,2 timeout -k 10 300 python -u scripts/sort_bench.py 200000000 35 3 > gpurun_out/os_bench_2e8.log 2>&1 || exit 1
GEOMS=0,2 timeout -k 10 400 python -u scripts/sort_bench.py 2000000001 35 2 > gpurun_out/os_bench_2e9.log 2>&1 || exit 1
echo done
