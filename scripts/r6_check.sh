#!/bin/bash
# Round 6 check on the GPU box: every GPU test, then the default bench line
# (config 2, with the sample parity check on the timed step's outputs).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
echo "tests ok"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok"
