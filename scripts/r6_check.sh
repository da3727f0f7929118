#!/bin/bash
# Round 6 check on the GPU box: every GPU test, the default bench line
# (config 2, with the sample parity check on the timed step's outputs), and the
# full config-5 line.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} \
  > gpurun_out/pytest_gpu.log 2>&1
echo "tests ok"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok"
timeout -k 10 900 python bench.py --config 5 --giant 2000000001 --steps 2 --warmup 1 \
  > gpurun_out/c5full.json 2> gpurun_out/c5full.err
echo "c5 ok"
