#!/bin/bash
# Run on the GPU box (via gpurun): parity tests, bench, kernel-trace profile.
#   scripts/gpu_check.sh [tests|bench|prof|pmc ...]   (default: tests bench prof)
# Every GPU step has its own time limit; the first failure ends the script.
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
mkdir -p gpurun_out
steps="${*:-tests bench prof}"
for s in $steps; do
  case "$s" in
    tests)
      timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$R/gpurun_out/prof" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/bench_prof.log" 2>&1) ;;
    pmc)
      # HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE in separate passes
      # PMC_PASSES: passes separated by ';', counters of one pass by spaces
      # PMC_DIR: where the pmc_<counters> directories go (default gpurun_out)
      P="${PMC_DIR:-gpurun_out}"
      mkdir -p "$R/$P"
      IFS=';' read -ra passes <<< "${PMC_PASSES:-FETCH_SIZE;WRITE_SIZE}"
      for pass in "${passes[@]}"; do
        tag=$(echo $pass | tr ' ' '_')
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace \
          --pmc $pass --output-format csv -d "$R/$P/pmc_$tag" -o run -- \
          python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu --no-refresh --no-h2d --check-docs 0 ${PMC_BENCH_ARGS:-} > "$R/$P/pmc_$tag.log" 2>&1)
      done ;;
    list)
      (cd /tmp && rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1) ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
