#!/bin/bash
# The non-default BASELINE configurations on the GPU box (via gpurun), each
# step under its own time limit; the first failure ends the script.
#   scripts/gpu_configs.sh [c1|c4|c4prof|c5|c5full|c5dist|c5dist4|c5dist4s|c3 ...] -> gpurun_out/cfg/
set -e
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
O=gpurun_out/cfg
mkdir -p $O
for s in ${*:-c1 c4 c4prof c5}; do
  case "$s" in
    c1) timeout -k 10 300 python bench.py --config 1 > $O/c1.json 2> $O/c1.err ;;
    c4) timeout -k 10 300 python bench.py --config 4 > $O/c4.json 2> $O/c4.err ;;
    c4prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$R/$O/c4prof" -o run -- \
        python3 "$R/bench.py" --config 4 --steps 3 --warmup 1 --no-cpu > "$R/$O/c4prof.log" 2>&1) ;;
    c5) timeout -k 10 300 python bench.py --config 5 > $O/c5.json 2> $O/c5.err ;;
    c5full) timeout -k 10 900 python bench.py --config 5 --giant 2000000001 --steps 2 --warmup 1 \
              > $O/c5full.json 2> $O/c5full.err ;;
    c5dist) timeout -k 10 300 python bench.py --config 5 --dist --tree dist --ranking ruling \
              > $O/c5dist.json 2> $O/c5dist.err ;;
    c5dist4) timeout -k 10 600 python bench.py --gpus 4 --config 5 --giant 4194304 --ranking ruling \
               --check --steps 2 --warmup 1 > $O/c5dist4.json 2> $O/c5dist4.err ;;
    c5dist4s) timeout -k 10 600 python bench.py --gpus 4 --config 5 --giant 4194304 --ranking ruling \
                --out sharded --check --steps 2 --warmup 1 > $O/c5dist4s.json 2> $O/c5dist4s.err ;;
    c3) timeout -k 10 900 python bench.py --config 3 > $O/c3.json 2> $O/c3.err ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
