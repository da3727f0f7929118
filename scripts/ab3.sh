#!/bin/bash
# A/B several builds of libcauseweave on ONE box, interleaved (box-to-box spread is ~10%):
#   bash scripts/ab3.sh '[{}]' "sweep flags" lib1.so lib2.so ...
V="$1"; X="$2"; shift 2
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib ($rep)"
    CW_LIB="$PWD/$lib" timeout -k 10 200 python -u scripts/sweep.py "$V" --rounds 2 $X > gpurun_out/ab_run.log 2>&1; rc=$?; grep variant gpurun_out/ab_run.log || { tail -20 gpurun_out/ab_run.log; exit 1; }; [ $rc -eq 0 ] || exit $rc
  done
done
