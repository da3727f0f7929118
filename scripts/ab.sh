#!/bin/bash
# A/B two builds of libcauseweave on ONE box (box-to-box spread is ~10%):
#   bash scripts/ab.sh cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so ['[{}]'] [sweep flags]
# Runs each build's sweep twice, interleaved; one JSON line per run.
A="$1"; B="$2"; V="$3"; [ -n "$V" ] || V="[{}]"; X="$4"
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$A" "$B"; do
    echo "== $lib ($rep)"
    CW_LIB="$PWD/$lib" timeout -k 10 200 python -u scripts/sweep.py "$V" --rounds 2 $X > gpurun_out/ab_run.log 2>&1; rc=$?; grep variant gpurun_out/ab_run.log || { tail -20 gpurun_out/ab_run.log; exit 1; }; [ $rc -eq 0 ] || exit $rc
  done
done
