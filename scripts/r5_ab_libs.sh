#!/bin/bash
# Round 5: timing A/B of library builds on config 2 (scripts/sweep.py with
# CW_LIB): LIBS="a.so b.so" [SWEEP='[{}]'] [ARGS=--yarns], two alternations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_ab_libs
mkdir -p $out
DEF='[{}]'
V="${SWEEP:-$DEF}"
for rep in 1 2; do
  for lib in $LIBS; do
    CW_LIB="$PWD/$lib" timeout -k 10 300 python -u scripts/sweep.py "$V" --rounds 3 $ARGS > $out/s.txt 2> $out/s.err || { tail -5 $out/s.err; exit 1; }
    echo "$lib $(cut -c1-300 $out/s.txt | tr '\n' ' ')"
  done
done
