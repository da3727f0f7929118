#!/bin/bash
# Round 5, first GPU pass: map self-cause and exact-path anchor parity, the
# yarn staging's parity, then an A/B of the staged yarns (libcauseweave.so)
# against the round-4 per-thread yarns (libcauseweave_base.so), yarns asked for.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_a
mkdir -p $out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_maps.py > $out/maps.log 2>&1 || { echo "maps failed"; tail -30 $out/maps.log; exit 1; }
tail -1 $out/maps.log
timeout -k 10 600 $T -s tests/test_gpu_exact.py > $out/exact.log 2>&1 || { echo "exact failed"; tail -40 $out/exact.log; exit 1; }
tail -1 $out/exact.log
grep -h "rounds\|reverse\|chain" $out/exact.log | head -10
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $out/parity.log 2>&1 || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for rep in 1 2; do
  for lib in cause_amd/libcauseweave_base.so cause_amd/libcauseweave.so; do
    CW_LIB="$PWD/$lib" timeout -k 10 300 python -u scripts/sweep.py '[{}]' --rounds 3 --yarns > $out/ab_$rep.txt 2> $out/ab_$rep.err || { tail -5 $out/ab_$rep.err; exit 1; }
    echo "$lib $(cut -c1-220 $out/ab_$rep.txt)"
  done
done
# the counters this box lists (address translation, for the giant path's walk)
(cd /tmp && timeout -k 5 60 rocprofv3 -L > "$OLDPWD/$out/counters.txt" 2>&1) || true
grep -io "[A-Za-z_0-9]*\(UTCL\|TLB\|TRANSLAT\)[A-Za-z_0-9]*" $out/counters.txt | sort -u | head -40
