#!/bin/bash
# Round 5: yarns by k_yarn_doc after the fused weave -- yarn parity on every
# list test that asks for yarns, then timing: yarns asked for (this build vs the
# in-kernel staged yarns of libcauseweave_r5a.so) and the plain weave.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_c
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_merge.py tests/test_gpu_stream.py tests/test_gpu_mirror.py tests/test_gpu_k32.py tests/test_gpu_runtime.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for lib in cause_amd/libcauseweave_r5a.so cause_amd/libcauseweave.so; do
  CW_LIB="$PWD/$lib" timeout -k 10 300 python -u scripts/sweep.py '[{}]' --rounds 3 --yarns > $out/y.txt 2> $out/y.err || { tail -5 $out/y.err; exit 1; }
  echo "$lib yarns $(cut -c1-200 $out/y.txt)"
done
timeout -k 10 300 python -u scripts/sweep.py '[{}]' --rounds 3 > $out/n.txt 2> $out/n.err || { tail -5 $out/n.err; exit 1; }
echo "plain $(cut -c1-200 $out/n.txt)"
