#!/bin/bash
# Round 5: k_yarn_doc variants -- yarn parity (the list parity tests), then the
# yarns step timed against the plain weave.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r5_d
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/sweep.py '[{}]' --rounds 3 --yarns > $out/y.txt 2> $out/y.err || { tail -5 $out/y.err; exit 1; }
echo "yarns $(cut -c1-200 $out/y.txt)"
