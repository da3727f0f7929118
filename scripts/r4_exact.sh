#!/bin/bash
# Round 4: the exact path's new rule on the GPU (tests + timings).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_exact
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k giant -x -v --timeout 300 --timeout-method thread \
  > $out/pytest_giant.log 2>&1 || { echo "giant pytest failed"; tail -40 $out/pytest_giant.log; exit 1; }
tail -3 $out/pytest_giant.log
timeout -k 10 600 python -u scripts/time_exact.py --sizes 1000000,67108863 --orphans 1,10,100,1000 \
  --nonlamport 50 --device --check-max 1100000 > $out/time_exact.jsonl 2> $out/time_exact.err || { tail -20 $out/time_exact.err; exit 1; }
cat $out/time_exact.jsonl | python -c "import sys,json; [print(json.loads(l)['case'], round(json.loads(l)['ms_per_weave'],2), json.loads(l).get('resolve_steps'), json.loads(l).get('phase2_rounds'), json.loads(l).get('mismatches')) for l in sys.stdin]"
