#!/bin/bash
# Round-4 final, part B (after profiles/pmc_traffic.json holds this build's
# counters): every GPU test, the default bench line, its rocprof kernel stats,
# the config 1 / 3 / 4 / 5 lines.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
out=gpurun_out/r4_final_b
rm -rf $out
mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
echo "tests ok"
