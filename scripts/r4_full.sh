#!/bin/bash
# Round 4: the whole GPU suite, smoke and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r4_full
mkdir -p $out
timeout -k 10 300 python -u __graft_entry__.py smoke > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d.get('refresh_caches',{}).get('ms_per_step'))"
