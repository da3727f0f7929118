#!/bin/bash
# Round 3: non-temporal last reads and write-once stores (a -DCW_NT=1 build,
# cause_amd/libcauseweave_nt.so) vs this build: parity of the NT build, A/B.
set -e
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/ab9
mkdir -p $O
CW_LIB=$PWD/cause_amd/libcauseweave_nt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bench_batch or golden or edge or config" > $O/pytest.log 2>&1
echo "parity (NT) ok"; tail -1 $O/pytest.log
bash scripts/ab.sh cause_amd/libcauseweave.so cause_amd/libcauseweave_nt.so > $O/ab.log 2>&1
cat $O/ab.log
