#!/bin/bash
# Round 5: the kernel trace of a bench run (yarns included: refresh_caches) --
# k_yarn_doc's own duration next to the HIP-event time of its launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
out=gpurun_out/r5_f
mkdir -p $out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-h2d > $R/$out/bench.log 2>&1) || { echo "prof failed"; tail -5 $R/$out/bench.log; exit 1; }
f=$(find $R/$out/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -20
python3 -c "import json; d=json.loads([l for l in open('$R/$out/bench.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['roofline']['frac'], d['refresh_caches']['ms_per_step'], d['refresh_caches']['kernels_ms_per_step'])"
