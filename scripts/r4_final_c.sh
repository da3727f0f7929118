#!/bin/bash
# Round-4 final, part C: the default bench line, rocprof kernel stats of the
# same command, the config 1 / 3 / 4 / 5 lines.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$PWD}"
cd "$R"
out=gpurun_out/r4_final_c
rm -rf $out
mkdir -p $out
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']); print(d.get('refresh_caches',{}).get('ms_per_step'))"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/$out/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu > "$R/$out/bench_prof.log" 2>&1) \
   || { echo "prof failed"; tail -5 $out/bench_prof.log; exit 1; }
echo "prof ok"
for c in 1 3 4 5; do
  timeout -k 10 600 python -u bench.py --config $c > $out/c$c.json 2> $out/c$c.err || { echo "config $c failed"; tail -10 $out/c$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/c$c.json')); print($c, d['value']/1e9, d['ms_per_step'], d['roofline'].get('kernel'), d['roofline'].get('frac'), d['roofline'].get('traffic'))"
done
echo "part C ok"
