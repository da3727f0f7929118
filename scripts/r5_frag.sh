#!/bin/bash
# Round 5: random reads over a fresh table vs one of scattered 2 MiB pieces
# (scripts/calib_frag.hip), with the UTCL1 translation counters of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
out=gpurun_out/r5_frag
mkdir -p $out
(rocprofv3 -L > $out/counters.txt 2>&1 || true)
grep -i -E "utcl|tlb|transl|ATC|walk" $out/counters.txt | head -40 > $out/xlat_counters.txt || true
timeout -k 10 120 scripts/calib_frag 0 > $out/fresh.jsonl 2> $out/fresh.err || { echo "fresh failed"; exit 1; }
timeout -k 10 300 scripts/calib_frag 1 280 > $out/frag.jsonl 2> $out/frag.err || { echo "frag failed"; cat $out/frag.err; exit 1; }
cat $out/fresh.jsonl $out/frag.jsonl $out/frag.err
for m in 0 1; do
  (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/$out/pmc_$m -o run -- $R/scripts/calib_frag $m 280 > $R/$out/pmc_$m.log 2>&1) || { echo "pmc $m failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for m in (0, 1):
    f = glob.glob(f"gpurun_out/r5_frag/pmc_{m}/**/run_counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    acc = collections.defaultdict(dict)
    for r in rows:
        if "k_chase" not in r["Kernel_Name"]: continue
        acc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    for d, v in sorted(acc.items(), key=lambda kv: int(kv[0])):
        req = v.get("TCP_UTCL1_REQUEST_sum", 0)
        print(m, d, {k.replace("TCP_UTCL1_", ""): f"{x:.3g}" for k, x in v.items()},
              "miss_frac %.3f" % (v.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / max(req, 1)))
PY
cat $out/xlat_counters.txt
