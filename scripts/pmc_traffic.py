"""HBM traffic per launch for every weave kernel, from rocprofv3 --pmc passes.

    python scripts/pmc_traffic.py gpurun_out [profiles/pmc_traffic.json] [--workload config2]

Reads the pmc.json written by scripts/pmc_summary.py (average counter value per
launch, FETCH_SIZE / WRITE_SIZE in KiB).  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
reads, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Keys are the kernel
names of cw_get_kernel_stats (bench.py's "kernels_ms_per_step").

The table records the build id of the library the counters were taken on
(cw_build_id, a hash of the sources): bench.py reports `traffic` only when the
library it times has that id, so a kernel change cannot inherit stale counters.
Workloads measured on the same build accumulate in one file.
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# k_tree_l is the library's "tree" stat, k_weave_doc its "weave", k_map_pack its "m_pack"
ALIAS = {"pack_bits": "packbits", "tree_l": "tree", "weave_doc": "weave", "map_pack": "m_pack",
         "gjoin": "join", "lvl_walk": "rank", "sup_rank": "rank", "lvl_apply": "rank",
         "lvl_emit": "rank", "gd_build": "index", "gcross_ns": "gcross", "gcross_fc": "gcross"}


def stat_name(sym):
    base = re.sub(r"<.*", "", sym).strip()
    base = base[2:] if base.startswith("k_") else base
    return ALIAS.get(base, base)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out")
    ap.add_argument("out", nargs="?", default=os.path.join("profiles", "pmc_traffic.json"))
    ap.add_argument("--workload", default="config2",
                    help="bench workload the passes ran (bench.py --config N -> configN)")
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    from cause_amd import abi

    bid = abi.build_id()
    pmc = json.load(open(os.path.join(a.dir, "pmc.json")))
    res = {}
    for sym, ctr in pmc.items():
        if "FETCH_SIZE" not in ctr or "WRITE_SIZE" not in ctr or sym.startswith("__"):
            continue
        if not sym.startswith("k_"):  # torch's own kernels (status readbacks)
            continue
        name = stat_name(sym)
        if name.startswith("os_"):
            # the one-sweep sort (onesweep.hip): by key width on the giant path,
            # as the histogram-scan-scatter kernels below; its scan is one block
            if not a.workload.startswith(("config1", "config5")) or name.startswith("os_scan") or \
                    "<" not in sym:
                continue
            width = "idsort" if "unsigned long" in sym else "gsort"
            part = "scatter" if name.startswith("os_pass") else "hist"
            name = f"{width}_{part}"
        elif name.startswith("radix_") or name.startswith("gscan_"):
            # the library reports sort passes by what they sort: on the giant
            # path (configs 1, 5) the 64-bit keys are the id sort, the 32-bit
            # ones the group-key sort; elsewhere they are not separable
            if not a.workload.startswith(("config1", "config5")) or not name.startswith("radix_") or \
                    "<" not in sym:
                continue  # (the scans serve both sorts)
            width = "idsort" if "unsigned long" in sym else "gsort"
            part = name.split("_", 1)[1].split("<")[0]
            name = f"{width}_{part}"
        if name in ("gd_first", "gd_set_sorted"):  # the library's "index" stat: both kernels
            name = "index"
        r = res.setdefault(name, {"kernel": [], "fetch_kib": 0.0, "write_kib": 0.0,
                                  "launches_sampled": ctr.get("launches")})
        r["kernel"].append(sym)
        if name.startswith(("idsort_", "gsort_")):
            # one launch a pass, a kernel per pass role (the id sort's payload):
            # the average a launch, weighted by each symbol's launches
            n = ctr.get("launches") or 1
            r["_n"] = r.get("_n", 0) + n
            r["_f"] = r.get("_f", 0.0) + ctr["FETCH_SIZE"] * n
            r["_w"] = r.get("_w", 0.0) + ctr["WRITE_SIZE"] * n
            r["fetch_kib"], r["write_kib"] = r["_f"] / r["_n"], r["_w"] / r["_n"]
            r["launches_sampled"] = r["_n"]
        else:
            # several symbols under one library stat (the ranking's levels, the
            # index's two kernels): their bytes per launch add up
            r["fetch_kib"] += ctr["FETCH_SIZE"]
            r["write_kib"] += ctr["WRITE_SIZE"]
        r["bytes"] = (2 * r["fetch_kib"] + r["write_kib"]) * 1024.0
    for r in res.values():
        r["kernel"] = " + ".join(r["kernel"])
        for k in ("_n", "_f", "_w"):
            r.pop(k, None)
    table = {"build_id": bid, "workloads": {}}
    if os.path.exists(a.out):
        old = json.load(open(a.out))
        if old.get("build_id") == bid:
            table = old
    table["workloads"][a.workload] = res
    json.dump(table, open(a.out, "w"), indent=1, sort_keys=True)
    print(f"build {bid}, workload {a.workload}")
    for k, v in sorted(res.items()):
        print(f"{k:12s} {v['bytes'] / 1e9:9.3f} GB/launch  ({v['kernel']})")


if __name__ == "__main__":
    main()
