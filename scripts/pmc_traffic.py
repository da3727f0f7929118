"""HBM traffic per launch for every weave kernel, from rocprofv3 --pmc passes.

    python scripts/pmc_traffic.py gpurun_out [profiles/pmc_traffic.json]

Reads the pmc.json written by scripts/pmc_summary.py (average counter value per
launch, FETCH_SIZE / WRITE_SIZE in KiB).  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
reads, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Keys are the kernel
names of cw_get_kernel_stats (bench.py's "kernels_ms_per_step").
"""
import json
import os
import re
import sys

ALIAS = {"pack_bits": "packbits", "tree_l": "tree"}  # k_tree_l is the library's "tree" stat


def stat_name(sym):
    base = re.sub(r"<.*", "", sym).strip()
    base = base[2:] if base.startswith("k_") else base
    return ALIAS.get(base, base)


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join("profiles", "pmc_traffic.json")
    pmc = json.load(open(os.path.join(d, "pmc.json")))
    res = {}
    for sym, ctr in pmc.items():
        if "FETCH_SIZE" not in ctr or "WRITE_SIZE" not in ctr or sym.startswith("__"):
            continue
        name = stat_name(sym)
        if name.startswith("radix_"):  # sort passes are reported per key width by the library
            continue
        res[name] = {"kernel": sym, "fetch_kib": ctr["FETCH_SIZE"], "write_kib": ctr["WRITE_SIZE"],
                     "bytes": (2 * ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024.0,
                     "launches_sampled": ctr.get("launches")}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items()):
        print(f"{k:12s} {v['bytes'] / 1e9:9.3f} GB/launch  ({v['kernel']})")


if __name__ == "__main__":
    main()
