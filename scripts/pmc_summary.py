"""Summarise rocprofv3 --pmc runs: per kernel, average counter value per launch.

    python scripts/pmc_summary.py gpurun_out  [-> prints a table, writes pmc.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            # (kernels in an anonymous namespace -- onesweep.hip's -- carry it
            # as a prefix: without it the name is cut at its parenthesis)
            kn = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            name = kn.split("(")[0]
            out[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    data = load(d)
    res = {}
    for k, ctrs in sorted(data.items()):
        res[k] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        res[k]["launches"] = max(len(v) for v in ctrs.values())
    json.dump(res, open(os.path.join(d, "pmc.json"), "w"), indent=1)
    cols = sorted({c for v in res.values() for c in v if c != "launches"})
    print("kernel".ljust(40) + "".join(c.rjust(16) for c in cols))
    for k, v in res.items():
        print(k[:40].ljust(40) + "".join(f"{v.get(c, 0):16.4g}" for c in cols))


if __name__ == "__main__":
    main()
