"""Print the key fields of a bench.py JSON line (file with possible noise lines)."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.log"):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print("value %.3e nodes/s  ms/step %.2f  kernel-sum %.2f" % (d["value"], d["ms_per_step"], d.get("kernel_sum_ms_per_step", 0)))
    r = d["roofline"]
    print("roofline:", r["kernel"], "%.0f GB/s frac %.3f traffic %s" % (r["achieved"], r["frac"], r["traffic"]))
    for k, v in d.get("kernels_ms_per_step", {}).items():
        print("  %-18s %8.3f ms  %8.1f GB/s" % (k, v, d.get("kernel_gbs", {}).get(k, 0)))
    if d.get("cpu_baseline"):
        print("cpu:", d["cpu_baseline"]["value"], d["cpu_baseline"]["sample"])
