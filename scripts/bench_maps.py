"""Time cw_weave_maps on the config-4 shape (BASELINE.json configs[3]):
CausalMap collections of 100 nodes, keys Zipf(1.1) over 256 tokens.

    python scripts/bench_maps.py [--colls 100000] [--steps 3]

Host-memory API (inputs copied to the GPU inside the timed call); prints one
JSON line with nodes/s, key weaves and the per-kernel HIP-event times.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--colls", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from cause_amd import abi, gen

    spec = gen.CONFIG4
    lay, tb = spec.layout()
    t0 = time.time()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, a.colls, nthreads=16)
    t_gen = time.time() - t0
    N = len(idk)
    with abi.Weaver(0) as w:
        res = w.weave_maps(off, idk, ck, ci, kd, tb, lay.key_bits)  # warm-up
        assert not res.status.any()
        w.set_profiling(True)
        w.reset_kernel_stats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            res = w.weave_maps(off, idk, ck, ci, kd, tb, lay.key_bits)
        dt = (time.perf_counter() - t0) / a.steps
        st = w.kernel_stats()
    print(json.dumps({
        "metric": "map nodes woven/sec (config 4 shape, host-memory API incl. PCIe)",
        "value": N / dt, "unit": "nodes/s", "ms_per_call": dt * 1e3, "colls": a.colls,
        "nodes": N, "key_weaves": int(len(res.seg_key)), "gen_s": t_gen,
        "kernels_ms_per_call": {k: round(v[1] / a.steps, 3) for k, v in
                                sorted(st.items(), key=lambda kv: -kv[1][1])}}))


if __name__ == "__main__":
    main()
