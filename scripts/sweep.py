"""A/B launch-geometry variants of the weave in ONE process on one workload.

    python scripts/sweep.py '[{}, {"CW_FUSED":"0"}]' [--docs 10000] [--rounds 3]

Each variant gets its own context (knobs are read at cw_ctx_create); rounds
interleave the variants; per-kernel ms come from the library's HIP events.
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--docs", type=int, default=10_000)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", action="store_true", help="compare outputs across variants")
    ap.add_argument("--yarns", action="store_true", help="ask for yarn_perm too (refresh-caches)")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    import torch

    from cause_amd import abi, gen

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.nodes)
    lay = spec.layout()
    t0 = time.time()
    import threading
    done = threading.Event()

    def beat():  # (a long generation must not look hung to the box's silence limit)
        while not done.wait(30):
            print(f"generating: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    off, idk, ck, kd = gen.generate(spec, 0, a.docs, nthreads=16)
    done.set()
    print(f"generated {len(idk):,} nodes in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    N, D = len(idk), a.docs
    dev = torch.device("cuda", 0)
    g_id = torch.from_numpy(idk.view(np.int64)).to(dev)
    g_ca = torch.from_numpy(ck.view(np.int64)).to(dev)
    g_kd = torch.from_numpy(kd).to(dev)
    o = {"weave_perm": torch.empty(N, dtype=torch.int32, device=dev),
         "visible_bits": torch.empty((N + 31) // 32, dtype=torch.int32, device=dev),
         "visible_count": torch.empty(D, dtype=torch.int32, device=dev),
         "max_ts": torch.empty(D, dtype=torch.int64, device=dev),
         "status": torch.empty(D, dtype=torch.int32, device=dev)}
    if a.yarns:
        o["yarn_perm"] = torch.empty(N, dtype=torch.int32, device=dev)
    ptrs = {k: t.data_ptr() for k, t in o.items()}
    ref = None
    results = {i: [] for i in range(len(variants))}
    stats = {}
    # contexts hold ~40 GB of scratch each at full size: one live context at a time,
    # variants visited twice (A B C ... A B C) so drift shows up
    for sweep in range(2):
        for i, v in enumerate(variants):
            for k, val in v.items():
                os.environ[k] = str(val)
            w = abi.Weaver(0)
            for k in v:
                del os.environ[k]
            w.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            w.weave_lists_device(off, g_id.data_ptr(), g_ca.data_ptr(), g_kd.data_ptr(), lay, ptrs)
            torch.cuda.synchronize()
            if a.check:
                if ref is None:
                    ref = {k: t.clone() for k, t in o.items()}
                else:
                    for k, t in o.items():
                        assert torch.equal(t, ref[k]), f"{k} differs from variant 0"
                assert int(o["status"].max()) == 0
            w.set_profiling(True)
            w.reset_kernel_stats()
            for r in range(a.rounds):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                w.weave_lists_device(off, g_id.data_ptr(), g_ca.data_ptr(), g_kd.data_ptr(), lay,
                                     ptrs)
                torch.cuda.synchronize()
                results[i].append(time.perf_counter() - t0)
            st = w.kernel_stats()
            print(f"sweep {sweep} variant {i}: {min(results[i]) * 1e3:.2f} ms", file=sys.stderr, flush=True)
            for k, x in st.items():
                stats.setdefault(i, {}).setdefault(k, []).append(x[1] / a.rounds)
            w.close()
            del w
            torch.cuda.empty_cache()
    if a.check:
        print("outputs identical across variants")
    for i, v in enumerate(variants):
        per = {k: round(min(x), 3) for k, x in sorted(stats[i].items(), key=lambda kv: -min(kv[1]))}
        print(json.dumps({"variant": v, "ms_min": round(min(results[i]) * 1e3, 2),
                          "ms_med": round(float(np.median(results[i])) * 1e3, 2),
                          "gnodes_s": round(N / min(results[i]) / 1e9, 3), "kernels": per}))


if __name__ == "__main__":
    main()
