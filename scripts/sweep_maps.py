"""A/B knob variants of cw_weave_maps in ONE process on the config-4 workload
(device memory, 10^6 collections x 100 nodes by default).

    python scripts/sweep_maps.py '[{}, {"CW_MAP_SMALL": "0"}]' [--colls 1000000] [--rounds 3]

Each variant gets its own context (knobs are read at cw_ctx_create); rounds
interleave the variants; per-kernel ms come from the library's HIP events.
--check compares every variant's outputs with the first one's.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--colls", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    import torch

    from cause_amd import abi, gen

    spec = gen.CONFIG4
    lay, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, a.colls, nthreads=16)
    N, D = len(idk), a.colls
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    ins = [t(idk), t(ck), t(ci), t(kd)]
    cap = N
    outs = {"seg_offsets": torch.empty(cap + 1, dtype=torch.int64, device=dev),
            "seg_coll": torch.empty(cap, dtype=torch.int32, device=dev),
            "seg_key": torch.empty(cap, dtype=torch.int64, device=dev),
            "seg_active": torch.empty(cap, dtype=torch.int64, device=dev),
            "seg_perm": torch.empty(N + cap, dtype=torch.int32, device=dev),
            "status": torch.empty(D, dtype=torch.int32, device=dev)}
    ptrs = {k: v.data_ptr() for k, v in outs.items()}
    res = {i: [] for i in range(len(variants))}
    ref = None
    for rnd in range(a.rounds):
        for i, v in enumerate(variants):
            for k, val in v.items():
                os.environ[k] = str(val)
            w = abi.Weaver(0)
            for k in v:
                del os.environ[k]
            w.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            S = w.weave_maps_device(off, [x.data_ptr() for x in ins], tb, lay.key_bits, ptrs, cap)
            torch.cuda.synchronize()
            if a.check and rnd == 0:
                got = [outs["seg_perm"][:N + S].cpu(), outs["seg_active"][:S].cpu(),
                       outs["seg_key"][:S].cpu(), outs["status"].cpu()]
                if ref is None:
                    ref = got
                else:
                    names = ["seg_perm", "seg_active", "seg_key", "status"]
                    bad = [nm for nm, x, y in zip(names, ref, got) if not torch.equal(x, y)]
                    if bad:
                        x, y = ref[names.index(bad[0])], got[names.index(bad[0])]
                        n = min(len(x), len(y))
                        diff = torch.nonzero(x[:n] != y[:n]).flatten()[:5].tolist()
                        print(json.dumps({"variant": v, "differs": bad, "S": S, "first": diff,
                                          "ref": [int(x[k]) for k in diff], "got": [int(y[k]) for k in diff]}))
                        raise SystemExit(1)
            w.set_profiling(True)
            w.reset_kernel_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                w.weave_maps_device(off, [x.data_ptr() for x in ins], tb, lay.key_bits, ptrs, cap)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            st = w.kernel_stats()
            res[i].append((dt * 1e3, {k: s[1] / 3 for k, s in st.items()}))
            w.close()
    for i, v in enumerate(variants):
        ms = sorted(r[0] for r in res[i])
        ker = {}
        for _, st in res[i]:
            for k, x in st.items():
                ker[k] = min(ker.get(k, 1e9), x)
        print(json.dumps({"variant": v, "ms_min": round(ms[0], 2), "ms_med": round(ms[len(ms) // 2], 2),
                          "gnodes_s": round(N / ms[0] / 1e6, 3),
                          "kernels": {k: round(x, 3) for k, x in sorted(ker.items(), key=lambda kv: -kv[1])[:4]}}))


if __name__ == "__main__":
    main()
