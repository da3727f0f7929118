"""Time VERDICT r5's exact-path case on the GPU: one 2^18-node config-2-shaped
document with a 16,384-long reverse chain (rank r caused by rank r + 1), against
the same document without the chain -- device-memory calls (inputs and outputs
resident), min of 7 after a warm-up, for each knob set given.

    python scripts/time_reverse_chain.py '[{}, {"CW_X2_JUMP1": "0"}]'

One JSON line per variant: clean and chain ms, the ratio, the exact path's
rounds (xins_round launches), all launches and the per-stage ms of one chain
call (cw_get_kernel_stats).
"""
import dataclasses
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from cause_amd import abi, gen

    variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 18) - 1, seed=35)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=8)
    n = len(idk)
    ck2 = ck.copy()
    srt = np.argsort(idk, kind="stable")
    for q in range(1, 1 + 16_384 - 1):
        ck2[srt[q]] = idk[srt[q + 1]]
    lay = spec.layout()
    dev = torch.device("cuda", 0)
    g_id = torch.from_numpy(idk.view(np.int64)).to(dev)
    g_kd = torch.from_numpy(kd).to(dev)
    g_c = {"clean": torch.from_numpy(ck.view(np.int64)).to(dev),
           "chain": torch.from_numpy(ck2.view(np.int64)).to(dev)}
    o = {"weave_perm": torch.empty(n, dtype=torch.int32, device=dev),
         "visible_bits": torch.empty((n + 31) // 32, dtype=torch.int32, device=dev),
         "visible_count": torch.empty(1, dtype=torch.int32, device=dev),
         "max_ts": torch.empty(1, dtype=torch.int64, device=dev),
         "status": torch.empty(1, dtype=torch.int32, device=dev)}
    ptrs = {k: t.data_ptr() for k, t in o.items()}
    for var in variants:
        old = {k: os.environ.get(k) for k in var}
        os.environ.update(var)
        try:
            w = abi.Weaver(0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        with w:
            rec = {"variant": var, "nodes": n, "chain": 16_384}
            for name in ("clean", "chain"):
                call = lambda: w.weave_lists_device(off, g_id.data_ptr(), g_c[name].data_ptr(),
                                                    g_kd.data_ptr(), lay, ptrs)
                call()
                torch.cuda.synchronize()
                t = []
                for _ in range(7):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    call()
                    torch.cuda.synchronize()
                    t.append(time.perf_counter() - t0)
                rec[f"{name}_ms"] = round(min(t) * 1e3, 3)
            w.reset_kernel_stats()
            w.set_profiling(True)
            w.weave_lists_device(off, g_id.data_ptr(), g_c["chain"].data_ptr(), g_kd.data_ptr(), lay, ptrs)
            torch.cuda.synchronize()
            w.set_profiling(False)
            st = w.kernel_stats()  # name -> (launches, total ms, algorithmic bytes)
            rec["ratio"] = round(rec["chain_ms"] / rec["clean_ms"], 2)
            rec["rounds"] = st.get("xins_round", (0, 0.0, 0.0))[0]
            rec["launches"] = sum(v[0] for v in st.values())
            rec["status"] = int(o["status"].cpu()[0])
            rec["stages_ms"] = {k: [v[0], round(v[1], 4)] for k, v in
                                sorted(st.items(), key=lambda kv: -kv[1][1])[:10]}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
