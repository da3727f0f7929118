"""Round 5: where the exact path's time goes on a 2^18-node config-2 document
with a 16,384-long reverse chain (tests/test_gpu_exact.py's case), inputs and
outputs in device memory: wall time per call (clean vs chain), and the stage
times of one chain call from the library's own kernel stats.

    python scripts/r5_exact_prof.py [--chain 16384] [--nodes 262143]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", type=int, default=16_384)
    ap.add_argument("--nodes", type=int, default=(1 << 18) - 1)
    a = ap.parse_args()
    import torch
    from cause_amd import abi, gen

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.nodes, seed=35)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=8)
    srt = np.argsort(idk, kind="stable")
    ck2 = ck.copy()
    for q in range(1, 1 + a.chain - 1):
        ck2[srt[q]] = idk[srt[q + 1]]
    lay = spec.layout()
    n = len(idk)
    dev = torch.device("cuda:0")
    g_id = torch.from_numpy(idk.view(np.int64)).to(dev)
    g_kd = torch.from_numpy(kd).to(dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev)
    vcount = torch.zeros(1, dtype=torch.int32, device=dev)
    mts = torch.zeros(1, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    out = {}
    with abi.Weaver(0) as w:
        for name, c in (("clean", ck), ("chain", ck2)):
            g_ca = torch.from_numpy(c.view(np.int64)).to(dev)
            ptrs = dict(weave_perm=perm.data_ptr(), visible_bits=bits.data_ptr(),
                        visible_count=vcount.data_ptr(), max_ts=mts.data_ptr(),
                        status=status.data_ptr())
            call = lambda: w.weave_lists_device(off, g_id.data_ptr(), g_ca.data_ptr(), g_kd.data_ptr(),
                                                lay, ptrs)
            call()
            torch.cuda.synchronize()
            t = []
            for _ in range(5):
                t0 = time.perf_counter()
                call()
                torch.cuda.synchronize()
                t.append(time.perf_counter() - t0)
            out[name + "_ms"] = round(min(t) * 1e3, 3)
            w.reset_kernel_stats()
            w.set_profiling(True)
            call()
            torch.cuda.synchronize()
            w.set_profiling(False)
            st = w.kernel_stats()
            out[name + "_stages_ms"] = {k: [v[0], round(v[1], 4)] for k, v in
                                        sorted(st.items(), key=lambda kv: -kv[1][1])}
            out[name + "_stage_sum_ms"] = round(sum(v[1] for v in st.values()), 3)
            out[name + "_launches"] = sum(v[0] for v in st.values())
    out["status"] = int(status.item())
    out["ratio"] = round(out["chain_ms"] / out["clean_ms"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
