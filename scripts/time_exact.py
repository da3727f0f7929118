"""Time the exact path (out-of-domain documents, exact.hip) on the GPU.

    python scripts/time_exact.py [--sizes 100000,1000000] [--batch]

* --batch: the config-2 batch (10,000 x 50,001 nodes) clean, and with 1% of
  its documents orphaned (one node's cause replaced by an absent older id).
* --sizes: one config-2-shaped list of each size on the giant path, clean and
  with each count of --orphans (default 10,100) absent causes; --nonlamport
  adds lists with that many non-Lamport causes (a cause with a larger id).
* --device: inputs and outputs resident in device memory (torch tensors), so
  the times are the weave's alone; otherwise host arrays (PCIe included).
Each case: ms per weave (3 timed calls after a warm-up), the exact path's
kernels (cw_get_kernel_stats) and, where the oracle finishes in seconds, a
check against the literal-rule oracle (or_list_fold_general).  One JSON line
per case.
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


def orphan(off, idk, ck, kd, docs, per_doc, rng):
    """Replace the cause of per_doc random non-root nodes in each of `docs`
    with an id older than the node that no node of the document has."""
    ck = ck.copy()
    for d in docs:
        a, b = int(off[d]), int(off[d + 1])
        srt = np.sort(idk[a:b])
        has = lambda x: (lambda k: k < len(srt) and srt[k] == x)(int(np.searchsorted(srt, x)))
        for j in rng.choice(np.flatnonzero(kd[a:b] != 4) + a, per_doc, replace=False):
            x = int(idk[j]) - 1
            while x > 0 and has(np.uint64(x)):
                x -= 1
            ck[j] = x if x > 0 else ck[j]
    return ck


def nonlamport(off, idk, ck, kd, docs, per_doc, rng):
    """Replace the cause of per_doc random non-root nodes with a younger id."""
    ck = ck.copy()
    for d in docs:
        a, b = int(off[d]), int(off[d + 1])
        srt = np.sort(idk[a:b])
        for j in rng.choice(np.flatnonzero(kd[a:b] != 4) + a, per_doc, replace=False):
            k = int(np.searchsorted(srt, idk[j]))
            if k + 1 < len(srt):
                ck[j] = srt[rng.integers(k + 1, len(srt))]
    return ck


class _Res:
    pass


def run(w, off, idk, ck, kd, lay, steps=3, device=False):
    from cause_amd import abi  # noqa: F401

    if device:
        import torch

        dev = torch.device("cuda", 0)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        N, D = len(idk), len(off) - 1
        g = [t(idk.view(np.int64)), t(ck.view(np.int64)), t(kd)]
        o = {"weave_perm": torch.empty(N, dtype=torch.int32, device=dev),
             "visible_bits": torch.empty((N + 31) // 32, dtype=torch.int32, device=dev),
             "visible_count": torch.empty(D, dtype=torch.int32, device=dev),
             "max_ts": torch.empty(D, dtype=torch.int64, device=dev),
             "status": torch.empty(D, dtype=torch.int32, device=dev)}
        ptrs = {k: v.data_ptr() for k, v in o.items()}
        call = lambda: w.weave_lists_device(off, g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                                            lay, ptrs)
    else:
        call = lambda: w.weave_lists(off, idk, ck, kd, lay)
    res = call()
    w.reset_kernel_stats()
    w.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = call()
    if device:
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    w.set_profiling(False)
    if device:
        res = _Res()
        h = {k: v.cpu().numpy() for k, v in o.items()}
        res.status = h["status"].view(np.uint32)
        res.weave_perm = h["weave_perm"].view(np.uint32)
        bits = np.unpackbits(h["visible_bits"].view(np.uint8), bitorder="little")[:len(idk)]
        res.visible = lambda: bits
    ks = {k: round(v[1] / steps, 3) for k, v in sorted(w.kernel_stats().items(),
                                                        key=lambda kv: -kv[1][1])}
    return res, dt * 1e3, ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="100000,1000000")
    ap.add_argument("--batch", action="store_true")
    ap.add_argument("--check-max", type=int, default=2_000_000)
    ap.add_argument("--orphans", default="10,100")
    ap.add_argument("--nonlamport", default="")
    ap.add_argument("--device", action="store_true")
    a = ap.parse_args()
    import oracle
    from cause_amd import abi, gen

    rng = np.random.default_rng(5)
    w = abi.Weaver(0)
    cases = []
    if a.batch:
        spec = gen.CONFIG2
        off, idk, ck, kd = gen.generate(spec, 0, 10_000, nthreads=16)
        bad = rng.choice(10_000, 100, replace=False)
        cases += [("config2 batch clean", spec, off, idk, ck, kd, None),
                  ("config2 batch, 1% of documents orphaned", spec, off, idk,
                   orphan(off, idk, ck, kd, bad, 1, rng), kd, bad)]
    for n in [int(x) for x in a.sizes.split(",") if x]:
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n)
        off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=16)
        cases.append((f"one list of {n + 1:,} nodes clean", spec, off, idk, ck, kd, None))
        for k in [int(x) for x in a.orphans.split(",") if x]:
            cases.append((f"one list of {n + 1:,} nodes, {k} orphans", spec, off, idk,
                          orphan(off, idk, ck, kd, [0], k, rng), kd, [0]))
        for k in [int(x) for x in a.nonlamport.split(",") if x]:
            cases.append((f"one list of {n + 1:,} nodes, {k} non-Lamport causes", spec, off, idk,
                          nonlamport(off, idk, ck, kd, [0], k, rng), kd, [0]))
    for name, spec, off, idk, ck2, kd, bad in cases:
        res, ms, ks = run(w, off, idk, ck2, kd, spec.layout(), device=a.device)
        st = w.kernel_stats()
        line = {"case": name, "nodes": int(len(idk)), "device_resident": a.device,
                "ms_per_weave": ms, "kernels_ms": ks,
                "resolve_steps": st.get("xsyn_resolve", (0,))[0] // 3,
                "phase2_rounds": st.get("xins_round", (0,))[0] // 3,
                "flagged_docs": int(np.count_nonzero(res.status & (abi.STATUS_ORPHAN |
                                                                   abi.STATUS_NON_LAMPORT)))}
        if bad is not None:
            chk = [int(d) for d in bad][:20]
            if all(int(off[d + 1] - off[d]) <= a.check_max for d in chk):
                mism = 0
                for d in chk:
                    lo, hi = int(off[d]), int(off[d + 1])
                    perm, vis, st = oracle.batch_lists(np.array([0, hi - lo], np.uint64), idk[lo:hi],
                                                       ck2[lo:hi], kd[lo:hi],
                                                       method=oracle.METHOD_GENERAL, nthreads=1)
                    ok = np.array_equal(res.weave_perm[lo:hi], perm) and \
                        np.array_equal(res.visible()[lo:hi], vis)
                    mism += 0 if ok else 1
                line["checked_docs"] = len(chk)
                line["mismatches"] = mism
        print(json.dumps(line), flush=True)
    w.close()


if __name__ == "__main__":
    main()
