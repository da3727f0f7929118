"""Time the exact path (out-of-domain documents, exact.hip) on the GPU.

    python scripts/time_exact.py [--sizes 100000,1000000] [--batch]

* --batch: the config-2 batch (10,000 x 50,001 nodes) clean, and with 1% of
  its documents orphaned (one node's cause replaced by an absent older id).
* --sizes: one config-2-shaped list of each size on the giant path, clean and
  with 10 orphans.
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
        ids = set(idk[a:b].tolist())
        for j in rng.choice(np.arange(a, b)[kd[a:b] != 4], per_doc, replace=False):
            x = int(idk[j]) - 1
            while x > 0 and x in ids:
                x -= 1
            ck[j] = x if x > 0 else ck[j]
    return ck


def run(w, off, idk, ck, kd, lay, steps=3):
    from cause_amd import abi  # noqa: F401

    res = w.weave_lists(off, idk, ck, kd, lay)
    w.reset_kernel_stats()
    w.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = w.weave_lists(off, idk, ck, kd, lay)
    dt = (time.perf_counter() - t0) / steps
    w.set_profiling(False)
    ks = {k: round(v[1] / steps, 3) for k, v in sorted(w.kernel_stats().items(),
                                                        key=lambda kv: -kv[1][1])}
    return res, dt * 1e3, ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="100000,1000000")
    ap.add_argument("--batch", action="store_true")
    ap.add_argument("--check-max", type=int, default=2_000_000)
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
        cases += [(f"one list of {n + 1:,} nodes clean", spec, off, idk, ck, kd, None),
                  (f"one list of {n + 1:,} nodes, 10 orphans", spec, off, idk,
                   orphan(off, idk, ck, kd, [0], 10, rng), kd, [0])]
    for name, spec, off, idk, ck2, kd, bad in cases:
        res, ms, ks = run(w, off, idk, ck2, kd, spec.layout())
        line = {"case": name, "nodes": int(len(idk)), "ms_per_weave": ms, "kernels_ms": ks,
                "synthetic_iterations": w.kernel_stats().get("xsyn_attach", (0,))[0] // 3,
                "flagged_docs": int(np.count_nonzero(res.status & abi.STATUS_ORPHAN))}
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
