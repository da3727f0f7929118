"""The exact path on the GPU: documents outside the fast path's domain get the
reference's literal weave (list.cljc:26-28 -> shared.cljc:225-241), bit-exact
against oracle METHOD_LITERAL -- order, rendered bits, counts, ::lamport-ts,
yarns -- with their status bits kept (exact.hip).

Inputs (tests/outdomain.py): absent causes, causes with a larger id, nil
causes, no root, ids below the root, non-id causes; in tiny reference-style
histories, the reference's edge cases, config-2-shaped documents up to the
full 50,001 nodes, next to in-domain documents in the same batch, through every
front end, host and device memory, and cw_weave_ranked.
"""
import dataclasses
import random

import numpy as np
import pytest

import oracle
from cause_amd import abi, gen, pack
from oracle import causal_ref as R
from tests import outdomain as X
from tests import refgen as G
from tests.test_gpu_parity import check_batch, oracle_batch, weaver  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def test_reference_style_histories_every_corruption(weaver):
    rng = random.Random(4)
    docs = []
    for kinds in [(k,) for k in X.KINDS] + [X.KINDS]:
        for steps in (5, 9, 20, 60):
            for _ in range(6):
                nodes, _ = G.random_history(rng, steps)
                d = X.corrupt([R.ROOT_NODE] + nodes, rng, kinds, rate=0.2)
                rng.shuffle(d)
                docs.append(d)
    for case in G.EDGE_CASES:
        for k in X.KINDS:
            docs.append(X.corrupt([R.ROOT_NODE] + list(case), rng, (k,), rate=0.3))
    b = pack.pack_lists(docs)
    res = check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    assert (res.status != 0).mean() > 0.8


def test_stress_histories_corrupted(weaver):
    rng = random.Random(8)
    docs = []
    for n in (50, 300, 1200):
        for p_special in (0.1, 0.4):
            nodes = G.stress_history(rng, n, p_special=p_special, p_conj=0.2, tx_chain=0.1)
            docs.append(X.corrupt(nodes, rng, X.KINDS, rate=0.03))
            docs.append(nodes)  # in-domain neighbours
    b = pack.pack_lists(docs)
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


@pytest.mark.parametrize("n,D", [(3000, 20), (50_000, 6)])
def test_config2_documents_corrupted(weaver, n, D):
    """Config-2-shaped documents, every other one broken (the bits of flagged
    and clean documents share words at the boundaries)."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n, seed=n + D)
    off, idk, ck, kd = gen.generate(spec, 0, D, nthreads=8)
    rng = np.random.default_rng(n)
    parts = []
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        one = (np.array([0, b - a], np.uint64), idk[a:b], ck[a:b], kd[a:b])
        if d % 2:
            one = X.corrupt_packed(*one, rng, rate=0.01)
        parts.append(one)
    sizes = [int(p[0][-1]) for p in parts]
    off2 = np.zeros(D + 1, np.uint64)
    off2[1:] = np.cumsum(sizes)
    cat = lambda j: np.concatenate([p[j] for p in parts])
    res = check_batch(weaver, off2, cat(1), cat(2), cat(3), spec.layout())
    assert (res.status[1::2] != 0).all() and not res.status[0::2].any()


def test_giant_document_corrupted():
    """One document above the giant-path threshold (one-document batch): the
    tree runs on the all-parallel path, the fold on one lane."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=150_000, seed=9)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=8)
    off, idk, ck, kd = X.corrupt_packed(off, idk, ck, kd, np.random.default_rng(2),
                                        rate=0.001, which="mixed")
    with abi.Weaver(0) as w:
        res = check_batch(w, off, idk, ck, kd, spec.layout())
    assert res.status[0] & (abi.STATUS_ORPHAN | abi.STATUS_NON_LAMPORT)


def test_device_memory_async_corrupted():
    """Device pointers, the context on a torch stream in async mode: the exact
    path runs inside the same call (ordered on that stream)."""
    import torch

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=4000, seed=5)
    off, idk, ck, kd = gen.generate(spec, 0, 12, nthreads=8)
    off, idk, ck, kd = X.corrupt_packed(off, idk, ck, kd, np.random.default_rng(3))
    lay = spec.layout()
    N, D = len(idk), len(off) - 1
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    g = [t(idk.view(np.int64)), t(ck.view(np.int64)), t(kd)]
    o = {"weave_perm": torch.empty(N, dtype=torch.int32, device=dev),
         "visible_bits": torch.empty((N + 31) // 32, dtype=torch.int32, device=dev),
         "visible_count": torch.empty(D, dtype=torch.int32, device=dev),
         "max_ts": torch.empty(D, dtype=torch.int64, device=dev),
         "status": torch.empty(D, dtype=torch.int32, device=dev),
         "yarn_perm": torch.empty(N, dtype=torch.int32, device=dev)}
    s = torch.cuda.Stream(dev)
    with abi.Weaver(0) as w:
        w.set_stream(s.cuda_stream)
        w.set_async(True)
        w.weave_lists_device(off, g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(), lay,
                             {k: v.data_ptr() for k, v in o.items()})
        s.synchronize()
    perm, vis, st, vcount, max_ts = oracle_batch(off, idk, ck, kd, lay)
    h = {k: v.cpu().numpy() for k, v in o.items()}
    assert np.array_equal(h["status"].view(np.uint32), st)
    assert np.array_equal(h["weave_perm"].view(np.uint32), perm)
    gvis = np.unpackbits(h["visible_bits"].view(np.uint8), bitorder="little")[:N]
    assert np.array_equal(gvis, vis)
    assert np.array_equal(h["visible_count"].view(np.uint32), vcount)
    assert np.array_equal(h["max_ts"].view(np.uint64), max_ts)
    mask = (1 << lay.site_bits) - 1
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        assert np.array_equal(h["yarn_perm"][a:b].view(np.uint32),
                              oracle.list_yarns(idk[a:b], lay.site_shift, mask))


@pytest.mark.parametrize("case", ["orphan", "orphan_few", "non_lamport", "no_root_first"])
def test_weave_ranked_exact(case):
    """cw_weave_ranked (the distributed giant list's last step) on a flagged
    list: the literal fold of the ranks."""
    import torch

    from cause_amd import giant
    from tests.test_gpu_giant import ranked_case

    par, kd, val = ranked_case(30_000, 17)
    par = par.view(np.uint32).copy()
    kd = kd.copy()
    rng = np.random.default_rng(1)
    if case in ("orphan", "orphan_few"):  # absent causes: phase 1 of the synthetic lists
        k = 40 if case == "orphan" else 7
        par[rng.choice(np.arange(1, len(par)), k, replace=False)] = 0xFFFFFFFF
    elif case == "non_lamport":
        js = rng.choice(np.arange(1, len(par) - 100), 40, replace=False)
        par[js] = js + rng.integers(1, 100, len(js))
    else:
        kd[0] &= ~np.uint8(4)  # rank 0 not flagged root
        par[5] = 0xFFFFFFFE    # and a nil cause (CW_NIL_RANK)
    n = len(par)
    # the same list as packed ids = ranks for the oracle
    ids = np.arange(n, dtype=np.uint64)
    causes = np.where(par == 0xFFFFFFFF, np.uint64(n + 5),
                      np.where(par == 0xFFFFFFFE, np.uint64(2**64 - 1), par.astype(np.uint64)))
    if kd[0] & 4:
        causes[0] = np.uint64(2**64 - 1)
    want, vis, st = oracle.batch_lists(np.array([0, n], np.uint64), ids, causes, kd,
                                       method=oracle.METHOD_LITERAL)
    with abi.Weaver(0) as w:
        ops = giant.HipOps(w, "cuda:0")
        dev = torch.device("cuda", 0)
        got = ops.weave_ranked(torch.from_numpy(par.view(np.int32)).to(dev),
                               torch.from_numpy(kd).to(dev), torch.from_numpy(val).to(dev))
        torch.cuda.synchronize()
    assert int(got["status"][0]) == int(st[0]) != 0
    assert np.array_equal(got["weave_perm"].cpu().numpy().view(np.uint32), val.view(np.uint32)[want])
    gvis = np.unpackbits(got["visible_bits"].cpu().numpy().view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(gvis, vis)
    assert int(got["visible_count"][0]) == int(vis.sum())


def _orphaned(spec, D, per_doc, rng, nil_every=0):
    """Config-2-shaped documents whose per_doc[d] random nodes get an absent,
    older cause (an id no node has) and, every nil_every-th, a nil cause: the
    synthetic-list path (no non-Lamport cause)."""
    off, idk, ck, kd = gen.generate(spec, 0, D, nthreads=8)
    ck = ck.copy()
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        ids = set(idk[a:b].tolist())
        js = rng.choice(np.arange(a + 1, b), min(per_doc[d], b - a - 1), replace=False)
        for q, j in enumerate(js):
            if nil_every and q % nil_every == nil_every - 1:
                ck[j] = np.uint64((1 << 64) - 1)
                continue
            x = int(idk[j]) - 1
            while x in ids:
                x -= 1
            ck[j] = x
    return off, idk, ck, kd


def _stage_launches(w, name):
    return w.kernel_stats().get(name, (0, 0.0, 0.0))[0]


def _nonlamport(spec, D, per_doc, rng, orphans=None):
    """Config-2-shaped documents whose per_doc[d] random nodes get a cause with
    a larger id (some a node's own id), plus orphans[d] absent causes."""
    off, idk, ck, kd = _orphaned(spec, D, orphans or [0] * D, rng)
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        srt = np.sort(idk[a:b])
        for j in rng.choice(np.arange(a + 1, b), per_doc[d], replace=False):
            k = int(np.searchsorted(srt, idk[j]))
            self_cause = rng.random() < 0.1 or k + 1 >= len(srt)
            ck[j] = srt[k] if self_cause else srt[rng.integers(k + 1, len(srt))]
    return off, idk, ck, kd


def test_orphan_documents_one_resolve_no_rounds():
    """Documents with 1 .. 500 orphans (and nil causes): phase 1 places every
    appended node from one static weave -- one resolve step and two weaves
    whatever the number of orphans (round 3 took one weave per orphan), no
    phase-2 round -- bit-exact against the literal fold."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=6000, seed=31)
    rng = np.random.default_rng(31)
    per = [1, 2, 3, 5, 8, 13, 21, 32, 4, 7, 16, 30, 200, 500, 64, 33]
    off, idk, ck, kd = _orphaned(spec, len(per), per, rng, nil_every=3)
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, spec.layout())
        w.set_profiling(False)
        assert (res.status & abi.STATUS_ORPHAN).all()
        assert _stage_launches(w, "xsyn_resolve") == 1
        assert _stage_launches(w, "xins_round") == 0
        assert "xfold" not in w.kernel_stats()


def test_non_lamport_documents_rounds():
    """Non-Lamport causes (a node caused by a younger node, or by its own id)
    next to orphans and clean documents: phase 2's insertion-tree rounds reach
    the fold's weave; the same batch through the serial fold (CW_XFOLD=1)
    agrees."""
    import os

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000, seed=32)
    rng = np.random.default_rng(32)
    nl = [1, 0, 3, 10, 0, 40, 2, 100]
    orph = [0, 5, 2, 0, 0, 30, 200, 3]
    off, idk, ck, kd = _nonlamport(spec, len(nl), nl, rng, orphans=orph)
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, spec.layout())
        w.set_profiling(False)
        assert 1 <= _stage_launches(w, "xins_round") <= 12
        assert "xfold" not in w.kernel_stats()
    assert all(bool(res.status[d] & abi.STATUS_NON_LAMPORT) == (nl[d] > 0) for d in range(len(nl)))
    os.environ["CW_XFOLD"] = "1"
    try:
        with abi.Weaver(0) as w:
            w.set_profiling(True)
            check_batch(w, off, idk, ck, kd, spec.layout())
            assert "xfold" in w.kernel_stats()
    finally:
        del os.environ["CW_XFOLD"]


@pytest.mark.parametrize("orphans", [1, 10, 300])
def test_giant_list_orphans_synthetic(orphans):
    """A one-document batch on the giant path with absent and nil causes: the
    synthetic lists are woven on the giant path too, one resolve step whatever
    the number of orphans (compared with the C restatement of the exact path's
    rule, or_list_fold_general, itself pinned to the literal fold by
    test_oracle)."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=300_000, seed=33 + orphans)
    rng = np.random.default_rng(orphans)
    off, idk, ck, kd = _orphaned(spec, 1, [orphans], rng, nil_every=4)
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_GENERAL)
        w.set_profiling(False)
        assert _stage_launches(w, "xsyn_resolve") == 1
        assert _stage_launches(w, "xins_round") == 0
        assert "xfold" not in w.kernel_stats()  # no serial lane
    assert res.status[0] & abi.STATUS_ORPHAN


def test_large_list_orphans_and_non_lamport():
    """a list of 2^23 nodes with 2,000 orphans and 50 non-Lamport
    causes -- above the old serial fold's limit, where round 3 returned
    CW_STATUS_UNWOVEN -- bit-exact against the oracle's general fold."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 23) - 1, seed=34)
    rng = np.random.default_rng(34)
    off, idk, ck, kd = _nonlamport(spec, 1, [50], rng, orphans=[2000])
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_GENERAL,
                          yarns=False)
        w.set_profiling(False)
        rounds = _stage_launches(w, "xins_round")
        print(f"2^23 nodes, 2000 orphans, 50 non-Lamport: {rounds} rounds")
        assert 1 <= rounds <= 12
    assert res.status[0] & abi.STATUS_NON_LAMPORT and res.status[0] & abi.STATUS_ORPHAN


def _rank_docs(docs):
    """Model documents (par, cls on ranks, rank 0 the root) -> a packed batch:
    id = rank, cause = the cause's rank, NIL or an id no node has."""
    from cause_amd.pack import KeyLayout
    from tests import exact_model as M

    off, I, C, K = [0], [], [], []
    for par, cls in docs:
        n = len(par)
        for r in range(n):
            I.append(r)
            p = par[r]
            C.append((1 << 64) - 1 if p == M.NIL else (n + 7 if p == M.END else p))
            K.append(cls[r] | (4 if r == 0 else 0))
        off.append(len(I))
    return (np.array(off, np.uint64), np.array(I, np.uint64), np.array(C, np.uint64),
            np.array(K, np.uint8), KeyLayout(32, 0, 0))


def test_chain_families_few_rounds():
    """VERDICT r4 weak #2 on the GPU: chains of causes through younger nodes
    (tests/exact_model.py chain_doc: reverse, zigzag, interleaved, with
    specials and hides) in one batch with clean documents -- bit-exact
    against the literal fold, in at most 2 log2 n + 4 anchor rounds (round
    4's rule took n - 2 rounds on a reverse chain)."""
    import math

    from tests import exact_model as M

    n = 4000
    docs = [M.chain_doc(f, n, random.Random(k)) for k, f in enumerate(M.CHAIN_FAMILIES)]
    docs.insert(3, M.random_doc(random.Random(5), n))  # a clean neighbour
    off, idk, ck, kd, lay = _rank_docs(docs)
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, lay)
        w.set_profiling(False)
        rounds = _stage_launches(w, "xins_round")
        assert "xfold" not in w.kernel_stats()
    print(f"{len(docs)} documents of {n} nodes, {len(M.CHAIN_FAMILIES)} chain families: {rounds} rounds")
    assert 1 <= rounds <= 2 * math.log2(n) + 4
    assert res.status[3] == 0 and (res.status[[0, 1, 2, 4, 5, 6, 7]] & abi.STATUS_NON_LAMPORT).all()


def test_round_cap_hands_still_moving_documents_to_the_serial_fold(monkeypatch):
    """a small document still moving after the anchor-round cap
    leaves layout 2 for the serial literal fold (only -> run, any_serial; it
    is emitted with the synthetic lists, then overwritten by k_xfold).  With
    the cap at one round (CW_X_ROUND_CAP) every chain family takes that
    handoff: k_xfold runs and the batch is bit-exact against the literal fold,
    the clean neighbour included."""
    from tests import exact_model as M

    monkeypatch.setenv("CW_X_ROUND_CAP", "1")
    n = 1500
    docs = [M.chain_doc(f, n, random.Random(k)) for k, f in enumerate(M.CHAIN_FAMILIES)]
    docs.insert(2, M.random_doc(random.Random(9), n))
    off, idk, ck, kd, lay = _rank_docs(docs)
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck, kd, lay, method=oracle.METHOD_LITERAL)
        w.set_profiling(False)
        assert "xfold" in w.kernel_stats()
    assert res.status[2] == 0


def _with_reverse_chain(off, idk, ck, a, L):
    """Ranks [a, a + L) of the one document: rank r caused by rank r + 1 (the
    last keeps its cause) -- a reverse chain of L early nodes."""
    ck = ck.copy()
    srt = np.argsort(idk, kind="stable")
    for q in range(a, a + L - 1):
        ck[srt[q]] = idk[srt[q + 1]]
    return ck


def test_reverse_chain_in_config2_document():
    """a 2^18-node config-2-shaped document with a
    16,384-long reverse chain, bit-exact against the oracle's general fold
    (pinned to the literal fold by test_exact), in few rounds; its time next
    to the same document without the chain is printed for profiles/."""
    import json
    import math
    import os
    import time

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 18) - 1, seed=35)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=8)
    n = len(idk)
    ck2 = _with_reverse_chain(off, idk, ck, 1, 16_384)
    lay = spec.layout()
    times = {}
    with abi.Weaver(0) as w:
        for name, c in (("clean", ck), ("chain", ck2)):
            w.weave_lists(off, idk, c, kd, lay)  # warm
            t = []
            for _ in range(5):
                t0 = time.perf_counter()
                w.weave_lists(off, idk, c, kd, lay)
                t.append(time.perf_counter() - t0)
            times[name] = min(t) * 1e3
        w.reset_kernel_stats()
        w.set_profiling(True)
        res = check_batch(w, off, idk, ck2, kd, lay, method=oracle.METHOD_GENERAL)
        w.set_profiling(False)
        rounds = _stage_launches(w, "xins_round")
    rec = {"nodes": n, "chain": 16_384, "rounds": rounds, "clean_ms": round(times["clean"], 3),
           "chain_ms": round(times["chain"], 3), "ratio": round(times["chain"] / times["clean"], 2),
           "note": "host-memory cw_weave_lists, min of 5 (H2D + D2H included)"}
    print(json.dumps(rec))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/r5_reverse_chain.json", "w") as fh:
        fh.write(json.dumps(rec) + "\n")
    assert res.status[0] & abi.STATUS_NON_LAMPORT
    assert 1 <= rounds <= 2 * math.log2(n) + 4
