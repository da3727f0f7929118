"""HIP weave vs the CPU oracle, bit-exact (run on the MI355X box: -m gpu).

Every call goes through the C ABI (cause_amd.abi -> libcauseweave.so).
Outputs compared: weave order (weave_perm), visibility (hide?, list.cljc:48-55),
visible count (list.cljc:77), ::lamport-ts (refresh-ts, shared.cljc:243-249),
yarns (spin, shared.cljc:121-132) and per-document status.
"""
import dataclasses
import random

import numpy as np
import pytest

import oracle
from oracle import causal_ref as R
from cause_amd import abi, gen, pack
from tests import refgen as G

pytestmark = pytest.mark.gpu


# Front ends: "front" = rank directories for every document (CW_FRONT_MIN_AVG=0
# also sends tiny documents through it; the whole weave of a document in one
# kernel, k_weave_doc, where it applies), "separate" = k_front, k_tree_l and
# k_tour as three kernels, "front3" = the three-kernel directory front end,
# "radix" = segmented radix sort + join.
FRONTS = {"front": {"CW_FRONT": "1", "CW_FRONT_MIN_AVG": "0"},
          "separate": {"CW_FRONT": "1", "CW_FRONT_MIN_AVG": "0", "CW_FUSED": "0"},
          "front3": {"CW_FRONT": "1", "CW_FRONT_MIN_AVG": "0", "CW_FRONT_FUSED": "0"},
          "radix": {"CW_FRONT": "0"},
          "radix-global": {"CW_FRONT": "0", "CW_PACK_SORT": "0"},  # no LDS pack sorts
          "hbm-walk": {"CW_TOUR": "0"},  # walk + rank + emit instead of the LDS tour
          "hbm-tree": {"CW_TREE_L": "0"}}  # k_tree, tables in HBM


@pytest.fixture(scope="module", params=sorted(FRONTS))
def weaver(request):
    import os

    old = {k: os.environ.get(k) for k in FRONTS[request.param]}
    os.environ.update(FRONTS[request.param])
    try:
        w = abi.Weaver(0)  # knobs are read when the context is created
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    with w:
        yield w


def oracle_batch(off, idk, ck, kd, layout, method=oracle.METHOD_LITERAL):
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=method)
    D = len(off) - 1
    vcount = np.array([int(vis[int(off[d]):int(off[d + 1])].sum()) for d in range(D)], np.uint32)
    max_ts = np.array([int(idk[int(off[d]):int(off[d + 1])].max() >> np.uint64(layout.ts_shift))
                       if off[d + 1] > off[d] else 0 for d in range(D)], np.uint64)
    return perm, vis, st, vcount, max_ts


def check_batch(weaver, off, idk, ck, kd, layout, method=oracle.METHOD_LITERAL, yarns=True):
    """Every document is compared, flagged ones too: the library reweaves
    documents outside the fast path's domain by the literal fold (exact.hip).
    Only documents with a repeated id (CW_STATUS_DUP, which the reference's
    ::nodes map cannot hold) have unspecified output."""
    res = weaver.weave_lists(off, idk, ck, kd, layout, yarns=yarns)
    perm, vis, st, vcount, max_ts = oracle_batch(off, idk, ck, kd, layout, method)
    ok = (st & abi.STATUS_DUP) == 0
    assert np.array_equal(res.status, st), (res.status, st)
    D = len(off) - 1
    gvis = res.visible()
    for d in np.nonzero(ok)[0]:
        b, e = int(off[d]), int(off[d + 1])
        assert np.array_equal(res.weave_perm[b:e], perm[b:e]), f"doc {d} order (status {st[d]})"
        assert np.array_equal(gvis[b:e], vis[b:e]), f"doc {d} visibility (status {st[d]})"
    assert np.array_equal(res.visible_count[ok], vcount[ok])
    ne = ok & (np.diff(off.astype(np.int64)) > 0)
    assert np.array_equal(res.max_ts[ne], max_ts[ne])
    if yarns and layout.site_bits:
        mask = (1 << layout.site_bits) - 1
        for d in np.nonzero(ok)[0]:
            b, e = int(off[d]), int(off[d + 1])
            want = oracle.list_yarns(idk[b:e], layout.site_shift, mask)
            assert np.array_equal(res.yarn_perm[b:e], want), f"doc {d} yarns"
    return res


def test_reference_edge_cases(weaver):
    docs = [[R.ROOT_NODE] + case for case in G.EDGE_CASES]
    rng = random.Random(1)
    for d in docs:
        rng.shuffle(d)
    b = pack.pack_lists(docs)
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


def test_reference_random_histories(weaver):
    rng = random.Random(42)
    docs = []
    for steps in (1, 2, 5, 9, 20, 60, 150):
        for _ in range(30):
            nodes, _ = G.random_history(rng, steps)
            d = [R.ROOT_NODE] + nodes
            rng.shuffle(d)
            docs.append(d)
    b = pack.pack_lists(docs)
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


def test_stress_histories(weaver):
    rng = random.Random(7)
    docs = []
    for n in (10, 100, 700):
        for p_special in (0.05, 0.3, 0.6):
            for tx_chain in (0.0, 0.3):
                d = G.stress_history(rng, n, p_special=p_special, p_conj=0.15,
                                     tx_chain=tx_chain)
                rng.shuffle(d)
                docs.append(d)
    b = pack.pack_lists(docs)
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


def test_tiny_and_empty_documents(weaver):
    docs = [[R.ROOT_NODE], [], [R.ROOT_NODE, ((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "x")],
            [R.ROOT_NODE, ((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, R.HIDE)]]
    b = pack.pack_lists(docs)
    res = weaver.weave_lists(b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    assert list(res.status) == [0, abi.STATUS_ROOT, 0, 0]
    assert list(res.visible_count) == [0, 0, 1, 0]
    assert list(res.weave_perm[:1]) == [0]


def test_out_of_domain_status(weaver):
    s = "aaaaaaaaaaaaa"
    docs = [
        [R.ROOT_NODE, ((1, s, 0), R.ROOT_ID, "x"), ((2, s, 0), (7, "bbbbbbbbbbbbb", 0), "y")],
        [R.ROOT_NODE, ((1, s, 0), (3, s, 0), "x"), ((3, s, 0), R.ROOT_ID, "y")],
        [((1, s, 0), R.ROOT_ID, "x")],
        [R.ROOT_NODE, ((1, s, 0), R.ROOT_ID, "x"), ((1, s, 0), R.ROOT_ID, "x")],
        [R.ROOT_NODE, ((1, s, 0), R.ROOT_ID, "x")],
    ]
    b = pack.pack_lists(docs)
    res = weaver.weave_lists(b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    assert res.status[0] & abi.STATUS_ORPHAN
    assert res.status[1] & abi.STATUS_NON_LAMPORT
    assert res.status[2] & abi.STATUS_ROOT
    assert res.status[3] & abi.STATUS_DUP
    assert res.status[4] == 0
    # the flagged documents (except the DUP one) are the reference's literal fold
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


def test_generated_config2_shape(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=5000)
    off, idk, ck, kd = gen.generate(spec, 0, 120)
    check_batch(weaver, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF)


def test_yarns_every_site_value(weaver):
    """k_yarn_doc's multisplit over the widest site field it takes (4 bits:
    the root's site 0 and sites 1..15, every one of the 16 classes in use),
    documents of the fused weave's sizes, yarn_perm against the oracle."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=20_000, n_sites=15, seed=77)
    assert spec.layout().site_bits == 4
    off, idk, ck, kd = gen.generate(spec, 0, 24)
    check_batch(weaver, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF)


def test_generated_mixed_sizes(weaver):
    """Documents spanning many sort tiles and many splitter blocks, plus
    tiny ones, in one batch."""
    parts = []
    for n, D, seed in ((3, 50, 1), (4095, 3, 2), (4097, 3, 3), (70_000, 2, 4), (17, 40, 5)):
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n, seed=seed)
        parts.append(gen.generate(spec, 0, D))
    lay = pack.KeyLayout(17, 4, 0)
    sizes = np.concatenate([np.diff(p[0]) for p in parts])
    off = np.zeros(len(sizes) + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    idk = np.concatenate([p[1] for p in parts])
    ck = np.concatenate([p[2] for p in parts])
    kd = np.concatenate([p[3] for p in parts])
    ck = np.where(ck == np.uint64(pack.NIL), ck, ck)  # same layout (site_bits 4)
    check_batch(weaver, off, idk, ck, kd, lay, method=oracle.METHOD_EFF)


def test_config1_single_large_list(weaver):
    off, idk, ck, kd = gen.generate(gen.CONFIG1, 0, 1)
    check_batch(weaver, off, idk, ck, kd, gen.CONFIG1.layout(), method=oracle.METHOD_LINKED)


def test_typing_chain_depth(weaver):
    """One site typing 200k characters in a row: the effective tree is a
    single chain of depth n (the Euler walk must not depend on depth)."""
    spec = dataclasses.replace(gen.CONFIG1, nodes_per_doc=200_000, n_sites=1, p_chain=1.0,
                               shuffle=True)
    off, idk, ck, kd = gen.generate(spec, 0, 1)
    check_batch(weaver, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_LINKED)


def test_all_caused_by_root(weaver):
    """cons- shape (list.cljc:42-43): every node caused by the root."""
    s = "aaaaaaaaaaaaa"
    doc = [R.ROOT_NODE] + [((t, s, 0), R.ROOT_ID, "c") for t in range(1, 30_001)]
    random.Random(3).shuffle(doc)
    b = pack.pack_lists([doc])
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout,
                method=oracle.METHOD_LINKED)


def _sibling_group_doc(rng, n, sizes):
    """Runs of g consecutive ids caused by one earlier node, g drawn from
    ``sizes``: sibling groups of every size around k_tree_l's per-tile hash
    list limit (16) and across its tile boundaries, with hides and shows
    among them so both classes form groups."""
    s = "aaaaaaaaaaaaa"
    doc = [R.ROOT_NODE]
    normal = [R.ROOT_ID]
    t = 1
    while t < n:
        g = rng.choice(sizes)
        parent = rng.choice(normal[-64:] if rng.random() < 0.5 else normal)
        for _ in range(g):
            if t >= n:
                break
            nid = (t, s, 0)
            u = rng.random()
            if u < 0.15 and parent != R.ROOT_ID:
                doc.append((nid, parent, R.HIDE))
            elif u < 0.2 and parent != R.ROOT_ID:
                doc.append((nid, parent, R.H_SHOW))
            else:
                doc.append((nid, parent, "x"))
                normal.append(nid)
            t += 1
    rng.shuffle(doc)
    return doc


def test_sibling_groups_of_every_size(weaver):
    rng = random.Random(11)
    docs = [_sibling_group_doc(rng, n, sizes)
            for n, sizes in ((5000, (1, 2, 3)), (9000, (15, 16, 17, 18)), (12_000, (1, 2, 40, 100)),
                             (3000, (2047, 2048, 2049)), (20_000, (1, 1, 1, 5, 16, 33)))]
    b = pack.pack_lists(docs)
    check_batch(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout,
                method=oracle.METHOD_LINKED)


def test_repeat_calls_are_identical(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000)
    off, idk, ck, kd = gen.generate(spec, 0, 30)
    a = weaver.weave_lists(off, idk, ck, kd, spec.layout())
    b = weaver.weave_lists(off, idk, ck, kd, spec.layout())
    assert np.array_equal(a.weave_perm, b.weave_perm)
    assert np.array_equal(a.visible_bits, b.visible_bits)


def test_key_bits_found_on_device(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000)
    off, idk, ck, kd = gen.generate(spec, 0, 10)
    a = weaver.weave_lists(off, idk, ck, kd, spec.layout())
    b = weaver.weave_lists(off, idk, ck, kd, spec.layout(), key_bits=0)
    assert np.array_equal(a.weave_perm, b.weave_perm)


def test_sparse_document_falls_back(weaver):
    """A document whose ids are too sparse for a rank-directory slot (ts gaps
    of 2^20) sends the whole batch through the radix front end."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000)
    off, idk, ck, kd = gen.generate(spec, 0, 6)
    lay = spec.layout()
    b, e = int(off[2]), int(off[3])
    sh = np.uint64(lay.ts_shift)
    stretch = lambda k: np.where(k == np.uint64(pack.NIL), k,
                                 ((k >> sh) * np.uint64(1 << 20) << sh) | (k & ((np.uint64(1) << sh) - np.uint64(1))))
    idk, ck = idk.copy(), ck.copy()
    idk[b:e], ck[b:e] = stretch(idk[b:e]), stretch(ck[b:e])
    wide = pack.KeyLayout(lay.ts_bits + 20, lay.site_bits, lay.tx_bits)
    check_batch(weaver, off, idk, ck, kd, wide, method=oracle.METHOD_EFF)


def test_duplicate_ids_beside_clean_documents(weaver):
    """A duplicated id (shared.cljc:166-171) flags its document only; the
    documents around it still weave exactly."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000)
    off, idk, ck, kd = gen.generate(spec, 0, 5)
    idk = idk.copy()
    b = int(off[1])
    idk[b + 10] = idk[b + 11] if idk[b + 11] != idk[b] else idk[b + 12]
    res = weaver.weave_lists(off, idk, ck, kd, spec.layout())
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    assert res.status[1] & abi.STATUS_DUP and st[1] & abi.STATUS_DUP
    assert not res.status[[0, 2, 3, 4]].any()
    gvis = res.visible()
    for d in (0, 2, 3, 4):
        b, e = int(off[d]), int(off[d + 1])
        assert np.array_equal(res.weave_perm[b:e], perm[b:e])
        assert np.array_equal(gvis[b:e], vis[b:e])


# walk / slot geometry only matters on the HBM walk path (CW_TOUR=0); the
# fused LDS tour takes its own splitter density (CW_TOUR_LOG2K)
_W = {"CW_TOUR": "0"}
KNOBS = [{}, dict(_W),
         {"CW_TOUR_LOG2K": "3"}, {"CW_TOUR_LOG2K": "4"}, {"CW_TOUR_LOG2K": "7"},
         {"CW_FRONT": "0"}, {"CW_FRONT_SLOT": "4096"},
         # the tree: k_tree (tables in HBM, the fallback for documents too large
         # for k_tree_l's LDS), k_tree_l with 1,024-rank tiles, the separate kernels
         {"CW_TREE_L": "0"}, {"CW_TREE_L": "1024"}, {"CW_FUSED": "0"}]


@pytest.mark.parametrize("n", [59_204, 60_000, 65_534, 65_535])
def test_tour_document_size_limits(n):
    """Documents at the fused tour's limits: the splitter blocks grow so the
    LDS tables fit (n = 65,535 is the largest u16 document; 65,536 nodes with
    the root go through the HBM walk)."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n - 1)
    off, idk, ck, kd = gen.generate(spec, 0, 3)
    with abi.Weaver(0) as w:
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF, yarns=False)
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n)
    off, idk, ck, kd = gen.generate(spec, 0, 2)
    with abi.Weaver(0) as w:
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF, yarns=False)


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()) or "default")
def test_config2_documents_any_geometry(knobs, monkeypatch):
    """Full-size config-2 documents (50,001 nodes) under every launch geometry
    knob: the output must not depend on splitter density, slot size, digit
    width or walker grouping."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    spec = gen.CONFIG2
    off, idk, ck, kd = gen.generate(spec, 0, 24)
    with abi.Weaver(0) as w:
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF, yarns=False)


@pytest.mark.parametrize("knobs", [{}, {"CW_FUSED": "0"}, {"CW_TOUR": "0"}],
                         ids=["default", "separate", "hbm-walk"])
def test_full_bench_batch_vs_oracle(knobs, monkeypatch):
    """The whole bench workload (10,000 config-2 documents, 5e8 nodes) against
    the oracle, every document, plus permutation validity."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    spec = gen.CONFIG2
    off, idk, ck, kd = gen.generate(spec, 0, 10_000, nthreads=32)
    with abi.Weaver(0) as w:
        res = w.weave_lists(off, idk, ck, kd, spec.layout(), yarns=False)
    assert not res.status.any(), np.nonzero(res.status)[0][:10]
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=32)
    assert not st.any()
    bad = [d for d in range(10_000)
           if not np.array_equal(res.weave_perm[int(off[d]):int(off[d + 1])],
                                 perm[int(off[d]):int(off[d + 1])])]
    if bad:
        d = bad[0]
        b, e = int(off[d]), int(off[d + 1])
        g, o = res.weave_perm[b:e], perm[b:e]
        lk, _ = oracle.list_weave(idk[b:e], ck[b:e], kd[b:e], oracle.METHOD_LINKED)
        diff = np.nonzero(g != o)[0]
        raise AssertionError(
            f"{len(bad)} documents differ, first {bad[:5]}; doc {d}: {len(diff)} positions, "
            f"first {diff[:4]}, gpu {g[diff[:4]]}, oracle {o[diff[:4]]}, gpu==linked "
            f"{np.array_equal(g, lk)}, oracle==linked {np.array_equal(o, lk)}, gpu is a perm "
            f"{len(np.unique(g)) == e - b}")
    assert np.array_equal(res.visible(), vis)


# ------------------------------------------------- one giant document (config 5)
# Giant-path front ends: the directory over the whole key range
# (k_gd_place, small key ranges: the default here), the sorted-id directory
# join (CW_GDIR=0: k_gd_build / k_gpack / k_gjoin, config 5's default) and
# the bucket index + searching join (CW_GJOIN=0).
GIANT_FRONTS = {"gdplace": {}, "gjoin": {"CW_GDIR": "0"},
                "bucket": {"CW_GDIR": "0", "CW_GJOIN": "0"},
                # the tile-local sibling links (k_glocal) at every size
                "glocal": {"CW_GDIR": "0", "CW_GLOCAL_MIN": "0"}}


def _weaver_with(env):
    import os

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return abi.Weaver(0)  # knobs are read when the context is created
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=sorted(GIANT_FRONTS))
def giant_weaver(request):
    """A context that sends every one-document batch through the giant-document
    tree (k_geff / radix sort / k_gsib / k_gthr + the walk's thread chase),
    under each giant front end."""
    with _weaver_with(dict(GIANT_FRONTS[request.param], CW_GIANT_MIN="0")) as w:
        yield w


def test_giant_path_small_documents(giant_weaver):
    """The reference's edge cases, random and stress histories, one per call."""
    rng = random.Random(31)
    docs = [[R.ROOT_NODE] + case for case in G.EDGE_CASES]
    for steps in (1, 9, 60, 300):
        for _ in range(3):
            nodes, _ = G.random_history(rng, steps)
            docs.append([R.ROOT_NODE] + nodes)
    for steps, tx in ((200, 0.0), (2000, 0.0), (1500, 0.3)):
        docs.append(G.stress_history(rng, steps, tx_chain=tx))
    docs.append([R.ROOT_NODE])
    # out of the fast path's domain: absent, younger and nil causes, no root,
    # a repeated id (its output is unspecified, its status is not)
    from tests import outdomain as X

    for kinds in [("orphan",), ("non_lamport",), ("nil_cause",), ("no_root",), X.KINDS]:
        nodes = G.stress_history(rng, 400, p_special=0.3)
        docs.append(X.corrupt(nodes, rng, kinds, rate=0.03))
    nodes = G.stress_history(rng, 300)
    docs.append(nodes + [nodes[7]])
    for d in docs:
        rng.shuffle(d)
        b = pack.pack_lists([d])
        check_batch(giant_weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)


@pytest.mark.parametrize("target_bits", [0, 31, 32, 33, 40, 43, 44])
def test_id_sort_carried_cause_key_widths(target_bits):
    """The id sort's carried cause and kind (round 6, onesweep.hip OsPayload:
    the cause's low 32 bits beside the index, its high bits and the kind above
    the key bits) at key widths either side of 32 and up to OS_PL_MAX_BITS = 43
    (44 takes the join that gathers by input index): one 150k-node list, ids
    and causes shifted left into a wider tx field (order and layout kept), with
    orphan causes (one past an id, one past the largest id) and a nil cause --
    the exact path then reweaves it -- against the oracle's general fold."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=150_000, seed=57)
    off, idk, ck, kd = gen.generate(spec, 0, 1)
    lay0 = spec.layout()
    shift = max(0, target_bits - lay0.key_bits)
    lay = pack.KeyLayout(lay0.ts_bits, lay0.site_bits, lay0.tx_bits + shift)
    nil = ck == np.uint64(pack.NIL)
    idk = idk << np.uint64(shift)
    ck = ck << np.uint64(shift)
    ck[nil] = np.uint64(pack.NIL)
    rng = np.random.default_rng(target_bits)
    some = rng.choice(np.arange(1, len(ck)), 40, replace=False)
    ck[some[:20]] = idk[some[:20]] + np.uint64(1)           # (1 << shift > 1: not an id)
    ck[some[20:39]] = idk.max() + np.uint64(1 << shift)      # past the largest id
    ck[some[39]] = np.uint64(pack.NIL)
    assert lay.key_bits == max(lay0.key_bits, target_bits)
    with _weaver_with({"CW_GDIR": "0", "CW_GIANT_MIN": "0"}) as w:
        res = check_batch(w, off, idk, ck, kd, lay, method=oracle.METHOD_GENERAL, yarns=False)
    assert res.status[0] & abi.STATUS_ORPHAN


def test_giant_join_misdeclared_key_bits():
    """ids wider than the declared key_bits on the sorted-id directory join
    (ADVICE r3): the directory is never read past its end, the list is flagged
    INTERNAL instead of faulting."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=100_000, seed=41)
    off, idk, ck, kd = gen.generate(spec, 0, 1)
    lay = spec.layout()
    with _weaver_with({"CW_GDIR": "0", "CW_GIANT_MIN": "0"}) as w:
        res = w.weave_lists(off, idk, ck, kd, lay, key_bits=max(1, lay.key_bits - 6))
        assert res.status[0] & abi.STATUS_INTERNAL
        again = w.weave_lists(off, idk, ck, kd, lay)  # the context still works
        assert again.status[0] == 0


def test_giant_path_shapes(giant_weaver):
    """Config 1, a deep typing chain (threads chased across every tile) and a
    root with 30k children."""
    off, idk, ck, kd = gen.generate(gen.CONFIG1, 0, 1)
    check_batch(giant_weaver, off, idk, ck, kd, gen.CONFIG1.layout(), method=oracle.METHOD_LINKED)
    spec = dataclasses.replace(gen.CONFIG1, nodes_per_doc=200_000, n_sites=1, p_chain=1.0)
    off, idk, ck, kd = gen.generate(spec, 0, 1)
    check_batch(giant_weaver, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_LINKED)
    s = "aaaaaaaaaaaaa"
    doc = [R.ROOT_NODE] + [((t, s, 0), R.ROOT_ID, "c") for t in range(1, 30_001)]
    random.Random(3).shuffle(doc)
    b = pack.pack_lists([doc])
    check_batch(giant_weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout,
                method=oracle.METHOD_LINKED)


@pytest.mark.parametrize("log2k", ["3", "5"])
def test_giant_path_splitter_blocks(log2k, monkeypatch):
    """The giant path under other splitter blocks than its default 16 nodes
    (CW_GIANT_LOG2K, lists of >= 2^22 nodes): 8 (the round-2 geometry) and 32."""
    monkeypatch.setenv("CW_GIANT_MIN", "0")
    monkeypatch.setenv("CW_GIANT_LOG2K", log2k)
    rng = random.Random(7)
    with abi.Weaver(0) as w:
        for steps, tx in ((2000, 0.0), (1500, 0.3)):
            d = G.stress_history(rng, steps, tx_chain=tx)
            rng.shuffle(d)
            b = pack.pack_lists([d])
            check_batch(w, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
        spec = dataclasses.replace(gen.CONFIG1, nodes_per_doc=200_000, n_sites=1, p_chain=1.0)
        off, idk, ck, kd = gen.generate(spec, 0, 1)
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_LINKED)
        # (the knob applies from 2^22 nodes: smaller lists keep 8-node blocks)
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 22) + 1000)
        off, idk, ck, kd = gen.generate(spec, 0, 1)
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF, yarns=False)


def test_giant_path_many_continuation_sublists(monkeypatch):
    """4-entry walk slots (CW_GIANT_LOG2CAP = 2, which sets the giant slot
    size itself, below the library's 16-entry minimum): every walk goes on
    through several continuation sublists, so the first ranking level's
    walkers pass more sublists than their 32-entry slots hold and the rest
    take the overflow path (pos + the overflow list).  The walk's
    continued-sublist counter proves the overflows happened."""
    monkeypatch.setenv("CW_GIANT_MIN", "0")
    monkeypatch.setenv("CW_GIANT_LOG2CAP", "2")
    with abi.Weaver(0) as w:
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 22) + 1000)
        off, idk, ck, kd = gen.generate(spec, 0, 1)
        check_batch(w, off, idk, ck, kd, spec.layout(), method=oracle.METHOD_EFF, yarns=False)
        cont = w.counter("continued_sublists")
        # 16-node splitter blocks in 4-entry slots: most sublists continue
        assert cont > len(idk) // 16, cont
        off, idk, ck, kd = gen.generate(gen.CONFIG1, 0, 1)
        check_batch(w, off, idk, ck, kd, gen.CONFIG1.layout(), method=oracle.METHOD_LINKED)
        assert w.counter("continued_sublists") > 0
    monkeypatch.setenv("CW_GIANT_LOG2CAP", "5")
    with abi.Weaver(0) as w:  # the default 32-entry slots overflow far less often
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=(1 << 22) + 1000)
        off, idk, ck, kd = gen.generate(spec, 0, 1)
        w.weave_lists(off, idk, ck, kd, spec.layout())
        assert w.counter("continued_sublists") < cont // 4


def test_few_large_documents_per_document_giant_path():
    """A batch of a few large documents goes through the giant path one
    document at a time (render bits merged at unaligned offsets); a small one
    in the middle and an empty one too."""
    docs = []
    for n, seed in ((150_000, 1), (70_001, 2), (3_000, 3), (90_000, 4)):
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n, seed=seed)
        off, idk, ck, kd = gen.generate(spec, 0, 1)
        docs.append((idk, ck, kd))
    off = np.zeros(len(docs) + 2, np.uint64)
    for i, (idk, _, _) in enumerate(docs):
        off[i + 1] = off[i] + len(idk)
    off[-1] = off[-2]  # an empty document at the end
    idk = np.concatenate([d[0] for d in docs])
    ck = np.concatenate([d[1] for d in docs])
    kd = np.concatenate([d[2] for d in docs])
    lay = dataclasses.replace(gen.CONFIG2, nodes_per_doc=150_000).layout()
    with abi.Weaver(0) as w:
        res = w.weave_lists(off, idk, ck, kd, lay)
    perm, vis, st, vcount, max_ts = oracle_batch(off, idk, ck, kd, lay, oracle.METHOD_LINKED)
    D = len(off) - 1
    assert res.status[-1] & abi.STATUS_ROOT
    assert not res.status[:-1].any()
    for d in range(D - 1):
        b, e = int(off[d]), int(off[d + 1])
        assert np.array_equal(res.weave_perm[b:e], perm[b:e]), d
    assert np.array_equal(res.visible(), vis.astype(bool))
    assert np.array_equal(res.visible_count[:-1], vcount[:-1])
    assert np.array_equal(res.max_ts[:-1], max_ts[:-1])


def test_giant_document_default_threshold(weaver):
    """A 3M-node config-2-shaped list: over the default threshold, so the giant
    tree, the chunked radix scan and the flat bucket index all run."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3_000_000)
    off, idk, ck, kd = gen.generate(spec, 0, 1)
    lay = spec.layout()
    check_batch(weaver, off, idk, ck, kd, lay, method=oracle.METHOD_EFF, yarns=False)
