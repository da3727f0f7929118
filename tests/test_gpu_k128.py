"""K128 ids on the GPU (cw_weave_lists_k128): ids that do not fit 63 bits --
lamport-ts >= 2^40, 2^16 sites, tx-indices up to 2^32 -- weave bit-exact like
the reference (list.cljc:26-28 -> shared.cljc:225-241; the id order is
clojure.core/compare on [ts site tx], util.cljc:4-10).

The expected results come from the oracle's literal fold (METHOD_LITERAL) run
on an order-preserving renumbering of each document's ids made here on the host
from the Clojure-shaped nodes (sorted by causal_ref.id_key, the restated
compare), so the oracle sees small keys with exactly the same order and
equalities; ::lamport-ts and yarns are checked against the nodes directly.
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

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def weaver():
    with abi.Weaver(0) as w:
        yield w


def renumber(docs):
    """Order-preserving small keys per document (ids and id-causes ranked by
    the restated compare) as a K64 batch for the oracle."""
    off = np.zeros(len(docs) + 1, np.uint64)
    idk, ck, kd = [], [], []
    for d, nodes in enumerate(docs):
        ids = sorted({n[0] for n in nodes} | {n[1] for n in nodes if pack.is_id(n[1])},
                     key=R.id_key)
        rank = {i: r for r, i in enumerate(ids)}
        for nid, cause, value in nodes:
            idk.append(rank[nid])
            ck.append(pack.NIL if cause is None else
                      rank[cause] if pack.is_id(cause) else pack.NON_ID_CAUSE)
            k = pack.kind_of(value)
            if nid == R.ROOT_ID and cause is None and value is None:
                k |= pack.KIND_ROOT
            kd.append(k)
        off[d + 1] = len(idk)
    return off, np.array(idk, np.uint64), np.array(ck, np.uint64), np.array(kd, np.uint8)


def expected_yarns(nodes):
    """spin (shared.cljc:121-132): site by site (String.compareTo), id-ascending."""
    order = sorted(range(len(nodes)),
                   key=lambda j: (R.java_str_key(nodes[j][0][1]), R.id_key(nodes[j][0])))
    return np.array(order, np.uint32)


def check_k128(weaver, docs):
    b = pack.pack_lists_k128(docs)
    res = weaver.weave_lists_k128(b.offsets, b.id_key, b.cause_key, b.kind)
    off, idk, ck, kd = renumber(docs)
    assert np.array_equal(off, b.offsets)
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_LITERAL)
    assert np.array_equal(res.status, st), (res.status, st)
    gvis = res.visible()
    for d, nodes in enumerate(docs):
        lo, hi = int(off[d]), int(off[d + 1])
        if st[d] & abi.STATUS_DUP:
            continue
        assert np.array_equal(res.weave_perm[lo:hi], perm[lo:hi]), f"doc {d} order"
        assert np.array_equal(gvis[lo:hi], vis[lo:hi]), f"doc {d} visibility"
        assert res.visible_count[d] == int(vis[lo:hi].sum())
        if nodes:
            assert res.max_ts[d] == max(n[0][0] for n in nodes), f"doc {d} lamport-ts"
            assert np.array_equal(res.yarn_perm[lo:hi], expected_yarns(nodes)), f"doc {d} yarns"
    return res


def widen(nodes, rng, ts_base, nsites_extra=0):
    """The same history with every non-root ts moved up by ts_base, every site
    renamed order-preservingly to a site of the wide range, tx-indices scaled."""
    sites = sorted({i[1] for n in nodes for i in (n[0], n[1]) if pack.is_id(i)} - {"0"},
                   key=R.java_str_key)
    wide = sorted({R.new_site_id(rng) for _ in range(len(sites) + nsites_extra)},
                  key=R.java_str_key)
    while len(wide) < len(sites):
        wide = sorted(set(wide) | {R.new_site_id(rng)}, key=R.java_str_key)
    ren = dict(zip(sites, sorted(rng.sample(wide, len(sites)), key=R.java_str_key)))
    ren["0"] = "0"

    def w(i):
        if not pack.is_id(i) or i == R.ROOT_ID:
            return i
        return (i[0] + ts_base, ren[i[1]], i[2] * 65_537)

    return [(w(i), w(c), v) for i, c, v in nodes]


def test_k128_reference_histories(weaver):
    rng = random.Random(128)
    docs = []
    for ts_base in (1 << 40, (1 << 62) + 12345):
        for steps in (1, 5, 20, 60, 150):
            for _ in range(8):
                nodes, _ = G.random_history(rng, steps)
                d = widen([R.ROOT_NODE] + nodes, rng, ts_base)
                rng.shuffle(d)
                docs.append(d)
        for case in G.EDGE_CASES:
            docs.append(widen([R.ROOT_NODE] + list(case), rng, ts_base))
    check_k128(weaver, docs)


def test_k128_out_of_domain(weaver):
    """Orphans, non-Lamport causes, nil causes, no root, ids below the root and
    non-id causes in K128: the exact path, like K64."""
    rng = random.Random(129)
    docs = []
    for kinds in [(k,) for k in X.KINDS] + [X.KINDS]:
        for steps in (9, 40, 120):
            nodes, _ = G.random_history(rng, steps)
            d = X.corrupt(widen([R.ROOT_NODE] + nodes, rng, 1 << 41), rng, kinds, rate=0.2)
            rng.shuffle(d)
            docs.append(d)
    res = check_k128(weaver, docs)
    assert (res.status != 0).mean() > 0.8


def test_k128_2e16_sites_large_ts(weaver):
    """One document of 70,001 nodes from 65,536+ sites, lamport-ts >= 2^62,
    tx-indices near 2^32: the ids need 63 + 17 + 32 bits."""
    rng = random.Random(130)
    n = 70_000
    sites = sorted({R.new_site_id(rng) for _ in range(66_000)}, key=R.java_str_key)
    assert len(sites) >= 1 << 16
    base = 1 << 62
    nodes = [R.ROOT_NODE]
    ts = 0
    nonspecial = [R.ROOT_ID]
    for j in range(n):
        ts += rng.random() < 0.4
        site = sites[rng.randrange(len(sites))]
        tx = rng.randrange(1 << 32)
        nid = (base + ts + 1, site, tx)
        cause = rng.choice(nonspecial[-64:]) if rng.random() < 0.7 else rng.choice(nonspecial)
        # the cause must be older: ids of the same ts order by site/tx
        if not R.lt(cause, nid):
            cause = R.ROOT_ID
        r = rng.random()
        v = R.HIDE if r < 0.08 else R.H_SHOW if r < 0.1 else "x"
        nodes.append((nid, cause, v))
        if not R.is_special(v):
            nonspecial.append(nid)
    rng.shuffle(nodes)
    res = check_k128(weaver, [nodes])
    assert res.status[0] == 0


def test_k128_equals_k64_on_config2(weaver):
    """The same config-2 documents as K64 (cw_weave_lists) and as K128: every
    output identical (the two layouts order the ids the same way)."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=20_000)
    off, idk, ck, kd = gen.generate(spec, 0, 16)
    X.corrupt_packed  # (in-domain here; out-of-domain K128 is covered above)
    lay = spec.layout()
    r64 = weaver.weave_lists(off, idk, ck, kd, lay)

    def to128(k):
        k = k.astype(np.uint64)
        nil = k == np.uint64(pack.NIL)
        hi = k >> np.uint64(lay.ts_shift)
        site = (k >> np.uint64(lay.site_shift)) & np.uint64((1 << lay.site_bits) - 1)
        tx = k & np.uint64((1 << lay.tx_bits) - 1)
        lo = (site << np.uint64(32)) | tx
        out = np.stack([hi, lo], axis=1)
        out[nil] = np.uint64(pack.NIL)
        return out

    r128 = weaver.weave_lists_k128(off, to128(idk), to128(ck), kd)
    for f in ("weave_perm", "visible_bits", "visible_count", "max_ts", "status", "yarn_perm"):
        assert np.array_equal(getattr(r64, f), getattr(r128, f)), f


def test_k128_device_memory(weaver):
    import torch

    rng = random.Random(131)
    docs = []
    for steps in (3, 30, 90):
        nodes, _ = G.random_history(rng, steps)
        docs.append(widen([R.ROOT_NODE] + nodes, rng, 1 << 50))
    b = pack.pack_lists_k128(docs)
    want = weaver.weave_lists_k128(b.offsets, b.id_key, b.cause_key, b.kind)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)
    ti, tc, tk = t(b.id_key.reshape(-1)), t(b.cause_key.reshape(-1)), t(b.kind)
    N, D = len(b.kind), len(docs)
    outs = {"weave_perm": torch.zeros(N, dtype=torch.int32, device=dev),
            "visible_bits": torch.zeros((N + 31) // 32, dtype=torch.int32, device=dev),
            "visible_count": torch.zeros(D, dtype=torch.int32, device=dev),
            "max_ts": torch.zeros(D, dtype=torch.int64, device=dev),
            "status": torch.zeros(D, dtype=torch.int32, device=dev),
            "yarn_perm": torch.zeros(N, dtype=torch.int32, device=dev)}
    torch.cuda.synchronize()
    weaver.weave_lists_k128_device(b.offsets, ti.data_ptr(), tc.data_ptr(), tk.data_ptr(),
                                   {k: v.data_ptr() for k, v in outs.items()})
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in outs.items()}
    assert np.array_equal(got["weave_perm"].view(np.uint32), want.weave_perm)
    assert np.array_equal(got["visible_bits"].view(np.uint32), want.visible_bits)
    assert np.array_equal(got["visible_count"].view(np.uint32), want.visible_count)
    assert np.array_equal(got["max_ts"].view(np.uint64), want.max_ts)
    assert np.array_equal(got["status"].view(np.uint32), want.status)
    assert np.array_equal(got["yarn_perm"].view(np.uint32), want.yarn_perm)


def test_k128_empty_and_tiny(weaver):
    docs = [[], [R.ROOT_NODE], [R.ROOT_NODE, ((1 << 45, "aaaaaaaaaaaaa", 1 << 31), R.ROOT_ID, "x")]]
    res = check_k128(weaver, docs)
    assert list(res.status) == [abi.STATUS_ROOT, 0, 0]
    assert list(res.visible_count) == [0, 0, 1]


def test_key_range_status_k64(weaver):
    """A K64 batch whose keys reach 64 bits: the documents with an id >= 2^63
    get CW_STATUS_KEY_RANGE; the others weave as usual."""
    rng = random.Random(132)
    docs = []
    for steps in (5, 30):
        nodes, _ = G.random_history(rng, steps)
        docs.append([R.ROOT_NODE] + nodes)
    b = pack.pack_lists(docs)
    off, idk, ck, kd = b.offsets, b.id_key.copy(), b.cause_key.copy(), b.kind
    lo, hi = int(off[1]), int(off[2])
    top = np.uint64(1 << 63)
    j = lo + int(np.argmax(idk[lo:hi]))  # the largest id of doc 1: no node's cause
    idk[j] |= top
    res = weaver.weave_lists(off, idk, ck, kd, b.layout, key_bits=0)
    assert res.status[1] & abi.STATUS_KEY_RANGE
    assert not res.status[0] & abi.STATUS_KEY_RANGE
    perm, vis, st = oracle.batch_lists(off[:2], idk[:lo], ck[:lo], kd[:lo],
                                       method=oracle.METHOD_LITERAL)
    assert np.array_equal(res.weave_perm[:lo], perm)


def test_causal_mirror_takes_k128():
    """The host mirror packs ids over 63 bits as K128 on its own."""
    from cause_amd import causal as C

    rng = random.Random(133)
    nodes, _ = G.random_history(rng, 40)
    wide = widen([R.ROOT_NODE] + nodes, rng, (1 << 62) + 7)
    ct = C.new_list_ct()
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in wide}
    with pytest.raises(pack.KeyRangeError):
        pack.pack_lists([wide])
    out = C.refresh_caches(C.list_weave, ct)
    ref = R.new_list_ct()
    ref["nodes"] = {n[0]: (n[1], n[2]) for n in wide}
    ref = R.refresh_caches(R.list_weave, ref)
    assert out["weave"] == ref["weave"]
    assert C.causal_list_to_edn(out) == R.causal_list_to_edn(ref)
    assert out["lamport_ts"] == ref["lamport_ts"]
