"""GPU merge (cw_merge_lists) vs the CPU oracle, bit-exact (-m gpu).

s/merge-trees (shared.cljc:300-314) and bulk s/insert (:151-184) equal the full
reweave of the union of the two node bags; duplicates with equal
bodies are kept once (insert's idempotency, :164-165), unequal bodies flag
CW_STATUS_DUP (:166-171), causes missing from the union flag CW_STATUS_ORPHAN
(:175-178).
"""
import dataclasses
import random

import numpy as np
import pytest

import oracle
from cause_amd import abi, causal, gen, pack
from oracle import causal_ref as R
from tests import refgen as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def weaver():
    with abi.Weaver(0) as w:
        yield w


def split_batch(off, idk, ck, kd, rng, overlap=0.2, drop_b=0.0):
    """Each document's nodes -> two overlapping random subsets a, b whose union
    is the document (value token = input index, so equal ids have equal bodies)."""
    A, B = [], []
    for d in range(len(off) - 1):
        lo, hi = int(off[d]), int(off[d + 1])
        idx = np.arange(lo, hi)
        rng.shuffle(idx)
        n = hi - lo
        cut = -(-n * (50 + int(overlap * 50)) // 100)  # ceil: the union is the document
        A.append(idx[:cut])
        B.append(idx[n - cut:] if n > 1 else idx[:0])
    def side(parts):
        o = np.zeros(len(parts) + 1, np.uint64)
        o[1:] = np.cumsum([len(p) for p in parts])
        cat = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        return (o, idk[cat], ck[cat], kd[cat], cat.astype(np.uint64)), cat
    return side(A), side(B)


def check_merge(weaver, off, idk, ck, kd, layout, rng, **kw):
    (a, ia), (b, ib) = split_batch(off, idk, ck, kd, rng, **kw)
    res = weaver.merge_lists(a, b, layout)
    assert not res.weave.status.any(), res.weave.status
    D = len(off) - 1
    assert np.array_equal(np.diff(res.offsets), np.diff(off).astype(np.uint64))
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    assert not st.any()
    wsrc = res.weave_src()
    gvis = res.weave.visible()
    for d in range(D):
        lo, hi = int(off[d]), int(off[d + 1])
        na = int(a[0][d + 1] - a[0][d])
        sa, sb = ia[int(a[0][d]):int(a[0][d + 1])], ib[int(b[0][d]):int(b[0][d + 1])]
        glob = np.array([sa[s] if s < na else sb[s - na] for s in wsrc[lo:hi]], np.int64)
        assert np.array_equal(glob - lo, perm[lo:hi].astype(np.int64)), f"doc {d} order"
        assert np.array_equal(gvis[lo:hi], vis[lo:hi]), f"doc {d} visibility"
        # merged nodes come out in id order
        ids = idk[np.array([sa[s] if s < na else sb[s - na] for s in res.src[lo:hi]], np.int64)]
        assert np.all(ids[1:] > ids[:-1])
    return res


def test_merge_generated_documents(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=4000)
    off, idk, ck, kd = gen.generate(spec, 0, 40)
    check_merge(weaver, off, idk, ck, kd, spec.layout(), np.random.default_rng(1))


def test_merge_disjoint_and_full_overlap(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000)
    off, idk, ck, kd = gen.generate(spec, 0, 10)
    for ov in (0.0, 1.0):
        check_merge(weaver, off, idk, ck, kd, spec.layout(), np.random.default_rng(2), overlap=ov)


def test_merge_reference_histories(weaver):
    rng = random.Random(5)
    docs = []
    for steps in (1, 9, 30, 120):
        for _ in range(5):
            nodes, _ = G.random_history(rng, steps)
            docs.append([R.ROOT_NODE] + nodes)
    b = pack.pack_lists(docs)
    check_merge(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout,
                np.random.default_rng(3))


def test_merge_with_itself_is_identity(weaver):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=2000)
    off, idk, ck, kd = gen.generate(spec, 0, 6)
    v = np.arange(len(idk), dtype=np.uint64)
    res = weaver.merge_lists((off, idk, ck, kd, v), (off, idk, ck, kd, v), spec.layout())
    assert not res.weave.status.any()
    plain = weaver.weave_lists(off, idk, ck, kd, spec.layout())
    assert np.array_equal(res.offsets, off)
    # every node kept once, from a (its first occurrence)
    sizes = np.diff(off).astype(np.int64)
    assert np.all(res.src < np.repeat(sizes, sizes))
    assert np.array_equal(res.weave_src(), plain.weave_perm)
    assert np.array_equal(res.weave.visible_bits[:len(plain.visible_bits)], plain.visible_bits)


def test_merge_conflict_and_orphan_status(weaver):
    s = "aaaaaaaaaaaaa"
    root = R.ROOT_NODE
    x1 = ((1, s, 0), R.ROOT_ID, "x")
    x1b = ((1, s, 0), R.ROOT_ID, "y")          # same id, other value
    y2 = ((2, s, 0), (1, s, 0), "z")
    orphan = ((3, s, 0), (9, "bbbbbbbbbbbbb", 0), "o")
    docs_a = [[root, x1], [root, x1], [root, x1], []]
    docs_b = [[x1b], [y2, orphan], [x1, y2], []]
    b = pack.pack_lists([a + bb for a, bb in zip(docs_a, docs_b)])
    tok = {}
    vals = np.array([tok.setdefault(n[2], len(tok)) for d in b.docs for n in d.nodes], np.uint64)
    ia, ib = [], []
    for d, (a, bb) in enumerate(zip(docs_a, docs_b)):
        lo = int(b.offsets[d])
        ia += range(lo, lo + len(a))
        ib += range(lo + len(a), lo + len(a) + len(bb))
    ia, ib = np.array(ia, np.int64), np.array(ib, np.int64)
    oa = np.concatenate([[0], np.cumsum([len(a) for a in docs_a])]).astype(np.uint64)
    ob = np.concatenate([[0], np.cumsum([len(x) for x in docs_b])]).astype(np.uint64)
    res = weaver.merge_lists((oa, b.id_key[ia], b.cause_key[ia], b.kind[ia], vals[ia]),
                             (ob, b.id_key[ib], b.cause_key[ib], b.kind[ib], vals[ib]), b.layout)
    st = res.weave.status
    assert st[0] & abi.STATUS_DUP
    assert st[1] & abi.STATUS_ORPHAN and not st[1] & abi.STATUS_DUP
    assert st[2] == 0 and list(np.diff(res.offsets)) == [2, 4, 3, 0]
    assert st[3] & abi.STATUS_ROOT


# ------------------------------------------------------------- host mirror ----
def _ct(nodes, like=None):
    ct = causal.new_list_ct(uuid=like["uuid"] if like else None, rng=random.Random(9))
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in [R.ROOT_NODE] + nodes}
    return causal.refresh_caches(causal.list_weave, ct)


def closure(all_nodes, some):
    """some plus every cause they need (a replica always holds whole causal pasts)."""
    by_id = {n[0]: n for n in all_nodes}
    keep = {n[0] for n in some}
    todo = list(keep)
    while todo:
        c = by_id[todo.pop()][1]
        if c in by_id and c not in keep:
            keep.add(c)
            todo.append(c)
    return [n for n in all_nodes if n[0] in keep]


def test_mirror_merge_trees_equals_incremental_inserts():
    """list_test.cljc:44-96 shape: the reference's edge cases split across two
    replicas and merged == inserting every node into one tree."""
    rng = random.Random(11)
    for case in G.EDGE_CASES:
        for _ in range(3):
            nodes = list(case)
            rng.shuffle(nodes)
            k = rng.randrange(len(nodes) + 1)
            ct1 = _ct(closure(case, nodes[:k]))
            ct2 = _ct(closure(case, nodes[k:]), like=ct1)
            m = causal.merge_trees(causal.list_weave, ct1, ct2)
            full = _ct(list(case), like=ct1)
            assert m["weave"] == full["weave"]
            assert causal.causal_list_to_edn(m) == causal.causal_list_to_edn(full)
            assert m["yarns"] == full["yarns"]


def test_mirror_merge_errors():
    ct1 = _ct([((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "x")])
    ct2 = _ct([((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "y")], like=ct1)
    with pytest.raises(causal.CauseError) as e:
        causal.merge_trees(causal.list_weave, ct1, ct2)
    assert e.value.causes == {"append-only", "edits-not-allowed"}
    other = dict(_ct([]), uuid="another-uuid-00000000")
    with pytest.raises(causal.CauseError) as e:
        causal.merge_trees(causal.list_weave, ct1, other)
    assert e.value.causes == {"uuid-missmatch"}


def test_mirror_insert_bulk_matches_refresh():
    rng = random.Random(13)
    nodes, _ = G.random_history(rng, 80)
    ct = _ct(nodes[:30])
    bulk = causal.insert_bulk(ct, nodes[30:])
    full = _ct(nodes, like=ct)
    assert bulk["weave"] == full["weave"]
    assert bulk["lamport_ts"] == max(n[0][0] for n in nodes)


# -------------------------------------------------------------------- weft ----
def _weft_ref(ct, ids):
    nct = lambda: R.new_list_ct(site_id=ct["site_id"], uuid=ct["uuid"])
    return R.weft(R.list_weave, nct, ct, ids)


def _ref_ct(nodes, rng):
    ct = R.new_list_ct(rng=rng)
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in [R.ROOT_NODE] + nodes}
    return R.refresh_caches(R.list_weave, ct)


def test_weft_matches_reference_restatement():
    """shared.cljc:268-293: cut every site's yarn at a random node, at an id
    that is no node, or drop the site; name sites with no node at all; weave;
    compare with the restatement -- causally closed cuts and the reference's
    "gibberish trees" alike (the library's exact path weaves those)."""
    rng = random.Random(21)
    checked = gibberish = bogus = 0
    for steps in (5, 20, 60, 150):
        for _ in range(25):
            nodes, _ = G.random_history(rng, steps)
            ref = _ref_ct(nodes, rng)
            sites = sorted({n[0][1] for n in nodes})
            ids = []
            T = rng.randint(1, max(n[0][0] for n in nodes))
            for s in sites:
                r = rng.random()
                if r < 0.2:
                    ids.append(rng.choice(ref["yarns"][s])[0])  # arbitrary cut
                elif r < 0.3:
                    ids.append((rng.randint(1, T + 3), s, 7))     # no such node
                elif r < 0.9:  # consistent cut: the site's state at time T
                    older = [n for n in ref["yarns"][s] if n[0][0] <= T]
                    if older:
                        ids.append(older[-1][0])
            if rng.random() < 0.2:
                ids.append((T, R.new_site_id(rng), 0))            # a site with no node
            if not ids:
                continue
            want = _weft_ref(ref, ids)
            kept = set(want["nodes"])
            gibberish += any(len(b) > 1 and b[0] is not None and b[0] not in kept
                             for b in want["nodes"].values())
            bogus += any(len(b) == 0 for b in want["nodes"].values())
            ct = causal.new_list_ct(site_id=ref["site_id"], uuid=ref["uuid"])
            ct["nodes"] = dict(ref["nodes"])
            got = causal.weft(ct, ids)
            assert got["weave"] == want["weave"]
            assert causal.causal_list_to_edn(got) == R.causal_list_to_edn(want)
            assert got["lamport_ts"] == want["lamport_ts"]
            assert got["nodes"] == want["nodes"]
            assert got["yarns"] == want["yarns"]
            checked += 1
    assert checked > 60 and gibberish > 5 and bogus > 5, (checked, gibberish, bogus)


def test_weft_status_bits(weaver):
    """A cut id that is not a node: CW_STATUS_WEFT; a cut that drops a cause:
    CW_STATUS_ORPHAN."""
    s1, s2 = "aaaaaaaaaaaaa", "bbbbbbbbbbbbb"
    a1 = ((1, s1, 0), R.ROOT_ID, "x")
    b2 = ((2, s2, 0), (1, s1, 0), "y")
    doc = [R.ROOT_NODE, a1, b2]
    b = pack.pack_lists([doc, doc, doc], min_site_bits=1)
    lay, S = b.layout, 1 << b.layout.site_bits
    rk = b.docs[0].site_rank
    cut = np.zeros(3 * S, np.uint64)
    cut[0 * S + rk[s1]] = lay.pack(1, rk[s1], 0)          # s1 only: fine
    cut[1 * S + rk[s1]] = lay.pack(5, rk[s1], 0)          # no node with that id
    cut[2 * S + rk[s2]] = lay.pack(2, rk[s2], 0)          # b2 without its cause
    res = weaver.weft_lists(b.offsets, b.id_key, b.cause_key, b.kind, lay, cut)
    st = res.weave.status
    # doc 1: s1's whole yarn (take-while never stops) + the node [(5 s1 0)]
    assert st[0] == 0 and list(np.diff(res.offsets)) == [2, 3, 2]
    assert st[1] & abi.STATUS_WEFT
    assert list(res.src[2:5]) == [0, 1, 0xFFFFFFFF]
    assert st[2] & abi.STATUS_ORPHAN
