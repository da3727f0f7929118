"""Golden fixtures (tests/golden/, written by tests/golden/make_golden.py).

CPU: the oracle reproduces the reference's own known answers (SURVEY.md
Appendix B orders of list_test.cljc:44-96, the EDN its tests assert, the Java
site order) and the committed packed vectors.  GPU (-m gpu): the HIP weave
reproduces the same vectors through the C ABI, with no oracle call at run time.
"""
import json
import os
import random

import numpy as np
import pytest

import oracle
from cause_amd import pack
from oracle import causal_ref as R

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EDGE = json.load(open(os.path.join(HERE, "edge_cases.json")))
VEC = np.load(os.path.join(HERE, "packed_vectors.npz"))  # allow_pickle=False (default)
GROUPS = sorted({k.rsplit("_", 2)[0] for k in VEC.files if k.endswith("_offsets")})


def _val(v):
    if isinstance(v, dict):
        ns, _, name = v["kw"].rpartition("/")
        return R.Keyword(ns or None, name)
    return v


def _id(x):
    return None if x is None else (x[0], x[1], x[2])


def case_nodes(c):
    return [R.ROOT_NODE] + [(_id(a), _id(b), _val(v)) for a, b, v in c["nodes"]]


def _short(n):
    (ts, site, _), _, v = n
    return [ts, site[:2], "hide" if v == R.HIDE else v]


def group(name):
    g = {k[len(name) + 1:]: VEC[k] for k in VEC.files if k.startswith(name + "_")}
    ts_bits, site_bits, tx_bits = (int(x) for x in g["layout"])
    g["layout"] = pack.KeyLayout(ts_bits, site_bits, tx_bits)
    return g


# ------------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("ci", range(len(EDGE["cases"])))
def test_oracle_reproduces_appendix_b(ci):
    """Full reweave (list.cljc:26-28) of each reference edge case: order and EDN."""
    c = EDGE["cases"][ci]
    nodes = case_nodes(c)
    random.Random(ci).shuffle(nodes)
    ct = R.new_list_ct()
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
    ct = R.list_weave(ct)
    assert ct["weave"][0] == R.ROOT_NODE
    assert [_short(n) for n in ct["weave"][1:]] == c["weave_after_root"]
    assert R.causal_list_to_edn(ct) == c["edn"]
    # the C oracle (packed keys), every method
    b = pack.pack_lists([nodes])
    where = {n[0]: i for i, n in enumerate(nodes)}
    want = np.array([where[n[0]] for n in ct["weave"]], np.uint32)
    for m in (oracle.METHOD_LITERAL, oracle.METHOD_LINKED, oracle.METHOD_EFF):
        perm, st = oracle.list_weave(b.id_key, b.cause_key, b.kind, m)
        assert st == 0 and np.array_equal(perm, want), m


def test_site_order_is_java_string_order():
    sites = list(EDGE["site_order"])
    random.Random(1).shuffle(sites)
    assert sorted(sites, key=pack.java_str_key) == EDGE["site_order"]


def test_known_list_answers():
    """list_test.cljc:162-173, answers read from the fixture."""
    want = EDGE["known_answers"]["list_hide_show"]["edn_after_each"]
    ct = R.new_list_ct(rng=random.Random(3))
    for v in "abc":
        ct = R.list_conj(ct, v)
    a_id = ct["weave"][1][0]
    got = [R.causal_list_to_edn(ct)]
    for v in (R.HIDE, R.H_SHOW, R.HIDE, R.H_SHOW):
        ct = R.append(R.list_weave, ct, a_id, v)
        got.append(R.causal_list_to_edn(ct))
    assert got == want


def _edn_json(m):
    return {":" + k.name: v for k, v in m.items()}


def test_known_map_answers():
    """map_test.cljc:17-43 and SURVEY F8a, answers read from the fixture."""
    ka = EDGE["known_answers"]
    foo, fizz = R.Keyword(None, "foo"), R.Keyword(None, "fizz")
    ct = R.new_map_ct(rng=random.Random(5))
    ct = R.map_assoc(R.map_assoc(ct, foo, "bar"), fizz, "buzz")
    got = [_edn_json(R.causal_map_to_edn(ct))]
    for v in (R.HIDE, R.H_SHOW, R.HIDE, R.H_SHOW):
        ct = R.append(R.map_weave, ct, foo, v)
        got.append(_edn_json(R.causal_map_to_edn(ct)))
    for v in ("boo", R.H_SHOW, R.H_SHOW):
        ct = R.append(R.map_weave, ct, foo, v)
    got.append(_edn_json(R.causal_map_to_edn(ct)))
    assert got == ka["map_hide_show"]["edn_after_each"]

    ct = R.map_assoc(R.new_map_ct(rng=random.Random(5)), foo, "bar")
    got = [_edn_json(R.causal_map_to_edn(ct))]
    ct = R.append(R.map_weave, ct, foo, "boo")
    got.append(_edn_json(R.causal_map_to_edn(ct)))
    boo_id = R.causal_map_to_list(ct)[0][0]
    for v in (R.HIDE, R.H_SHOW):
        ct = R.append(R.map_weave, ct, boo_id, v)
        got.append(_edn_json(R.causal_map_to_edn(ct)))
    assert got == ka["map_hide_show_by_id"]["edn_after_each"]

    a = R.Keyword(None, "a")
    ct = R.map_assoc(R.new_map_ct(rng=random.Random(5)), a, 1)
    ct = R.map_assoc(R.map_dissoc(ct, a), a, 2)
    assert _edn_json(R.causal_map_to_edn(ct)) == ka["map_quirk_f8a"]["edn"]


@pytest.mark.parametrize("name", GROUPS)
def test_oracle_reproduces_packed_vectors(name):
    g = group(name)
    for m in (oracle.METHOD_LITERAL, oracle.METHOD_LINKED, oracle.METHOD_EFF):
        perm, vis, st = oracle.batch_lists(g["offsets"], g["id_key"], g["cause_key"], g["kind"],
                                           method=m)
        assert not st.any()
        assert np.array_equal(perm, g["weave_perm"]), m
        assert np.array_equal(vis, g["visible"]), m


# ------------------------------------------------------------------- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("name", GROUPS)
def test_hip_weave_reproduces_packed_vectors(name):
    from cause_amd import abi

    g = group(name)
    off = g["offsets"]
    with abi.Weaver(0) as w:
        res = w.weave_lists(off, g["id_key"], g["cause_key"], g["kind"], g["layout"])
    assert not res.status.any()
    assert np.array_equal(res.weave_perm, g["weave_perm"])
    assert np.array_equal(res.visible(), g["visible"].astype(bool))
    assert np.array_equal(res.max_ts, g["max_ts"])
    assert np.array_equal(res.yarn_perm, g["yarn_perm"])
    D = len(off) - 1
    vc = [int(g["visible"][int(off[d]):int(off[d + 1])].sum()) for d in range(D)]
    assert np.array_equal(res.visible_count, np.array(vc, np.uint32))


@pytest.mark.gpu
def test_hip_weave_reproduces_appendix_b():
    from cause_amd import abi

    docs = []
    for ci, c in enumerate(EDGE["cases"]):
        nodes = case_nodes(c)
        random.Random(100 + ci).shuffle(nodes)
        docs.append(nodes)
    b = pack.pack_lists(docs)
    with abi.Weaver(0) as w:
        res = w.weave_lists(b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    assert not res.status.any()
    vis = res.visible()
    for d, (nodes, c) in enumerate(zip(docs, EDGE["cases"])):
        lo, hi = int(b.offsets[d]), int(b.offsets[d + 1])
        woven = [nodes[p] for p in res.weave_perm[lo:hi]]
        assert woven[0] == R.ROOT_NODE
        assert [_short(n) for n in woven[1:]] == c["weave_after_root"]
        assert [n[2] for n, v in zip(woven, vis[lo:hi]) if v] == c["edn"]
