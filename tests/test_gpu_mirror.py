"""The reference's own list tests (list_test.cljc), run against the host mirror
whose every weave is the HIP full reweave (cause_amd.causal -> C ABI)."""
import random

import pytest

from cause_amd import causal as C
from oracle import causal_ref as R
from tests import refgen as G

pytestmark = pytest.mark.gpu


def _to_mirror(v):
    """Oracle keyword values -> mirror keywords (same ns/name)."""
    return C.Keyword(v.ns, v.name) if isinstance(v, R.Keyword) else v


def _mnode(nd):
    return (nd[0], nd[1], _to_mirror(nd[2]))


def _list(*vals, rng=None):
    ct = C.new_list_ct(rng=rng or random.Random(3))
    for v in vals:
        ct = C.list_conj(ct, v)
    return ct


def test_hide_and_show_and_hide_and_show():
    """list_test.cljc:162-173"""
    cl = _list("a", "b", "c")
    a_node = cl["weave"][1]
    assert C.causal_list_to_edn(cl) == ["a", "b", "c"]
    cl = C.append(C.list_weave, cl, a_node[0], C.HIDE)
    assert C.causal_list_to_edn(cl) == ["b", "c"]
    cl = C.append(C.list_weave, cl, a_node[0], C.H_SHOW)
    assert C.causal_list_to_edn(cl) == ["a", "b", "c"]
    cl = C.append(C.list_weave, cl, a_node[0], C.HIDE)
    assert C.causal_list_to_edn(cl) == ["b", "c"]
    cl = C.append(C.list_weave, cl, a_node[0], C.H_SHOW)
    assert C.causal_list_to_edn(cl) == ["a", "b", "c"]


def test_core_cljc_list_protocol():
    """list_test.cljc:175-202"""
    foo = C.Keyword(None, "foo")
    assert C.causal_list_to_edn(_list()) == []
    assert C.causal_list_to_edn(_list(foo, "bar"))
    assert C.causal_list_to_edn(_list(foo, C.HIDE)) == []
    ct = _list(foo)
    n = C.causal_list_to_list(ct)[0]
    ct2 = C.append(C.list_weave, C.append(C.list_weave, ct, n[0], C.HIDE), n[0], C.H_SHOW)
    assert C.count(ct2) == 1
    assert C.count(_list()) == 0 and C.count(_list(foo)) == 1 and C.count(_list(foo, C.HIDE)) == 0
    node = ((1, "site-id", 0), C.ROOT_ID, foo)
    one = C.insert(C.list_weave, C.new_list_ct(), node)
    assert C.causal_list_to_list(one) == [node]
    two = C.append(C.list_weave, one, C.ROOT_ID, "bar")
    assert C.causal_list_to_list(two)[1:] == [node]


@pytest.mark.parametrize("case", range(len(G.EDGE_CASES)))
def test_known_idempotent_insert_edge_cases(case):
    """list_test.cljc:34-96: insert node by node, then refresh-caches; and the
    GPU weave equals the oracle's literal incremental weave."""
    ct = C.new_list_ct()
    ref = R.new_list_ct()
    for nd in G.EDGE_CASES[case]:
        ct = C.insert(C.list_weave, ct, _mnode(nd))
        ref = R.insert(R.list_weave, ref, nd)
    fresh = C.refresh_caches(C.list_weave, ct)
    assert fresh["weave"] == ct["weave"]
    assert fresh["lamport_ts"] == ct["lamport_ts"] == ref["lamport_ts"]
    assert fresh["yarns"] == {k: [_mnode(n) for n in v] for k, v in ref["yarns"].items()}
    assert [n[0] for n in ct["weave"]] == [n[0] for n in ref["weave"]]


def test_try_to_find_new_idempotent_edge_cases():
    """list_test.cljc:98-116, GPU weave vs the literal incremental weave."""
    rng = random.Random(77)
    batch_ct, batch_ref = [], []
    for _ in range(99):
        nodes, ref = G.random_history(rng, 9)
        ct = C.new_list_ct()
        ct["nodes"] = {nd[0]: (nd[1], _to_mirror(nd[2])) for nd in [R.ROOT_NODE] + nodes}
        batch_ct.append(ct)
        batch_ref.append(ref)
    woven = C.weave_lists(batch_ct)          # one GPU call for all 99 histories
    for ct, ref in zip(woven, batch_ref):
        assert [n[0] for n in ct["weave"]] == [n[0] for n in ref["weave"]]
        assert [_to_mirror(v) for v in R.causal_list_to_edn(ref)] == C.causal_list_to_edn(ct)


def test_concurrent_runs_stick_together():
    """list_test.cljc:157-160"""
    rng = random.Random(9)
    ct_ref, nodes, phrases = G.rand_weave_of_phrases(rng, 5)
    ct = C.new_list_ct()
    ct["nodes"] = {nd[0]: (nd[1], nd[2]) for nd in [R.ROOT_NODE] + nodes}
    s = "".join(C.causal_list_to_edn(C.list_weave(ct)))
    for ph in phrases:
        assert ph in s


def test_insert_errors_mirror_the_reference():
    """shared.cljc:163-178 error causes."""
    ct = C.new_list_ct()
    with pytest.raises(C.CauseError) as e:
        C.insert(C.list_weave, ct, ((1, "aaaaaaaaaaaaa", 0), (5, "bbbbbbbbbbbbb", 0), "x"))
    assert e.value.causes == {"cause-must-exist"}
    ct = C.insert(C.list_weave, ct, ((1, "aaaaaaaaaaaaa", 0), C.ROOT_ID, "x"))
    with pytest.raises(C.CauseError) as e:
        C.insert(C.list_weave, ct, ((1, "aaaaaaaaaaaaa", 0), C.ROOT_ID, "y"))
    assert e.value.causes == {"append-only", "edits-not-allowed"}
    assert C.insert(C.list_weave, ct, ((1, "aaaaaaaaaaaaa", 0), C.ROOT_ID, "x")) is ct


# ------------------------------------------------------------------ map_test.cljc
MKW = lambda s: C.Keyword(None, s)


def _cmap(*kvs):
    ct = C.new_map_ct(rng=random.Random(5))
    for k, v in zip(kvs[::2], kvs[1::2]):
        ct = C.map_assoc(ct, k, v)
    return ct


def test_map_basic():
    """map_test.cljc:5-15, the nested causal list included: (assoc :list
    (swap! (atom (c/list)) conj "a" "b" "c")) materialises as ("a" "b" "c")."""
    ct = _cmap(MKW("foo"), "bar")
    ct = C.map_assoc(ct, MKW("fizz"), "buzz")
    ct = C.map_assoc(ct, MKW("fizz"), "bang")
    ct = C.map_dissoc(ct, MKW("foo"))
    lst = C.new_list_ct(rng=random.Random(6))
    for v in ("a", "b", "c"):
        lst = C.list_conj(lst, v)
    ct = C.map_assoc(ct, MKW("list"), lst)
    assert C.causal_map_to_edn(ct) == {MKW("fizz"): "bang", MKW("list"): ["a", "b", "c"]}


def test_nested_causal_values_in_lists_and_maps():
    """s/causal->edn recursion (shared.cljc:320-328) through lists and maps:
    a list holding a map holding a list."""
    inner = C.new_list_ct(rng=random.Random(7))
    for v in ("x", "y"):
        inner = C.list_conj(inner, v)
    m = _cmap(MKW("k"), inner, MKW("n"), 1)
    outer = C.new_list_ct(rng=random.Random(8))
    outer = C.list_conj(outer, "head")
    outer = C.list_conj(outer, m)
    assert C.causal_list_to_edn(outer) == ["head", {MKW("k"): ["x", "y"], MKW("n"): 1}]


def test_map_hide_and_show():
    """map_test.cljc:17-31"""
    foo, fizz = MKW("foo"), MKW("fizz")
    ct = _cmap(foo, "bar", fizz, "buzz")
    assert C.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = C.append(C.map_weave, ct, foo, C.HIDE)
    assert C.causal_map_to_edn(ct) == {fizz: "buzz"}
    ct = C.append(C.map_weave, ct, foo, C.H_SHOW)
    assert C.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = C.append(C.map_weave, ct, foo, C.HIDE)
    assert C.causal_map_to_edn(ct) == {fizz: "buzz"}
    ct = C.append(C.map_weave, ct, foo, C.H_SHOW)
    assert C.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = C.append(C.map_weave, ct, foo, "boo")
    ct = C.append(C.map_weave, ct, foo, C.H_SHOW)
    ct = C.append(C.map_weave, ct, foo, C.H_SHOW)
    assert C.causal_map_to_edn(ct) == {foo: "boo", fizz: "buzz"}


def test_map_hide_and_show_by_node_id():
    """map_test.cljc:33-43"""
    foo = MKW("foo")
    ct = _cmap(foo, "bar")
    ct = C.append(C.map_weave, ct, foo, "boo")
    assert C.causal_map_to_edn(ct) == {foo: "boo"}
    boo_id = C.causal_map_to_list(ct)[0][0]
    ct = C.append(C.map_weave, ct, boo_id, C.HIDE)
    assert C.causal_map_to_edn(ct) == {foo: "bar"}
    ct = C.append(C.map_weave, ct, boo_id, C.H_SHOW)
    assert C.causal_map_to_edn(ct) == {foo: "boo"}


def test_map_protocol_and_quirk():
    """map_test.cljc:45-89 and SURVEY F8a."""
    foo, a = MKW("foo"), MKW("a")
    assert C.map_count(_cmap()) == 0
    assert C.map_get(_cmap(foo, "bar"), foo) == "bar"
    gone = C.map_dissoc(_cmap(foo, "bar"), foo)
    assert C.map_count(gone) == 0 and C.map_get(gone, foo) is None
    back = C.append(C.map_weave, gone, foo, C.H_SHOW)
    assert C.map_count(back) == 1 and C.map_get(back, foo) == "bar"
    node = ((1, "site-id", 0), MKW("fizz"), "buzz")
    one = C.insert(C.map_weave, C.new_map_ct(), node)
    assert C.causal_map_to_list(one) == [node]
    ct = C.map_assoc(C.map_dissoc(_cmap(a, 1), a), a, 2)
    assert C.causal_map_to_edn(ct) == {}


def test_map_batch_matches_python_restatement():
    """Many random map histories (incl. F8c id keys) in one GPU call vs causal_ref."""
    rng = random.Random(99)
    sites = [C.new_site_id(rng) for _ in range(3)]
    cts, py = [], []
    for _ in range(60):
        nodes, values = [], []
        for m in range(rng.randint(1, 30)):
            nid = (m + 1, rng.choice(sites), 0)
            r = rng.random()
            if r < 0.55 or not nodes:
                nd = (nid, f"k{rng.randint(0, 6)}", f"v{m}")
                values.append(nid)
            elif r < 0.7:
                nd = (nid, f"k{rng.randint(0, 6)}", "HIDE")
            else:
                pool = values if rng.random() < 0.8 else [x[0] for x in nodes]
                nd = (nid, rng.choice(pool), rng.choice(["HIDE", "H_HIDE", "H_SHOW", f"w{m}"]))
            nodes.append(nd)
        conv = lambda v, M: {"HIDE": M.HIDE, "H_HIDE": M.H_HIDE, "H_SHOW": M.H_SHOW}.get(v, v)
        ct = C.new_map_ct()
        ct["nodes"] = {n[0]: (n[1], conv(n[2], C)) for n in nodes}
        cts.append(ct)
        p = R.new_map_ct()
        p["nodes"] = {n[0]: (n[1], conv(n[2], R)) for n in nodes}
        py.append(R.map_weave(p))
    got = C.weave_maps(cts)
    for g, p in zip(got, py):
        want = {k: [(n[0], n[1], str(n[2])) for n in w] for k, w in p["weave"].items()}
        have = {k: [(n[0], n[1], str(n[2])) for n in w] for k, w in g["weave"].items()}
        assert have == want
        assert {k: str(v) for k, v in C.causal_map_to_edn(g).items()} == \
            {k: str(v) for k, v in R.causal_map_to_edn(p).items()}


@pytest.mark.parametrize("colls,n_lo,n_hi", [(40, 2, 40), (2, 2500, 3500)])
def test_map_nil_root_absent_and_younger_causes_match_python_restatement(colls, n_lo, n_hi):
    """Maps the reference folds whatever the causes: nil causes and the root id
    (the nil key, under its root), absent ids (the nil key, appended), children
    of those, and undo/redo of a younger node.  Small maps take the fused
    kernel, the 2,500+-node ones the general path; both vs causal_ref on real
    Clojure-shaped values."""
    rng = random.Random(7 + n_lo)
    sites = [C.new_site_id(rng) for _ in range(3)]
    conv = lambda v, M: {"HIDE": M.HIDE, "H_HIDE": M.H_HIDE, "H_SHOW": M.H_SHOW}.get(v, v)
    cts, py = [], []
    for _ in range(colls):
        n = rng.randint(n_lo, n_hi)
        ts = rng.sample(range(1, 4 * n), n)
        nodes = []
        for m, t in enumerate(ts):
            nid = (t, rng.choice(sites), 0)
            r = rng.random()
            if r < 0.5 or not nodes:
                nd = [nid, f"k{rng.randint(0, 3)}", rng.choice([f"v{m}", f"v{m}", "HIDE"])]
            elif r < 0.58:
                nd = [nid, None, rng.choice([f"n{m}", "HIDE"])]
            elif r < 0.66:
                nd = [nid, R.ROOT_ID, rng.choice([f"r{m}", "HIDE", "H_SHOW"])]
            elif r < 0.74:
                nd = [nid, (10 ** 9 + m, sites[0], 0), rng.choice([f"a{m}", "H_HIDE"])]
            else:
                nd = [nid, "LATER", rng.choice(["HIDE", "H_HIDE", "H_SHOW", f"w{m}"])]
            nodes.append(nd)
        for nd in nodes:
            if nd[1] == "LATER":  # any other node: older, or younger (non-Lamport)
                nd[1] = rng.choice([x for x in nodes if x is not nd])[0]
        ct = C.new_map_ct()
        ct["nodes"] = {nd[0]: (nd[1], conv(nd[2], C)) for nd in nodes}
        cts.append(ct)
        p = R.new_map_ct()
        p["nodes"] = {nd[0]: (nd[1], conv(nd[2], R)) for nd in nodes}
        py.append(R.map_weave(p))
    got = C.weave_maps(cts)
    nil_keys = 0
    for g, p in zip(got, py):
        want = {k: [(n[0], n[1], str(n[2])) for n in w] for k, w in p["weave"].items()}
        have = {k: [(n[0], n[1], str(n[2])) for n in w] for k, w in g["weave"].items()}
        assert have == want
        nil_keys += None in have
        assert {k: str(v) for k, v in C.causal_map_to_edn(g).items()} == \
            {k: str(v) for k, v in R.causal_map_to_edn(p).items()}
    assert nil_keys >= colls // 2


def test_map_exotic_site_ids_sort_before_zero():
    """Map nodes from site-ids that sort before "0" in String.compareTo order
    (" a ", " f ", " z ", as list_test.cljc:85-96 uses): the GPU map weave
    equals the literal restatement (map.cljc:21-59) key by key."""
    sites = [" a ", " f ", " z ", "A~aaaaaaaaaaa", "zzzzzzzzzzzzz"]
    keys = [MKW("a"), MKW("b"), "s"]
    for seed in range(6):
        rng = random.Random(100 + seed)
        nodes = {}
        for ts in range(1, 80):
            site = rng.choice(sites)
            r = rng.random()
            if r < 0.55 or not nodes:
                body = (rng.choice(keys), rng.choice(["x", "y", 1, 2]))
            elif r < 0.7:
                body = (rng.choice(keys), R.HIDE)
            else:  # undo / redo of an earlier node: an id cause (F8c keys too)
                body = (rng.choice(list(nodes)), rng.choice([R.H_HIDE, R.H_SHOW, R.HIDE]))
            nodes[(ts, site, rng.randrange(3))] = body
        ct, ref = C.new_map_ct(), R.new_map_ct()
        ct["nodes"], ref["nodes"] = dict(nodes), dict(nodes)
        got, want = C.map_weave(ct), R.map_weave(ref)
        assert got["weave"] == want["weave"], seed
        assert C.causal_map_to_edn(got) == R.causal_map_to_edn(want), seed


def test_mirror_threads_use_their_own_contexts():
    """Concurrent weaves from several host threads (swap! retries, SURVEY
    §8(b) threading): each thread gets its own context, results match."""
    import concurrent.futures as cf

    rng = random.Random(11)
    cts = []
    for _ in range(24):
        nodes, _ = G.random_history(rng, 40)
        ct = C.new_list_ct()
        ct["nodes"] = {nd[0]: (nd[1], nd[2]) for nd in [R.ROOT_NODE] + nodes}
        cts.append(ct)
    want = [C.causal_list_to_edn(C.list_weave(ct)) for ct in cts]
    with cf.ThreadPoolExecutor(6) as ex:
        for _ in range(3):
            got = list(ex.map(lambda ct: C.causal_list_to_edn(C.list_weave(ct)), cts))
            assert got == want
