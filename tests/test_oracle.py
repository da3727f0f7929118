"""Pin the CPU oracle to the reference's own tests (CPU only).

The reference (Clojure) cannot run in this image; its test files hold the
fixtures and known answers that pin our restatement:

* list_test.cljc:34-41, 44-96   incremental insert == refresh-caches (9 edge cases)
* list_test.cljc:98-116         random idempotence search (99 runs x 9 nodes)
* list_test.cljc:118-160        concurrent runs stick together
* list_test.cljc:162-173        hide/show toggling -> ("a" "b" "c") / ("b" "c")
* list_test.cljc:175-202        list protocol answers (count/seq/first/last/rest)
* map_test.cljc:5-89            map EDN answers, hide/show by key and by node id

Then the C oracle (packed keys; literal, F4 linked, F5 effective tree) is
cross-checked against the Python literal restatement.
"""
import random

import numpy as np
import pytest

import oracle
from oracle import causal_ref as R
from cause_amd import pack
from tests import refgen as G


# ----------------------------------------------------------------- list_test.cljc
def idempotent(ct):
    """list_test.cljc:34-41"""
    ref = R.refresh_caches(R.list_weave, ct)
    assert ct["site_id"] == ref["site_id"]
    assert ct["lamport_ts"] == ref["lamport_ts"]
    assert ct["nodes"] == ref["nodes"]
    assert ct["yarns"] == ref["yarns"]
    assert ct["weave"] == ref["weave"]


@pytest.mark.parametrize("case", range(len(G.EDGE_CASES)))
def test_known_idempotent_insert_edge_cases(case):
    ct = R.new_list_ct()
    for nd in G.EDGE_CASES[case]:
        ct = R.insert(R.list_weave, ct, nd)
    idempotent(ct)


def test_try_to_find_new_idempotent_edge_cases():
    """list_test.cljc:98-116 (seeded)."""
    rng = random.Random(1234)
    for _ in range(99):
        sites = [R.new_site_id(rng) for _ in range(5)]
        ct = R.new_list_ct(rng=rng)
        for _ in range(9):
            assert ct["weave"] == R.list_weave(ct)["weave"]
            ct = R.insert(R.list_weave, ct, G.rand_node(ct, rng, sites))
        assert ct["weave"] == R.list_weave(ct)["weave"]


def test_concurrent_runs_stick_together():
    """list_test.cljc:157-160"""
    rng = random.Random(7)
    for _ in range(5):
        ct, _, phrases = G.rand_weave_of_phrases(rng, 5)
        s = "".join(R.causal_list_to_edn(ct))
        for ph in phrases:
            assert ph in s


def _list(*vals, rng=None):
    ct = R.new_list_ct(rng=rng or random.Random(3))
    for v in vals:
        ct = R.list_conj(ct, v)
    return ct


def test_hide_and_show_and_hide_and_show():
    """list_test.cljc:162-173"""
    cl = _list("a", "b", "c")
    a_node = cl["weave"][1]
    assert R.causal_list_to_edn(cl) == ["a", "b", "c"]
    cl = R.append(R.list_weave, cl, a_node[0], R.HIDE)
    assert R.causal_list_to_edn(cl) == ["b", "c"]
    cl = R.append(R.list_weave, cl, a_node[0], R.H_SHOW)
    assert R.causal_list_to_edn(cl) == ["a", "b", "c"]
    cl = R.append(R.list_weave, cl, a_node[0], R.HIDE)
    assert R.causal_list_to_edn(cl) == ["b", "c"]
    cl = R.append(R.list_weave, cl, a_node[0], R.H_SHOW)
    assert R.causal_list_to_edn(cl) == ["a", "b", "c"]


def test_core_cljc_list_protocol():
    """list_test.cljc:175-202 (collection protocol answers over visible nodes)."""
    foo = R.Keyword(None, "foo")
    assert R.causal_list_to_edn(_list()) == []
    assert R.causal_list_to_edn(_list(foo, "bar"))
    assert R.causal_list_to_edn(_list(foo, R.HIDE)) == []
    ct = _list(foo)
    n = R.causal_list_to_list(ct)[0]
    ct2 = R.append(R.list_weave, R.append(R.list_weave, ct, n[0], R.HIDE), n[0], R.H_SHOW)
    assert len(R.causal_list_to_edn(ct2)) == 1
    assert len(R.causal_list_to_edn(_list())) == 0
    assert len(R.causal_list_to_edn(_list(foo))) == 1
    assert len(R.causal_list_to_edn(_list(foo, R.HIDE))) == 0
    node = ((1, "site-id", 0), R.ROOT_ID, foo)
    one = R.insert(R.list_weave, R.new_list_ct(), node)
    assert R.causal_list_to_list(one) == [node]                      # seq / first / last
    two = R.append(R.list_weave, one, R.ROOT_ID, "bar")
    assert R.causal_list_to_list(two)[1:] == [node]                  # next / rest


# ------------------------------------------------------------------ map_test.cljc
KW = lambda s: R.Keyword(None, s)


def _map(*kvs):
    ct = R.new_map_ct(rng=random.Random(5))
    for k, v in zip(kvs[::2], kvs[1::2]):
        ct = R.map_assoc(ct, k, v)
    return ct


def test_basic_map():
    """map_test.cljc:5-15 (the nested list is materialised by causal->edn)."""
    ct = _map(KW("foo"), "bar")
    ct = R.map_assoc(ct, KW("fizz"), "buzz")
    ct = R.map_assoc(ct, KW("fizz"), "bang")
    ct = R.map_dissoc(ct, KW("foo"))
    ct = R.map_assoc(ct, KW("list"), _list("a", "b", "c"))
    assert R.causal_map_to_edn(ct) == {KW("fizz"): "bang", KW("list"): ["a", "b", "c"]}


def test_map_hide_and_show():
    """map_test.cljc:17-31"""
    foo, fizz = KW("foo"), KW("fizz")
    ct = _map(foo, "bar", fizz, "buzz")
    assert R.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = R.append(R.map_weave, ct, foo, R.HIDE)
    assert R.causal_map_to_edn(ct) == {fizz: "buzz"}
    ct = R.append(R.map_weave, ct, foo, R.H_SHOW)
    assert R.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = R.append(R.map_weave, ct, foo, R.HIDE)
    assert R.causal_map_to_edn(ct) == {fizz: "buzz"}
    ct = R.append(R.map_weave, ct, foo, R.H_SHOW)
    assert R.causal_map_to_edn(ct) == {foo: "bar", fizz: "buzz"}
    ct = R.append(R.map_weave, ct, foo, "boo")
    ct = R.append(R.map_weave, ct, foo, R.H_SHOW)
    ct = R.append(R.map_weave, ct, foo, R.H_SHOW)
    assert R.causal_map_to_edn(ct) == {foo: "boo", fizz: "buzz"}


def test_map_hide_and_show_by_node_id():
    """map_test.cljc:33-43"""
    foo = KW("foo")
    ct = _map(foo, "bar")
    assert R.causal_map_to_edn(ct) == {foo: "bar"}
    ct = R.append(R.map_weave, ct, foo, "boo")
    assert R.causal_map_to_edn(ct) == {foo: "boo"}
    boo_id = R.causal_map_to_list(ct)[0][0]
    ct = R.append(R.map_weave, ct, boo_id, R.HIDE)
    assert R.causal_map_to_edn(ct) == {foo: "bar"}
    ct = R.append(R.map_weave, ct, boo_id, R.H_SHOW)
    assert R.causal_map_to_edn(ct) == {foo: "boo"}


def test_map_protocol():
    """map_test.cljc:45-89 (count/get answers)."""
    foo = KW("foo")
    assert R.map_count(_map()) == 0
    assert R.map_count(_map(foo, "bar")) == 1
    assert R.map_get(_map(foo, "bar"), foo) == "bar"
    gone = R.map_dissoc(_map(foo, "bar"), foo)
    assert R.map_count(gone) == 0 and R.map_get(gone, foo) is None
    back = R.append(R.map_weave, gone, foo, R.H_SHOW)   # (assoc :foo :causal/h.show)
    assert R.map_count(back) == 1 and R.map_get(back, foo) == "bar"
    node = ((1, "site-id", 0), KW("fizz"), "buzz")
    one = R.insert(R.map_weave, R.new_map_ct(), node)
    assert R.causal_map_to_list(one) == [node]


def test_map_quirk_assoc_after_dissoc_stays_hidden():
    """the key-level hide precedes newer values (map.cljc:50-52)."""
    a = KW("a")
    ct = R.map_assoc(R.map_dissoc(_map(a, 1), a), a, 2)
    assert R.causal_map_to_edn(ct) == {}


# ----------------------------------------------- C oracle vs the Python restatement
def _py_weave_perm(nodes):
    ct = R.new_list_ct()
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
    w = R.list_weave(ct)["weave"]
    where = {n[0]: i for i, n in enumerate(nodes)}
    return np.array([where[n[0]] for n in w], np.uint32)


def _packed(nodes):
    b = pack.pack_lists([nodes])
    return b.id_key, b.cause_key, b.kind, b.layout


def _check_all_methods(nodes, rng=None):
    nodes = list(nodes)
    if rng is not None:
        rng.shuffle(nodes)
    expect = _py_weave_perm(nodes)
    i, c, k, _ = _packed(nodes)
    for m in (oracle.METHOD_LITERAL, oracle.METHOD_LINKED, oracle.METHOD_EFF):
        perm, st = oracle.list_weave(i, c, k, m)
        assert st == 0
        assert np.array_equal(perm, expect), m
    # visibility: literal hide? on the packed weave == the Python EDN
    vis = oracle.list_visible(i, c, k, expect)
    ct = R.new_list_ct()
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
    ct = R.list_weave(ct)
    want = [nodes[p][2] for p, v in zip(expect, vis) if v]
    assert want == R.causal_list_to_edn(ct)


@pytest.mark.parametrize("case", range(len(G.EDGE_CASES)))
def test_c_oracle_edge_cases(case):
    _check_all_methods([R.ROOT_NODE] + G.EDGE_CASES[case], random.Random(case))


def test_c_oracle_random_reference_histories():
    rng = random.Random(99)
    for steps in (5, 9, 20, 60):
        for _ in range(40):
            nodes, _ = G.random_history(rng, steps)
            _check_all_methods([R.ROOT_NODE] + nodes, rng)


def test_c_oracle_stress_histories():
    rng = random.Random(2024)
    for n in (30, 120, 400):
        for p_special in (0.1, 0.35, 0.6):
            nodes = G.stress_history(rng, n, p_special=p_special, p_conj=0.15)
            _check_all_methods(nodes, rng)


def test_c_oracle_incremental_any_causal_order():
    """literal insertion in creation order and in random
    topological orders equals the full reweave."""
    rng = random.Random(11)
    for _ in range(40):
        nodes = G.stress_history(rng, 80, p_special=0.3, p_conj=0.2)
        i, c, k, _ = _packed(nodes)
        full, _ = oracle.list_weave(i, c, k, oracle.METHOD_LITERAL)
        order = list(range(len(nodes)))
        inc, _ = oracle.list_insert_sequence(i, c, k, order)
        assert np.array_equal(inc, full)
        # random topological order: repeatedly pick any node whose cause is in
        byid = {n[0]: j for j, n in enumerate(nodes)}
        placed, pending = {0}, list(range(1, len(nodes)))
        topo = [0]
        while pending:
            ready = [j for j in pending if byid[nodes[j][1]] in placed]
            j = rng.choice(ready)
            pending.remove(j)
            placed.add(j)
            topo.append(j)
        inc2, _ = oracle.list_insert_sequence(i, c, k, topo)
        assert np.array_equal(inc2, full)


def test_c_oracle_status_bits():
    nodes = [R.ROOT_NODE, ((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "x"),
             ((2, "aaaaaaaaaaaaa", 0), (9, "bbbbbbbbbbbbb", 0), "y")]
    i, c, k, _ = _packed(nodes)
    _, st = oracle.list_weave(i, c, k, oracle.METHOD_EFF)
    assert st & 4  # ORPHAN
    nodes = [R.ROOT_NODE, ((1, "aaaaaaaaaaaaa", 0), (3, "aaaaaaaaaaaaa", 0), "x"),
             ((3, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "y")]
    i, c, k, _ = _packed(nodes)
    _, st = oracle.list_weave(i, c, k, oracle.METHOD_EFF)
    assert st & 8  # NON_LAMPORT
    nodes = [((1, "aaaaaaaaaaaaa", 0), R.ROOT_ID, "x")]
    i, c, k, _ = _packed(nodes)
    _, st = oracle.list_weave(i, c, k, oracle.METHOD_EFF)
    assert st & 1  # ROOT


def test_seen_since_asap_never_decides():
    """clause B implies clause C, so dropping B leaves the weave
    unchanged (checked on the Python restatement)."""
    rng = random.Random(5)
    orig = R.weave_later

    def no_b(nl, nm, nr, seen):
        sr = R.is_special(R.peek_node(nr))
        sm = R.is_special(R.peek_node(nm))
        a = sr and R.first(nm) != R.second(nr) and ((not sm) or R.lt(R.first(nm), R.first(nr)))
        c = R.lt(R.first(nm), R.first(nr)) and ((not sm) or sr)
        return a or c

    for _ in range(30):
        nodes = G.stress_history(rng, 60, p_special=0.3)
        want = _py_weave_perm(nodes)
        R.weave_later = no_b
        try:
            got = _py_weave_perm(nodes)
        finally:
            R.weave_later = orig
        assert np.array_equal(want, got)


def test_java_string_order_of_site_ids():
    """Pins the id order used by (sort ::nodes) on the reference's exotic site
    ids (list_test.cljc:64-95): String.compareTo on UTF-16 code units."""
    sites = ["A~iIXinAXkGX7", " z ", "9FyYzf9pum6E4", "0", " a ", "7hLbMKLvcll_4", " f "]
    ranked = sorted(sites, key=pack.java_str_key)
    assert ranked == [" a ", " f ", " z ", "0", "7hLbMKLvcll_4", "9FyYzf9pum6E4",
                      "A~iIXinAXkGX7"]
    # a supplementary char (surrogate pair D83D..) sorts BELOW U+FFFD in Java
    assert pack.java_str_key("\U0001F600") < pack.java_str_key("�")


# ------------------------------------------------------------------------ maps
def _map_nodes(rng, n, nkeys=6, nsites=4):
    """Random CausalMap history: key-caused values and key hides, id-caused
    h.hide/h.show on value nodes (base/core.cljc:313-320 undo shape)."""
    sites = [R.new_site_id(rng) for _ in range(nsites)]
    keys = [KW(f"k{j}") for j in range(nkeys)]
    nodes, values, clock = [], [], 0
    for _ in range(n):
        clock += rng.randint(0, 2)
        site = rng.choice(sites)
        r = rng.random()
        if r < 0.6 or not values:
            nd = ((clock + 1, site, 0), rng.choice(keys), rng.randrange(100))
            values.append(nd[0])
        elif r < 0.75:
            nd = ((clock + 1, site, 0), rng.choice(keys), R.HIDE)
        else:
            nd = ((clock + 1, site, 0), rng.choice(values), rng.choice([R.H_HIDE, R.H_SHOW, R.HIDE]))
        clock += 1
        if any(x[0] == nd[0] for x in nodes):
            continue
        nodes.append(nd)
    return nodes


def _exotic_map_nodes(rng, n):
    """_map_nodes plus the causes c.map/weave folds whatever they are: nil, the
    root id, an absent id (the nil key) and a younger node (non-Lamport)."""
    nodes = _map_nodes(rng, n)
    out = []
    for nd in nodes:
        r = rng.random()
        if r < 0.1:
            nd = (nd[0], None, nd[2])
        elif r < 0.2:
            nd = (nd[0], R.ROOT_ID, nd[2])
        elif r < 0.3:
            nd = (nd[0], (10 ** 6 + rng.randrange(9), nd[0][1], 0), nd[2])
        elif r < 0.4 and len(nodes) > 1:
            nd = (nd[0], rng.choice([x[0] for x in nodes if x[0] != nd[0]]), nd[2])
        out.append(nd)
    return out


@pytest.mark.parametrize("exotic", [False, True])
def test_c_oracle_map_matches_python(exotic):
    rng = random.Random(77)
    for _ in range(60 if not exotic else 200):
        n = rng.randint(1, 40)
        nodes = _exotic_map_nodes(rng, n) if exotic else _map_nodes(rng, n)
        ct = R.new_map_ct()
        ct["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
        ct = R.map_weave(ct)
        want = R.causal_map_to_edn(ct)
        # pack: key tokens for keyword causes, ids for id causes, nil = cause_is_id 2
        lay = pack.layout_for([[(n[0], n[1] if R.valid_id(n[1]) else None, n[2]) for n in nodes]
                               + [R.ROOT_NODE]])
        rank = pack.intern_sites([n[0] for n in nodes] + [n[1] for n in nodes if R.valid_id(n[1])]
                                 + [R.ROOT_ID])
        key_tok = {}
        idk = np.array([lay.pack(n[0][0], rank[n[0][1]], n[0][2]) for n in nodes], np.uint64)
        cause, cis = [], []
        for n in nodes:
            if R.valid_id(n[1]):
                cause.append(lay.pack(n[1][0], rank[n[1][1]], n[1][2]))
                cis.append(1)
            elif n[1] is None:
                cause.append(0)
                cis.append(2)
            else:
                cause.append(key_tok.setdefault(n[1], len(key_tok)))
                cis.append(0)
        cis = np.array(cis, np.uint8)
        cause = oracle.map_causes(np.array(cause, np.uint64), cis)
        kind = np.array([pack.kind_of(n[2]) for n in nodes], np.uint8)
        root = lay.pack(0, rank["0"], 0)
        nk, npos, sk, sa = oracle.map_weave(idk, cause, cis, kind, root)
        inv = {v: k for k, v in key_tok.items()}
        ids = {int(lay.pack(x[0], rank[x[1]], x[2])): x for x in
               [nd[0] for nd in nodes] + [nd[1] for nd in nodes if R.valid_id(nd[1])] + [R.ROOT_ID]}

        def key_of(k):
            if k == oracle.NIL:
                return None
            if k & (1 << 63):
                return inv[k & ~(1 << 63)]
            return ids[k]  # an id key

        got = {}
        for s_key, act in zip(sk, sa):
            if act >= 0:
                got[key_of(int(s_key))] = nodes[act][2]
        assert got == want
        # per-node placement equals the Python key weaves
        for k, wk in ct["weave"].items():
            for pos, n in enumerate(wk[1:], 1):
                j = next(x for x, m in enumerate(nodes) if m[0] == n[0])
                assert npos[j] == pos, (k, n)
