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
