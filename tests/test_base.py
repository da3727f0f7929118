"""CausalBase materialisation (cause_amd/base.py).

CPU: the transaction bookkeeping builds the nodes the reference's own tests
expect (base/core_test.cljc:17-58).  GPU (-m gpu): cb->edn weaves every
collection in batched GPU calls and resolves refs, reproducing the EDN the
reference's tests assert (base/core_test.cljc:8-15, 60-90), and the history is
sorted on the GPU."""
import random

import pytest

from cause_amd import base as B
from cause_amd import causal as C

K = lambda name: C.Keyword(None, name)


def cb0():
    return B.new_cb(rng=random.Random(7))


def test_map_to_nodes():
    """base/core_test.cljc:17-22"""
    cb = cb0()
    _, tx, nodes = B.map_to_nodes(cb, 0, {K("a"): 1, K("b"): 2})
    assert tx == 2
    s = cb["site_id"]
    assert nodes == [((1, s, 0), K("a"), 1), ((1, s, 1), K("b"), 2)]


def test_list_to_nodes():
    """base/core_test.cljc:23-29"""
    cb = cb0()
    _, tx, nodes, last = B.list_to_nodes(cb, 0, [1, 2, 3])
    s = cb["site_id"]
    assert tx == 3
    assert nodes == [((1, s, 0), (0, "0", 0), 1), ((1, s, 1), (1, s, 0), 2),
                     ((1, s, 2), (1, s, 1), 3)]
    assert last == (1, s, 2)


@pytest.mark.parametrize("value,tx,ncoll", [
    ({K("a"): {K("aa"): 1, K("bb"): 2, K("cc"): 3}}, 4, 2),
    ({K("a"): {K("b"): {K("c"): K("d")}}}, 3, 3),
    ([1, [2, [3]]], 5, 3),
    ([1, "hello", "world"], 11, 1),
    ([K("div"), {K("title"): "don't break"}, [K("span"), "break"]], 10, 3)])
def test_flatten_value(value, tx, ncoll):
    """base/core_test.cljc:33-58"""
    cb, tx_i, ref = B.flatten_value(cb0(), 0, value)
    assert tx_i == tx
    assert B.is_ref(ref)
    assert len(cb["collections"]) == ncoll


def test_transact_validations():
    """base/core.cljc:217-227"""
    with pytest.raises(C.CauseError):
        B.transact_(cb0(), [["nope", None, [1]]])
    cb = B.transact_(cb0(), [[None, None, [1]]])
    with pytest.raises(C.CauseError):
        B.transact_(cb, [["nope", None, [1]]])
    with pytest.raises(C.CauseError):
        B.transact_(cb0(), [[None, None, 5]])


# ------------------------------------------------------------------- GPU ----
def edn(cb):
    return B.cb_to_edn(cb)[0]


@pytest.mark.gpu
def test_cb_to_edn():
    """base/core_test.cljc:8-15"""
    cb = B.transact_(cb0(), [[None, None, [K("div"), {K("foo"): "bar"}, "wat", [K("p"), "baz"]]]])
    assert edn(cb) == [K("div"), {K("foo"): "bar"}, "w", "a", "t", [K("p"), "b", "a", "z"]]


@pytest.mark.gpu
def test_transact_maps():
    """base/core_test.cljc:60-71"""
    assert edn(cb0()) is None
    cb = B.transact_(cb0(), [[None, None, {K("a"): 1}]])
    r = cb["root_uuid"]
    assert edn(cb) == {K("a"): 1}
    assert edn(B.transact_(cb, [[r, K("a"), "hi"]])) == {K("a"): "hi"}
    assert edn(B.transact_(cb, [[r, None, {K("a"): 2, K("b"): 3}]])) == {K("a"): 2, K("b"): 3}
    assert edn(B.transact_(cb, [[r, K("b"), {K("c"): 2}]])) == {K("a"): 1, K("b"): {K("c"): 2}}
    assert edn(B.transact_(cb, [[r, K("a"), C.HIDE], [r, None, {K("b"): 2, K("c"): "hi"}],
                                [r, None, {K("b"): C.HIDE}]])) == {K("c"): "hi"}


@pytest.mark.gpu
def test_transact_lists():
    """base/core_test.cljc:72-83"""
    cb = B.transact_(cb0(), [[None, None, [1, 2]]])
    r = cb["root_uuid"]
    assert edn(cb) == [1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, 0]])) == [0, 1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, [0]]])) == [0, 1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, [-2, -1, 0]]])) == [-2, -1, 0, 1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, "hi"]])) == ["h", "i", 1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, ["hi"]]])) == ["h", "i", 1, 2]
    assert edn(B.transact_(cb, [[r, C.ROOT_ID, [["hi"]]]])) == [["h", "i"], 1, 2]


@pytest.mark.gpu
def test_history_sorted_and_site_shared():
    """base/core_test.cljc:84-90 (one site across nested collections) and the
    ::history order (sorted reverse paths, base/core.cljc:22, 107-115)."""
    cb = B.transact_(cb0(), [[None, None, [K("div"), {K("a"): 1}, [K("span"), {K("b"): 2}, "abc"]]]])
    cb = B.transact_(cb, [[cb["root_uuid"], C.ROOT_ID, "xy"]])
    h = B.history(cb)
    assert len(h) == len(cb["history"])
    assert all(i[1] == cb["site_id"] for i, _ in h)
    assert [i for i, _ in h] == sorted(i for i, _ in cb["history"])
    # expand-reverse-path (base/core.cljc:270-275): each entry names its node
    for i, u in h:
        assert i in cb["collections"][u]["nodes"]
