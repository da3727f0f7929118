"""The exact path's rule on CPU (no GPU): documents outside the fast path's
domain -- absent causes, non-Lamport causes, nil causes, no root, ids below the
root, non-id causes.

1. The C literal fold (oracle/weave_oracle.c, clause for clause
   shared.cljc:194-241) agrees with the Python restatement on real
   Clojure-shaped values (oracle/causal_ref.py) for such documents: two
   independent restatements of the reference, pinned to each other where the
   reference's own tests say nothing (they never build such a bag).
2. The general fold (the rule exact.hip's k_xfold implements, restated in
   oracle/weave_oracle.c or_list_fold_general) equals the literal fold on
   thousands of random out-of-domain histories, clean and dirty.
"""
import random

import numpy as np
import pytest

import oracle
from cause_amd import gen, pack
from oracle import causal_ref as R
from tests import outdomain as X
from tests import refgen as G


def _py_literal(nodes):
    ct = R.new_list_ct()
    ct["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
    w = R.list_weave(ct)["weave"]
    where = {n[0]: i for i, n in enumerate(nodes)}
    vis = [not R.hide_q(a, b) for a, b in zip(w, w[1:] + [None])]
    return np.array([where[n[0]] for n in w], np.uint32), np.array(vis, np.uint8)


def _c(nodes, method):
    b = pack.pack_lists([nodes])
    perm, st = oracle.list_weave(b.id_key, b.cause_key, b.kind, method)
    vis = oracle.list_visible(b.id_key, b.cause_key, b.kind, perm)
    return perm, vis, st


@pytest.mark.parametrize("kind", X.KINDS + ("all",))
def test_c_literal_matches_python_literal_out_of_domain(kind):
    rng = random.Random(hash(kind) & 0xFFFF)
    kinds = X.KINDS if kind == "all" else (kind,)
    for steps in (6, 12, 30):
        for _ in range(25):
            nodes, _ = G.random_history(rng, steps)
            bad = X.corrupt([R.ROOT_NODE] + nodes, rng, kinds, rate=0.2)
            rng.shuffle(bad)
            want, wvis = _py_literal(bad)
            got, gvis, st = _c(bad, oracle.METHOD_LITERAL)
            assert np.array_equal(got, want)
            assert np.array_equal(gvis, wvis)
            gen_perm, _, _ = _c(bad, oracle.METHOD_GENERAL)
            assert np.array_equal(gen_perm, want)


def test_edge_cases_corrupted():
    """The reference's 9 edge cases (list_test.cljc:44-96), each broken every way."""
    rng = random.Random(7)
    for case in G.EDGE_CASES:
        for kind in X.KINDS:
            bad = X.corrupt([R.ROOT_NODE] + list(case), rng, (kind,), rate=0.3)
            want, _ = _py_literal(bad)
            for m in (oracle.METHOD_LITERAL, oracle.METHOD_GENERAL):
                got, _, _ = _c(bad, m)
                assert np.array_equal(got, want), (kind, m)


def test_general_equals_literal_on_stress_histories():
    rng = random.Random(2025)
    for n in (40, 150, 500):
        for p_special in (0.1, 0.4):
            for kinds in (("orphan",), ("non_lamport",), ("nil_cause", "no_root"), X.KINDS):
                nodes = G.stress_history(rng, n, p_special=p_special, p_conj=0.2,
                                         tx_chain=0.1)
                bad = X.corrupt(nodes, rng, kinds, rate=0.05)
                b = pack.pack_lists([bad])
                lit, st1 = oracle.list_weave(b.id_key, b.cause_key, b.kind, oracle.METHOD_LITERAL)
                gen_, st2 = oracle.list_weave(b.id_key, b.cause_key, b.kind, oracle.METHOD_GENERAL)
                assert st1 == st2
                assert np.array_equal(lit, gen_), (n, p_special, kinds)


def test_general_equals_literal_on_corrupted_config2_documents():
    """Packed corruptions of config-2-shaped documents (the GPU tests' inputs)."""
    import dataclasses

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=3000, seed=77)
    off, idk, ck, kd = gen.generate(spec, 0, 10, nthreads=4)
    off, idk, ck, kd = X.corrupt_packed(off, idk, ck, kd, np.random.default_rng(1))
    p1, v1, s1 = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_LITERAL, nthreads=8)
    p2, v2, s2 = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_GENERAL, nthreads=8)
    assert (s1 != 0).all()
    assert np.array_equal(s1, s2)
    assert np.array_equal(p1, p2)
    assert np.array_equal(v1, v2)


def test_in_domain_general_equals_fast_forms():
    """On in-domain histories the general rule reduces to SURVEY F4/F5."""
    rng = random.Random(3)
    for _ in range(40):
        nodes = G.stress_history(rng, 120, p_special=0.3, p_conj=0.2)
        b = pack.pack_lists([nodes])
        g, st = oracle.list_weave(b.id_key, b.cause_key, b.kind, oracle.METHOD_GENERAL)
        e, _ = oracle.list_weave(b.id_key, b.cause_key, b.kind, oracle.METHOD_EFF)
        assert st == 0 and np.array_equal(g, e)
