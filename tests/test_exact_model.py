"""The exact path's rule on CPU (tests/exact_model.py) against the reference
fold, before any GPU: phase 1 (appended nodes placed through the regions of
one static weave, no iteration over them) and phase 2 (insertion-tree rounds
for documents with a non-Lamport cause whose node has an older child).

1. The model's literal fold on ranks is pinned to the C literal fold
   (oracle/weave_oracle.c, clause for clause shared.cljc:194-241) on packed,
   corrupted reference-style histories: order and hide? bits.
2. Phase 1 alone equals the fold on thousands of corrupted rank histories
   without an early node (absent causes, nil causes, no root, specials up to
   90%, hide-of-hide chains).
3. Phase 1 + phase 2 equal the fold on thousands of histories with
   non-Lamport causes (including a node caused by its own id), and the rounds
   stay few at realistic rates.
"""
import random

import numpy as np
import pytest

import oracle
from cause_amd import pack
from oracle import causal_ref as R
from tests import exact_model as M
from tests import outdomain as X
from tests import refgen as G


def _ranks(idk, ck, kd):
    """Packed document -> (par, cls, root, order) on ranks in id order."""
    order = np.argsort(idk, kind="stable")
    sk = idk[order]
    par, cls, root = [], [], []
    for j in order:
        c = ck[j]
        if c == np.uint64((1 << 64) - 1):
            par.append(M.NIL)
        else:
            p = int(np.searchsorted(sk, c))
            par.append(p if p < len(sk) and sk[p] == c else M.END)
        cls.append(int(kd[j]) & 3)
        root.append(bool(int(kd[j]) & 4))
    return par, cls, root, order


@pytest.mark.parametrize("kinds", [("orphan",), ("non_lamport",), ("nil_cause",), ("no_root",),
                                   X.KINDS])
def test_model_fold_matches_c_literal(kinds):
    rng = random.Random(hash(kinds) & 0xFFFF)
    for steps in (5, 12, 40):
        for _ in range(12):
            nodes, _ = G.random_history(rng, steps)
            bad = X.corrupt([R.ROOT_NODE] + nodes, rng, kinds, rate=0.2)
            rng.shuffle(bad)
            b = pack.pack_lists([bad])
            if len(set(b.id_key.tolist())) != len(b.id_key):
                continue  # a repeated id: not a ::nodes map
            want, _ = oracle.list_weave(b.id_key, b.cause_key, b.kind, oracle.METHOD_LITERAL)
            wvis = oracle.list_visible(b.id_key, b.cause_key, b.kind, want)
            par, cls, root, order = _ranks(b.id_key, b.cause_key, b.kind)
            W = M.fold(par, cls)
            assert [int(order[r]) for r in W] == [int(x) for x in want]
            assert M.render(W, par, cls, root) == [bool(v) for v in wvis]
            got, _ = M.exact_weave(par, cls)
            assert got == W


def _random_case(rng, early):
    n = rng.choice((5, 9, 20, 40, 80, 150))
    par, cls = M.random_doc(rng, n, p_special=rng.choice((0.1, 0.3, 0.6, 0.9)),
                            p_hide_of_hide=rng.choice((0.2, 0.7)))
    return M.corrupt(rng, par, cls, p_orphan=rng.choice((0.0, 0.05, 0.2, 0.5, 0.8)),
                     p_nonlamport=rng.choice((0.02, 0.05, 0.2)) if early else 0.0,
                     p_nil=rng.choice((0.0, 0.05)), drop_root=rng.random() < 0.1)


def test_phase1_equals_the_fold_without_early_nodes():
    rng = random.Random(2024)
    checked = 0
    for _ in range(2000):
        par, cls = _random_case(rng, early=False)
        assert not any(M.early_nodes(par))
        assert M.phase1_weave(par, cls) == M.fold(par, cls)
        checked += 1
    assert checked == 2000


def test_phase2_rounds_reach_the_fold():
    rng = random.Random(77)
    with_early = 0
    for _ in range(3000):
        par, cls = _random_case(rng, early=True)
        want = M.fold(par, cls)
        got, rounds = M.exact_weave(par, cls)
        assert got == want
        with_early += any(M.early_nodes(par))
    assert with_early > 1200


def test_rounds_are_few_at_realistic_rates():
    """Long typing histories with 0.1-1% non-Lamport causes and up to 3%
    orphans: phase 1 is already the fold for most, the rest need a few rounds."""
    rng = random.Random(5)
    rounds = []
    for _ in range(24):
        par, cls = M.random_doc(rng, 400, p_special=0.12, p_chain=0.7)
        par, cls = M.corrupt(rng, par, cls, p_orphan=rng.choice((0.002, 0.01, 0.03)),
                             p_nonlamport=rng.choice((0.001, 0.003, 0.01)))
        got, r = M.exact_weave(par, cls)
        assert got == M.fold(par, cls)
        rounds.append(r)
    assert max(rounds) <= 6
    assert np.mean(rounds) <= 2.5


@pytest.mark.parametrize("family", M.CHAIN_FAMILIES)
@pytest.mark.parametrize("n", [300, 4000])
def test_chains_settle_in_log_rounds(family, n):
    """chains of causes through younger nodes (reverse,
    zigzag, interleaved, with specials) took Theta(chain length) rounds with
    round 4's insertion-tree rule (n - 2 on a reverse chain).  With BEFORE
    anchors they settle in at most 2 log2 n + 4 rounds, equal to the fold."""
    import math

    par, cls = M.chain_doc(family, n, random.Random(n))
    got, rounds = M.exact_weave(par, cls, max_rounds=1000)
    assert rounds <= 2 * math.log2(n) + 4, rounds
    assert got == M.fold(par, cls)
