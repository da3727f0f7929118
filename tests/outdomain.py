"""Documents outside the fast path's domain (test inputs only).

The reference's full reweave (list.cljc:26-28 -> shared.cljc:225-241) accepts
any bag of nodes; these generators break the fast path's assumptions on
purpose, the ways a reconstituted ::nodes map can:

* ``orphan``      -- nodes deleted from the bag, so their children's causes are
                     absent (the (empty? right) append, shared.cljc:236-238);
* ``non_lamport`` -- a cause that is a node with a larger id;
* ``nil_cause``   -- a non-root node whose cause is nil;
* ``no_root``     -- the root [[0 "0" 0] nil nil] missing;
* ``low_root``    -- nodes whose ids sort before the root (ts 0, a site-id
                     below "0" in String.compareTo order);
* ``key_cause``   -- a cause that is not an id at all (a keyword-like string).

Clojure-shaped (``corrupt``) for the Python restatement, and packed
(``corrupt_packed``) for batches from the generator.
"""
from __future__ import annotations

import numpy as np

from oracle import causal_ref as R

KINDS = ("orphan", "non_lamport", "nil_cause", "no_root", "low_root", "key_cause")


def corrupt(nodes, rng, kinds=KINDS, rate=0.1):
    """A copy of ``nodes`` (root first, Clojure-shaped) broken in the given ways."""
    nodes = list(nodes)
    n = len(nodes)
    k = max(1, int(rate * n))
    if "orphan" in kinds and n > 3:
        drop = set(rng.sample(range(1, n), min(k, n - 2)))
        nodes = [nd for j, nd in enumerate(nodes) if j not in drop]
    if "non_lamport" in kinds and len(nodes) > 3:
        ids = sorted((nd[0] for nd in nodes), key=R.id_key)
        for _ in range(k):
            j = rng.randrange(1, len(nodes))
            i, c, v = nodes[j]
            later = [x for x in ids if R.lt(i, x)]
            if later:
                nodes[j] = (i, rng.choice(later), v)
    if "nil_cause" in kinds and len(nodes) > 2:
        for _ in range(max(1, k // 3)):
            j = rng.randrange(1, len(nodes))
            nodes[j] = (nodes[j][0], None, nodes[j][2])
    if "key_cause" in kinds and len(nodes) > 2:
        j = rng.randrange(1, len(nodes))
        nodes[j] = (nodes[j][0], "some-key", nodes[j][2])
    if "low_root" in kinds:
        nodes.append(((0, " a ", 0), R.ROOT_ID, "<"))
        nodes.append(((0, " b ", 0), (0, " a ", 0), R.HIDE))
    if "no_root" in kinds:
        nodes = [nd for nd in nodes if nd[0] != R.ROOT_ID]
    return nodes


def corrupt_packed(off, idk, ck, kd, rng, rate=0.02, which=None):
    """Break documents of a packed batch in place (each document gets one of
    the packed-level corruptions, or ``which``): absent causes, causes with a
    larger id, nil causes, no root.  Returns the new (off, idk, ck, kd)."""
    NIL = np.uint64((1 << 64) - 1)
    outs = []
    D = len(off) - 1
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        i, c, k = idk[a:b].copy(), ck[a:b].copy(), kd[a:b].copy()
        w = which or ["orphan", "non_lamport", "nil_cause", "no_root", "mixed"][d % 5]
        m = max(1, int(rate * len(i)))
        nonroot = np.flatnonzero((k & 4) == 0)
        if w in ("orphan", "mixed") and len(nonroot) > 2:
            keep = np.ones(len(i), bool)
            keep[rng.choice(nonroot, min(m, len(nonroot) - 1), replace=False)] = False
            i, c, k = i[keep], c[keep], k[keep]
            nonroot = np.flatnonzero((k & 4) == 0)
        if w in ("non_lamport", "mixed") and len(nonroot) > 2:
            js = rng.choice(nonroot, m)
            srt = np.sort(i)
            for j in js:
                pos = np.searchsorted(srt, i[j], side="right")
                if pos < len(srt):
                    c[j] = srt[rng.integers(pos, len(srt))]
        if w in ("nil_cause", "mixed") and len(nonroot) > 2:
            c[rng.choice(nonroot, max(1, m // 4))] = NIL
        if w == "no_root":
            keep = (k & 4) == 0
            i, c, k = i[keep], c[keep], k[keep]
        outs.append((i, c, k))
    noff = np.zeros(D + 1, np.uint64)
    noff[1:] = np.cumsum([len(o[0]) for o in outs])
    cat = lambda j, dt: np.concatenate([o[j] for o in outs]) if outs else np.zeros(0, dt)
    return noff, cat(0, np.uint64), cat(1, np.uint64), cat(2, np.uint8)
