"""A CPU model of the exact path's data-parallel rule (test infrastructure).

The reference folds s/weave-node over (sort ::nodes) whatever the causes are
(list.cljc:26-28 -> shared.cljc:225-241).  This module restates, on ranks in
id order, (a) that fold literally and (b) the rule exact.hip runs on the GPU
for documents outside the fast path's domain, so that the rule can be checked
against the fold on thousands of corrupted histories before (and while) the
kernels implement it.  Nothing in the product imports this.

Inputs, per document, in id order (rank r = position in (sort ::nodes)):
  par[r]  rank of the cause, NIL (nil cause) or END (no node has that id);
          a rank > r is a non-Lamport cause (a younger node);
  cls[r]  0 normal, 1 :causal/hide, 2 :causal/h.hide, 3 :causal/h.show.

The rule (derivation in DESIGN.md section 5f):

Phase 1, orphans without an iteration.  With nodes in id order, a node whose
cause is absent or younger (and which has no older child) is appended: it goes
under T(m), the node last in the weave at that moment.  Every node placed after
an appended node o stays inside the region that o opens, so T of the next
appended node o' depends only on o's region -- not on where o itself went:
  * o non-special: T(o') = the last node older than o' in o's subtree of the
    effective tree (F5);
  * o special: o hides nothing and heads a special run; let N = the nearest
    non-special ancestor of T(o).  The oldest non-special node y in (o, o')
    whose effective parent is N (a non-special node caused through specials
    ends there too) is woven at the end after o's run; T(o') = the last node
    older than o' in y's subtree, or, without such a y, in o's special run.
Both are queries on ONE weave of a static forest in which every appended node
hangs under the head H as a non-special root.  A second weave with every
appended node under its T gives the fold's result.

Phase 2, documents with a non-Lamport cause whose node has an older child
("early" nodes: weave-asap?'s second clause, shared.cljc:199-200).  From any
weave W, `anchors` finds every node's insertion split in W restricted to the
older nodes and names it by a node that does not move from round to round where
it can: BEFORE x (right before x_f, the node's older child woven first) or
AFTER s (right after s: the cause, the end of the special run after it, or the
last older node of an appended node's region).  `build` lays the anchors out
(BEFORE chains under a placeholder at their bottom's place), giving W'.
W' == W holds exactly for the fold's weave and each round fixes at least the
oldest misplaced node; with BEFORE anchors a chain of early nodes (a reverse
chain: node r caused by r + 1) settles in two rounds instead of n - 2.
"""
from __future__ import annotations

import random

NIL = -1
END = -2


# --- the reference fold (shared.cljc:225-241 on ranks) ----------------------

def fold(par, cls):
    """The literal fold: W = []; for each node in id order, weave-node.  Ids of
    woven nodes are smaller than the incoming one, so clauses B and C of
    weave-later? never hold and clause A is special(nr) & cause(nr) != m &
    !special(m)."""
    W = []
    for m in range(len(par)):
        c, sp = par[m], cls[m] != 0
        asap, at = False, len(W)
        for i in range(len(W) + 1):
            nl = W[i - 1] if i > 0 else None
            nr = W[i] if i < len(W) else None
            if not asap:
                asap = (c == NIL and nl is None) or (nl is not None and nl == c) or \
                       (nr is not None and par[nr] == m)
            if nr is None:
                at = i
                break
            if asap and not (cls[nr] != 0 and par[nr] != m and not sp):
                at = i
                break
        W.insert(at, m)
    return W


def render(W, par, cls, root=None):
    """hide? (list.cljc:48-55) on a finished weave: rendered bits by position."""
    out = []
    for i, v in enumerate(W):
        nx = W[i + 1] if i + 1 < len(W) else None
        hid = cls[v] != 0 or (root is not None and root[v]) or \
            (nx is not None and cls[nx] in (1, 2) and par[nx] == v)
        out.append(not hid)
    return out


# --- the effective-tree preorder over a synthetic list -----------

def f5_preorder(spar, scls):
    """Synthetic list: index 0 = H, spar[i] < i (spar[0] unused).  Effective
    parent: a special keeps its parent, a non-special climbs through special
    parents.  Children: specials by descending index, then non-specials."""
    n = len(spar)
    eff = [0] * n
    for i in range(1, n):
        p = spar[i]
        if scls[i] == 0:
            while p != 0 and scls[p] != 0:
                p = spar[p]
        eff[i] = p
    kids = [[] for _ in range(n)]
    for i in range(n - 1, 0, -1):  # descending index
        kids[eff[i]].append(i)
    out, st = [], [0]
    while st:
        v = st.pop()
        out.append(v)
        ks = [k for k in kids[v] if scls[k] != 0] + [k for k in kids[v] if scls[k] == 0]
        st.extend(reversed(ks))
    return out, eff


# --- phase 1 ------------------------------------------------------------------

def appended(par, cls, early):
    """Nodes that weave-asap? never holds for: absent or younger cause and no
    older child.  (Phase 1 treats an early node with such a cause as appended
    too; phase 2 corrects it.)"""
    return [(p == END or (p >= 0 and p >= r)) for r, p in enumerate(par)]


def early_nodes(par):
    e = [False] * len(par)
    for r, p in enumerate(par):
        if p >= 0 and p > r:
            e[p] = True
    return e


class _Weave:
    """Positions of a synthetic weave and the two queries the GPU answers with
    a min-tree over ranks by position."""

    def __init__(self, order, scls):
        self.R = order                      # synthetic index at each position
        self.pos = [0] * len(order)
        for q, s in enumerate(order):
            self.pos[s] = q
        self.scls = scls

    def first_after(self, p, key, v):
        """First q > p with key(q) < v, else len."""
        for q in range(p + 1, len(self.R)):
            if key(q) < v:
                return q
        return len(self.R)

    def last_in(self, lo, hi, v):
        """Last q in [lo, hi) with R[q] < v (the node there), else None."""
        for q in range(hi - 1, lo - 1, -1):
            if self.R[q] < v:
                return self.R[q]
        return None

    def end(self, s):
        """End of s's subtree: its next node in preorder is older (s is
        non-special with non-special ancestors, or a root under H)."""
        return self.first_after(self.pos[s], lambda q: self.R[q], s)

    def end_special(self, s):
        """End of the special children's part of s's subtree."""
        return self.first_after(self.pos[s], lambda q: 0 if self.scls[self.R[q]] == 0 else self.R[q], s)


def phase1(par, cls):
    """Synthetic parents (index r + 1 = rank r, 0 = H) and classes of the final
    F5 weave, plus the static forest used to find them."""
    n = len(par)
    app = appended(par, cls, None)
    spar = [0] * (n + 1)
    scls = [0] * (n + 1)
    for r in range(n):
        p = par[r]
        s = r + 1
        if app[r]:
            spar[s], scls[s] = 0, 0          # a root under H, structurally non-special
        elif p == NIL:
            spar[s], scls[s] = 0, cls[r]
        else:
            spar[s], scls[s] = p + 1, cls[r]
    order, eff = f5_preorder(spar, scls)
    W = _Weave(order, scls)
    sp_orphan = lambda s: s > 0 and app[s - 1] and cls[s - 1] != 0
    Nof = {}

    def nns(s):
        """Nearest non-special ancestor-or-self in the static forest; a special
        appended node stands for its N."""
        while True:
            if s == 0:
                return 0
            if sp_orphan(s):
                return Nof[s]
            if scls[s] == 0:
                return s
            s = spar[s]

    def deff(s):
        """Effective parent of a non-special regular node (climb its cause)."""
        return nns(spar[s]) if spar[s] != 0 else 0

    T = {}
    prev, prev_special = 0, False
    for r in range(n):
        if not app[r]:
            continue
        o = r + 1
        if not prev_special:
            end = W.end(prev) if prev != 0 else len(order)
            t = W.last_in(W.pos[prev], end, o)
            in_run = False
        else:
            N = Nof[prev]
            y = None
            for s in range(prev + 1, o):
                if cls[s - 1] == 0 and not app[s - 1] and deff(s) == N:
                    y = s
                    break
            if y is not None:
                t = W.last_in(W.pos[y], W.end(y), o)
                in_run = False
            else:
                t = W.last_in(W.pos[prev], W.end_special(prev), o)
                in_run = True
        T[o] = t
        if cls[r] != 0:
            Nof[o] = Nof[prev] if in_run else nns(t)
        prev, prev_special = o, cls[r] != 0
    fpar = list(spar)
    fcls = [0] + list(cls)
    for o, t in T.items():
        fpar[o] = t
        if fcls[o] in (1, 2):
            fcls[o] = 3          # an appended hide hides nothing: weaves like an h.show
    return fpar, fcls


def phase1_weave(par, cls):
    fpar, fcls = phase1(par, cls)
    order, _ = f5_preorder(fpar, fcls)
    return [s - 1 for s in order[1:]]


# --- phase 2: anchor rounds (round 5) -----------------------------------------
#
# A node m whose insertion split is right before x_f, the first of its older
# children in the weave (weave-asap?'s second test, shared.cljc:199-200), is
# anchored BEFORE x_f instead of AFTER whatever node precedes x_f in W: that
# node is what changes from round to round along a chain of early nodes (a
# reverse chain, node r caused by r + 1, moved one link a round).  x_f has at
# most one such m (its own cause), so the BEFORE anchors form chains
# m_k -> ... -> m_1 -> b ending in an AFTER-anchored bottom b, and the fold
# lays a chain out as m_k A_k m_(k-1) ... m_1 A_1 b A_b (A_i = m_i's after-
# subtrees).  As a tree with children by descending index: a placeholder P_b
# takes b's place under b's parent (just below b's index) and holds m_k .. m_1
# and b as children, each with its own after-children.

def anchors(W, par, cls, region=False):
    """Anchors of every node from the weave W: ('A', s) = right after synthetic
    s (rank + 1, 0 = H), ('B', x) = right before rank x (its older child)."""
    n = len(par)
    pos = [0] * n
    for q, v in enumerate(W):
        pos[v] = q
    kids = [[] for _ in range(n)]
    for x, p in enumerate(par):
        if p >= 0 and p > x:
            kids[p].append(x)
    out = [None] * n
    prev_app = None
    for m in range(n):
        c, sp = par[m], cls[m] != 0
        older = lambda q: W[q] < m
        xs = [pos[x] for x in kids[m]]
        xf = min(xs) if xs else None
        if c == NIL:
            cp = -1
        elif c >= 0 and c < m:
            cp = pos[c]
        else:
            cp = None
        if cp is None and xf is None:          # appended
            if region and prev_app is not None:
                a = pos[prev_app]
                e = next((q for q in range(a + 1, len(W)) if W[q] < prev_app), len(W))
            else:
                a, e = 0, len(W)
            last = next((q for q in range(e - 1, a - 1, -1) if older(q)), None)
            out[m] = ('A', 0 if last is None else W[last] + 1)
            prev_app = m
            continue
        if cp is not None and (xf is None or cp < xf):
            if sp:                             # right after the cause: no skip
                out[m] = ('A', 0 if c == NIL else c + 1)
                continue
            stop = len(W)
            for q in range(cp + 1, len(W)):
                if not older(q):
                    continue
                v = W[q]
                if cls[v] == 0 or par[v] == m:
                    stop = q
                    break
        else:
            stop = xf
        if xf is not None and stop == xf:
            out[m] = ('B', W[xf])
            continue
        before = next((q for q in range(stop - 1, -1, -1) if older(q)), None)
        out[m] = ('A', 0 if before is None else W[before] + 1)
    return out


def build(anc):
    """The weave of a set of anchors (ranks in order): BEFORE chains under a
    placeholder at their bottom's place, then a plain preorder with children
    by descending key (placeholder of b: key b + 0.5 on the synthetic scale)."""
    n = len(anc)
    bchild = {}
    for m, (t, a) in enumerate(anc):
        if t == 'B':
            assert a not in bchild and a < m
            bchild[a] = m

    def bottom(m):
        while anc[m][0] == 'B':
            m = anc[m][1]
        return m

    kids = {}
    def add(p, key, v):
        kids.setdefault(p, []).append((key, v))
    for m, (t, a) in enumerate(anc):
        s = m + 1
        if t == 'A':
            if m in bchild:               # a chain bottom: its placeholder
                add(a, s - 0.5, ('P', m))
                add(('P', m), s, s)
            else:
                add(a, s, s)
        else:
            add(('P', bottom(m)), s, s)
    out, st = [], [0]
    while st:
        v = st.pop()
        if not isinstance(v, tuple) and v != 0:
            out.append(v - 1)
        ks = sorted(kids.get(v, []), key=lambda kv: -kv[0])
        st.extend(v2 for _, v2 in reversed(ks))
    return out


def exact_weave(par, cls, max_rounds=None):
    """Phase 1, then rounds with BEFORE anchors."""
    W = phase1_weave(par, cls)
    rounds = 0
    if any(early_nodes(par)):
        while True:
            W2 = build(anchors(W, par, cls, region=rounds > 0))
            rounds += 1
            if W2 == W:
                break
            W = W2
            if max_rounds and rounds >= max_rounds:
                break
    return W, rounds


def chain_doc(family, n, rng):
    """Adversarial documents of early nodes: chains of
    causes through younger nodes, as a buggy or malicious site can make them
    (s/insert checks only that the cause exists, shared.cljc:175-178).
      reverse          node r caused by r + 1 (the last by the root)
      reverse_special  the same with random hides / shows in the chain
      zigzag           odd r caused by r + 2 (younger), even r by r - 1
      zigzag_random    causes r + k / r - k for random small k, alternating
      two_reverse      two interleaved reverse chains (r caused by r + 2)
      reverse_hidden   a reverse chain over half the nodes, the rest hides
                       and shows of random chain nodes
      reverse_older    every third node caused by an older node instead
    Rank 0 is the root (nil cause)."""
    par, cls = [NIL], [0]
    for r in range(1, n):
        last = r + 1 >= n
        if family == "reverse" or family == "reverse_special":
            par.append(0 if last else r + 1)
        elif family == "zigzag":
            par.append(r + 2 if r % 2 and r + 2 < n else r - 1)
        elif family == "zigzag_random":
            k = rng.randint(1, 3)
            par.append(min(n - 1, r + k) if r % 2 else max(0, r - k))
        elif family == "two_reverse":
            par.append(r + 2 if r + 2 < n else 0)
        elif family == "reverse_hidden":
            h = n // 2
            par.append((r + 1 if r + 1 < h else 0) if r < h else rng.randrange(1, h))
        elif family == "reverse_older":
            par.append(r - 1 if r % 3 == 0 else (0 if last else r + 1))
        else:
            raise ValueError(family)
        if family == "reverse_special":
            cls.append(rng.choice((0, 0, 1, 2, 3)))
        elif family == "reverse_hidden" and r >= n // 2:
            cls.append(rng.choice((1, 2, 3)))
        else:
            cls.append(0)
    return par, cls


CHAIN_FAMILIES = ("reverse", "reverse_special", "zigzag", "zigzag_random", "two_reverse",
                  "reverse_hidden", "reverse_older")


# --- random documents on ranks ------------------------------------------------

def random_doc(rng, n, p_special=0.15, p_hide_of_hide=0.2, p_chain=0.6, p_conj=0.05):
    """A Lamport-valid history on ranks: rank 0 the root (nil cause)."""
    par, cls = [NIL], [0]
    last_w = 0
    for r in range(1, n):
        u = rng.random()
        specials = [j for j in range(1, r) if cls[j] != 0]
        if u < p_special:
            k = rng.choice((1, 1, 2, 3))
            if specials and rng.random() < p_hide_of_hide:
                c = rng.choice(specials)
            else:
                c = rng.randrange(r)
        else:
            k = 0
            if rng.random() < p_conj:
                c = last_w
            elif rng.random() < p_chain:
                c = r - 1
            else:
                c = rng.randrange(r)
        par.append(c)
        cls.append(k)
        last_w = r
    return par, cls


def corrupt(rng, par, cls, p_orphan=0.05, p_nonlamport=0.0, p_nil=0.0, drop_root=False):
    """Drop nodes (their children's causes become absent), point causes at
    younger nodes, nil causes."""
    n = len(par)
    keep = [True] * n
    for r in range(1, n):
        if rng.random() < p_orphan:
            keep[r] = False
    if drop_root:
        keep[0] = False
    newr = {}
    for r in range(n):
        if keep[r]:
            newr[r] = len(newr)
    P, C = [], []
    for r in range(n):
        if not keep[r]:
            continue
        p = par[r]
        P.append(NIL if p == NIL else (newr[p] if p in newr else END))
        C.append(cls[r])
    m = len(P)
    for r in range(m):
        if rng.random() < p_nonlamport and r + 1 < m:
            P[r] = rng.randrange(r, m)   # r itself: a node caused by its own id
        elif rng.random() < p_nil and r > 0:
            P[r] = NIL
    return P, C


if __name__ == "__main__":
    rng = random.Random(1)
    bad = 0
    for it in range(2000):
        n = rng.choice((5, 9, 20, 40, 80))
        par, cls = random_doc(rng, n, p_special=rng.choice((0.1, 0.3, 0.6)))
        par, cls = corrupt(rng, par, cls, p_orphan=rng.choice((0.0, 0.05, 0.2, 0.5)),
                           p_nonlamport=rng.choice((0.0, 0.0, 0.05, 0.2)),
                           p_nil=rng.choice((0.0, 0.05)), drop_root=rng.random() < 0.1)
        want = fold(par, cls)
        got, rounds = exact_weave(par, cls)
        if got != want:
            bad += 1
            if bad < 5:
                print("MISMATCH", it, par, cls, want, got)
    print("mismatches", bad)
