"""Pure-Python restatement of Cause's causal-tree weave -- TEST INFRASTRUCTURE ONLY.

Used by tests/ as the checker (small cases only: the literal fold is
Theta(n^2) Python).  The product path (cause_amd/) never imports this module.

It restates, on real Clojure-shaped values (ids ``(ts, site, tx)`` with string
site-ids, keyword specials, arbitrary values):

* ``weave_node`` / ``weave_asap`` / ``weave_later``  -- shared.cljc:194-241
* ``insert`` / ``append`` / ``spin`` / ``refresh_ts`` / ``refresh_caches``
  -- shared.cljc:104-192, 243-266
* ``list_weave`` / ``hide_q`` / ``causal_list_to_edn`` / ``causal_list_to_list``
  -- list.cljc:11-72
* ``map_weave`` / ``active_node`` / ``map_get`` / ``map_count`` / ``map_assoc``
  / ``map_dissoc`` / ``causal_map_to_edn`` -- map.cljc:12-109

Clojure semantics kept on purpose: ``compare`` on ids is lexicographic with
Java ``String.compareTo`` (UTF-16 code units) on the site-id (util.cljc:4-10);
``(first nil)`` / ``(second nil)`` / ``(peek nil)`` are ``None``.
"""
from __future__ import annotations

import random


class Keyword:
    """A Clojure keyword ``:ns/name`` (only equality/hash/repr are needed)."""

    __slots__ = ("ns", "name")

    def __init__(self, ns, name):
        self.ns, self.name = ns, name

    def __eq__(self, other):
        return isinstance(other, Keyword) and (self.ns, self.name) == (other.ns, other.name)

    def __hash__(self):
        return hash(("kw", self.ns, self.name))

    def __repr__(self):
        return f":{self.ns}/{self.name}" if self.ns else f":{self.name}"


HIDE = Keyword("causal", "hide")
H_HIDE = Keyword("causal", "h.hide")
H_SHOW = Keyword("causal", "h.show")
SPECIAL = frozenset([HIDE, H_HIDE, H_SHOW])           # shared.cljc:21
ROOT_ID = (0, "0", 0)                                  # shared.cljc:22
ROOT_NODE = (ROOT_ID, None, None)                      # shared.cljc:23
SITE_ID_LENGTH = 13                                    # shared.cljc:25
UUID_LENGTH = 21                                       # shared.cljc:24


def java_str_key(s: str) -> bytes:
    """Sort key equal to Java String.compareTo order (UTF-16 code units)."""
    return s.encode("utf-16-be")


def id_key(i):
    """Sort key of an ::id under clojure.core/compare (vectors of equal length
    compare element-wise; Long, String.compareTo, Long)."""
    ts, site, tx = i
    return (ts, java_str_key(site), tx)


def lt(a, b) -> bool:
    """``(<< a b)`` on ids (util.cljc:4-10)."""
    return id_key(a) < id_key(b)


def is_special(v) -> bool:
    return isinstance(v, Keyword) and v in SPECIAL


def first(x):
    return None if x is None else x[0]


def second(x):
    return None if x is None or len(x) < 2 else x[1]


def peek_node(x):
    """(peek node): the value -- the id itself for weft's one-element [id] node."""
    return None if x is None else x[-1]


def valid_id(x) -> bool:
    """``(spec/valid? ::s/id x)`` -- shared.cljc:31-40."""
    if not (isinstance(x, tuple) and len(x) == 3):
        return False
    ts, site, tx = x
    nat = lambda v: isinstance(v, int) and not isinstance(v, bool) and v >= 0
    return nat(ts) and nat(tx) and isinstance(site, str) and (
        len(site) == SITE_ID_LENGTH or site == "0")


# --------------------------------------------------------------- the weave kernel
def weave_asap(nl, nm, nr) -> bool:
    """shared.cljc:194-200"""
    return first(nl) == second(nm) or first(nm) == second(nr)


def weave_later(nl, nm, nr, seen) -> bool:
    """shared.cljc:202-223"""
    sr = is_special(peek_node(nr))
    sm = is_special(peek_node(nm))
    a = sr and first(nm) != second(nr) and ((not sm) or lt(first(nm), first(nr)))
    b = ((first(nl) == second(nr) or second(nl) == second(nr) or second(nr) in seen)
         and lt(first(nm), first(nr)) and ((not sm) or sr))
    c = lt(first(nm), first(nr)) and ((not sm) or sr)
    return a or b or c


def weave_node(current, node, more=None):
    """shared.cljc:225-241"""
    left_len = 0
    prev_asap = False
    seen = set()
    while True:
        nl = current[left_len - 1] if left_len else None
        right_empty = left_len >= len(current)
        nr = None if right_empty else current[left_len]
        asap = prev_asap or weave_asap(nl, node, nr)
        if right_empty or (asap and not weave_later(nl, node, nr, seen)):
            return current[:left_len] + [node] + list(more or []) + current[left_len:]
        if asap:
            seen.add(first(nl))
        prev_asap = asap
        left_len += 1


# ------------------------------------------------------------------ causal tree
def new_node(ts, site, *rest):
    """shared.cljc:77-84: (ts site cause value) or (ts site tx cause value)."""
    if len(rest) == 2:
        return ((ts, site, 0), rest[0], rest[1])
    tx, cause, value = rest
    return ((ts, site, tx), cause, value)


def _rng_uid(rng, length):
    first_alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
    alpha = "0123456789" + first_alpha
    return rng.choice(first_alpha) + "".join(rng.choice(alpha) for _ in range(length - 1))


def new_site_id(rng=random):
    """util.cljc:15-23 (nano-id over the id alphabet, first char non-digit)."""
    return _rng_uid(rng, SITE_ID_LENGTH)


def new_list_ct(site_id=None, uuid=None, rng=random):
    """list.cljc:11-18"""
    return {"type": "list", "lamport_ts": 0, "uuid": uuid or _rng_uid(rng, UUID_LENGTH),
            "site_id": site_id or new_site_id(rng),
            "nodes": {ROOT_ID: (None, None)},
            "yarns": {"0": [ROOT_NODE]},
            "weave": [ROOT_NODE]}


def new_map_ct(site_id=None, uuid=None, rng=random):
    """map.cljc:12-19"""
    return {"type": "map", "lamport_ts": 0, "uuid": uuid or _rng_uid(rng, UUID_LENGTH),
            "site_id": site_id or new_site_id(rng), "nodes": {}, "yarns": {}, "weave": {}}


def _node_of(i, body):
    """(new-node [k v]) = (into [k] v), shared.cljc:78-79 (body () -> [id])."""
    return (i,) + tuple(body)


def spin_sequential(ct, nodes):
    """shared.cljc:112-119"""
    node = nodes[0]
    site = node[0][1]
    yarns = dict(ct["yarns"])
    yarn = yarns.get(site)
    if yarn:
        if lt(yarn[-1][0], node[0]):
            yarns[site] = yarn + list(nodes)
        else:
            # u/insert with {:uniq true} (util.cljc:25-48): skip if already present
            keys = [id_key(n[0]) for n in yarn]
            k = id_key(node[0])
            lo, hi = 0, len(keys)
            while lo < hi:
                mid = (lo + hi) // 2
                if keys[mid] < k:
                    lo = mid + 1
                else:
                    hi = mid
            if lo < len(yarn) and yarn[lo] == node:
                return ct
            yarns[site] = yarn[:lo] + [node] + list(nodes[1:]) + yarn[lo:]
    else:
        yarns[site] = list(nodes)
    out = dict(ct)
    out["yarns"] = yarns
    return out


def spin(ct, node=None, more=None):
    """shared.cljc:121-149 (the multi-node branch spins node by node: its
    ``is-sequential?`` test is always false)."""
    if node is None:
        out = ct
        for i in sorted(ct["nodes"], key=id_key):
            out = spin_sequential(out, [_node_of(i, ct["nodes"][i])])
        return out
    out = spin_sequential(ct, [node])
    for m in (more or []):
        out = spin_sequential(out, [m])
    return out


def refresh_ts(ct):
    """shared.cljc:243-249"""
    out = dict(ct)
    out["lamport_ts"] = max([0] + [y[-1][0][0] for y in ct["yarns"].values()])
    return out


def refresh_caches(weave_fn, ct):
    """shared.cljc:259-266: spin (over the ct's current yarns), refresh-ts, weave."""
    base = dict(ct)
    base.setdefault("yarns", {})
    return weave_fn(refresh_ts(spin(base)))


def yarns_to_nodes(ct):
    """shared.cljc:251-257"""
    out = dict(ct)
    out["nodes"] = {n[0]: tuple(n[1:]) for y in ct["yarns"].values() for n in y}
    return out


def weft(weave_fn, new_ct_fn, ct, ids):
    """shared.cljc:268-293: each named site's yarn up to and including its cut
    id, then yarns->nodes and the full reweave.  A cut id that is not a node
    keeps the whole yarn (take-while never stops) and adds
    ``(new-node [id nil])`` = ``(into [id] nil)`` = the one-element node [id]."""
    filtered = [i for i in ids if i != ROOT_ID]
    new = new_ct_fn()
    yarns = dict(new["yarns"])
    for i in filtered:
        pre = []
        for n in ct["yarns"].get(i[1], []):
            if n[0] == i:
                break
            pre.append(n)
        body = ct["nodes"].get(i)
        pre.append(_node_of(i, body if body is not None else ()))
        yarns[i[1]] = pre
    new["yarns"] = yarns
    new["site_id"] = ct["site_id"]
    new["lamport_ts"] = max(i[0] for i in filtered)
    return weave_fn(yarns_to_nodes(new))


class CauseError(Exception):
    def __init__(self, msg, causes):
        super().__init__(msg)
        self.causes = causes


def insert(weave_fn, ct, node, more=None):
    """shared.cljc:151-184"""
    nodes = [node] + list(more or [])
    txs = {(n[0][0], n[0][1]) for n in nodes}
    if len(txs) > 1:
        raise CauseError("All nodes must belong to the same tx.", {"txs"})
    existing = ct["nodes"].get(node[0])
    if existing is not None:
        if (node[1], node[2]) == existing:
            return ct
        raise CauseError("This node is already in the tree and can't be changed.",
                         {"append-only", "edits-not-allowed"})
    is_key = isinstance(node[1], (Keyword, str))
    if not is_key and node[1] not in ct["nodes"]:
        raise CauseError("The cause of this node is not in the tree.", {"cause-must-exist"})
    out = dict(ct)
    if node[0][0] > ct["lamport_ts"]:
        out["lamport_ts"] = node[0][0]
    nm = dict(out["nodes"])
    for n in nodes:
        nm[n[0]] = (n[1], n[2])
    out["nodes"] = nm
    out = spin(out, node, more)
    return weave_fn(out, node, more)


def append(weave_fn, ct, cause, value):
    """shared.cljc:186-192"""
    ct2 = dict(ct)
    ct2["lamport_ts"] = ct["lamport_ts"] + 1
    return insert(weave_fn, ct2, new_node(ct2["lamport_ts"], ct2["site_id"], cause, value))


def merge_trees(weave_fn, ct1, ct2, rng=None):
    """shared.cljc:300-314 (reduce insert over ct2's nodes; ``rng`` shuffles
    the hash-map order)."""
    if ct1["type"] != ct2["type"]:
        raise CauseError("Causal type missmatch. Merge not allowed.", {"type-missmatch"})
    if ct1["uuid"] != ct2["uuid"]:
        raise CauseError("Causal UUID missmatch. Merge not allowed.", {"uuid-missmatch"})
    items = list(ct2["nodes"].items())
    if rng is not None:
        rng.shuffle(items)
    out = ct1
    for i, body in items:
        out = insert(weave_fn, out, _node_of(i, body))
    return out


# ------------------------------------------------------------------------ lists
def list_weave(ct, node=None, more=None):
    """list.cljc:20-34"""
    if node is None:
        out = dict(ct)
        w = []
        for i in sorted(ct["nodes"], key=id_key):
            w = weave_node(w, _node_of(i, ct["nodes"][i]))
        out["weave"] = w
        return out
    if node[0] not in ct["nodes"]:
        return ct
    out = dict(ct)
    out["weave"] = weave_node(ct["weave"], node, more)
    return out


def hide_q(node, nxt) -> bool:
    """list.cljc:48-55"""
    return (is_special(peek_node(node))
            or ((peek_node(nxt) == HIDE or peek_node(nxt) == H_HIDE)
                and first(node) == second(nxt))
            or node == ROOT_NODE)


def causal_to_edn(v):
    """shared.cljc:320-328 (nested causal values are opaque here)."""
    if isinstance(v, dict) and "type" in v and "weave" in v:
        return causal_list_to_edn(v) if v["type"] == "list" else causal_map_to_edn(v)
    return v


def causal_list_to_edn(ct):
    """list.cljc:57-66"""
    w = ct["weave"]
    return [causal_to_edn(peek_node(n)) for k, n in enumerate(w)
            if not hide_q(n, w[k + 1] if k + 1 < len(w) else None)]


def causal_list_to_list(ct):
    """list.cljc:68-72"""
    w = ct["weave"]
    return [n for k, n in enumerate(w) if not hide_q(n, w[k + 1] if k + 1 < len(w) else None)]


def list_conj(ct, v):
    """list.cljc:36-40: append with cause = id of the LAST weave node."""
    return append(list_weave, ct, ct["weave"][-1][0], v)


def list_cons(v, ct):
    """list.cljc:42-43"""
    return append(list_weave, ct, ROOT_ID, v)


# ------------------------------------------------------------------------- maps
def map_weave(ct, node=None, more=None):
    """map.cljc:21-45"""
    if node is None:
        out = dict(ct)
        out["weave"] = {}
        for i in sorted(ct["nodes"], key=id_key):
            out = map_weave(out, _node_of(i, ct["nodes"][i]))
        return out
    i, cause, v = node
    cause_is_id = valid_id(cause)
    if cause_is_id:
        body = ct["nodes"].get(cause)
        key = None if body is None else body[0]
    else:
        key = cause
    cause_in_weave = cause if cause_is_id else ROOT_ID
    if i not in ct["nodes"]:
        return ct
    kw = ct["weave"].get(key) or [ROOT_NODE]
    kw = weave_node(kw, (i, cause_in_weave, v))
    out = dict(ct)
    w = dict(ct["weave"])
    w[key] = kw
    out["weave"] = w
    if more:
        return map_weave(out, more[0], more[1:] or None)
    return out


BLANK = object()


def active_node(k, wk):
    """map.cljc:47-59"""
    wk = wk or []
    first_v = wk[1][2] if len(wk) > 1 else None
    if first_v == HIDE or first_v == H_HIDE:
        return BLANK
    for idx, n in enumerate(wk):
        nr_v = wk[idx + 1][2] if idx + 1 < len(wk) else None
        if n[0] == ROOT_ID:
            continue
        if is_special(n[2]):
            continue
        if nr_v == HIDE or nr_v == H_HIDE:
            continue
        return (n[0], k, n[2])
    return BLANK


def map_get(ct, k):
    """map.cljc:61-66"""
    n = active_node(k, ct["weave"].get(k))
    return None if n is BLANK else n[2]


def map_count(ct):
    """map.cljc:68-73"""
    return sum(1 for k, wk in ct["weave"].items() if active_node(k, wk) is not BLANK)


def map_assoc(ct, k, v):
    """map.cljc:75-81"""
    if v != map_get(ct, k):
        return append(map_weave, ct, k, v)
    return ct


def map_dissoc(ct, k):
    """map.cljc:83-89"""
    v = map_get(ct, k)
    if v is not None and v is not False:   # Clojure truthiness
        return append(map_weave, ct, k, HIDE)
    return ct


def causal_map_to_edn(ct):
    """map.cljc:94-103"""
    out = {}
    for k, wk in ct["weave"].items():
        n = active_node(k, wk)
        if n is not BLANK:
            out[n[1]] = causal_to_edn(n[2])
    return out


def causal_map_to_list(ct):
    """map.cljc:105-109"""
    return [n for k, wk in ct["weave"].items()
            for n in [active_node(k, wk)] if n is not BLANK]
