"""Host-side mirror of the reference's list interface, with the weave on the GPU.

Same names, argument meaning and errors as the reference (causal.collections.
shared / list); a causal tree is a dict with the reference's ct keys
(``nodes``, ``yarns``, ``weave``, ``lamport_ts``, ``site_id``, ``uuid``, ``type``).
Every ``weave`` arity is a full reweave on the MI355X through the C ABI
(cw_weave_lists) -- exact by SURVEY F7 (incremental insertion in any causal
order equals the full reweave).  There is no CPU weave in this module.

    shared.cljc:151-192   insert / append           -> insert, append, insert_bulk
    shared.cljc:300-314   merge-trees               -> merge_trees / merge_lists (cw_merge_lists)
    shared.cljc:268-293   weft                      -> weft / weft_lists (cw_weft_lists)
    shared.cljc:259-266   refresh-caches            -> refresh_caches
    list.cljc:20-34       weave (all arities)       -> list_weave / weave_lists
    list.cljc:36-43       conj- / cons-             -> list_conj / list_cons
    list.cljc:48-72       hide? / ->edn / ->list    -> causal_list_to_edn / _to_list
"""
from __future__ import annotations

import random
import threading

import numpy as np

from . import abi, pack


class Keyword:
    """A Clojure keyword ``:ns/name``."""

    __slots__ = ("ns", "name")

    def __init__(self, ns, name):
        self.ns, self.name = ns, name

    def __eq__(self, other):
        return (getattr(other, "ns", None), getattr(other, "name", None)) == (self.ns, self.name) \
            and hasattr(other, "ns")

    def __hash__(self):
        return hash(("kw", self.ns, self.name))

    def __repr__(self):
        return f":{self.ns}/{self.name}" if self.ns else f":{self.name}"


HIDE = Keyword("causal", "hide")          # core.cljc:15
H_HIDE = Keyword("causal", "h.hide")
H_SHOW = Keyword("causal", "h.show")
ROOT_ID = (0, "0", 0)                      # shared.cljc:22
ROOT_NODE = (ROOT_ID, None, None)          # shared.cljc:23


class CauseError(Exception):
    """ex-info of the reference: ``causes`` is the :causes set."""

    def __init__(self, msg, causes):
        super().__init__(msg)
        self.causes = causes


_local = threading.local()


def weaver() -> abi.Weaver:
    """This thread's GPU context (device 0).  A cw_ctx is not thread-safe
    (include/causeweave.h), and swap! may run a weave-fn on several threads at
    once: each host thread gets its own context, so calls never share one."""
    w = getattr(_local, "weaver", None)
    if w is None:
        w = _local.weaver = abi.Weaver(0)
    return w


def causal_to_edn(v):
    """s/causal->edn (shared.cljc:320-328): a causal collection (a list or map
    ct held as a value) materialises recursively, anything else is itself."""
    if isinstance(v, dict) and v.get("type") in ("list", "map") and "weave" in v:
        return causal_list_to_edn(v) if v["type"] == "list" else causal_map_to_edn(v)
    return v


def new_node(ts, site, *rest):
    """shared.cljc:77-84"""
    if len(rest) == 2:
        return ((ts, site, 0), rest[0], rest[1])
    tx, cause, value = rest
    return ((ts, site, tx), cause, value)


def _uid(rng, n):
    first = "ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
    return rng.choice(first) + "".join(rng.choice("0123456789" + first) for _ in range(n - 1))


def new_site_id(rng=random):
    return _uid(rng, 13)


def new_list_ct(site_id=None, uuid=None, rng=random):
    """list.cljc:11-18"""
    return {"type": "list", "lamport_ts": 0, "uuid": uuid or _uid(rng, 21),
            "site_id": site_id or new_site_id(rng),
            "nodes": {ROOT_ID: (None, None)}, "yarns": {"0": [ROOT_NODE]},
            "weave": [ROOT_NODE], "_visible": [False]}


def weave_lists(cts):
    """Full reweave of many list cts in ONE GPU call (the batch entry point).
    Returns new cts with ::weave, ::yarns, ::lamport-ts and rendered flags."""
    docs = [[(i, b[0], b[1]) for i, b in ct["nodes"].items()] for ct in cts]
    try:
        b = pack.pack_lists(docs)
        res = weaver().weave_lists(b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    except pack.KeyRangeError:  # ids over 63 bits: the K128 layout
        b = pack.pack_lists_k128(docs)
        res = weaver().weave_lists_k128(b.offsets, b.id_key, b.cause_key, b.kind)
    vis = res.visible()
    out = []
    for d, (ct, nodes) in enumerate(zip(cts, docs)):
        lo, hi = int(b.offsets[d]), int(b.offsets[d + 1])
        st = int(res.status[d])
        # c.list/weave's full reweave never throws: absent / non-Lamport / nil
        # causes and a missing root get the literal fold's weave (the library's
        # exact path); only a repeated id is impossible for a ::nodes map
        if st & (abi.STATUS_DUP | abi.STATUS_INTERNAL):
            raise CauseError(f"document outside the weave's domain (status {st})", {"weave-domain"})
        new = dict(ct)
        new["weave"] = [nodes[p] for p in res.weave_perm[lo:hi]]
        new["_visible"] = [bool(v) for v in vis[lo:hi]]
        yarns = {}
        if res.yarn_perm is not None:
            for p in res.yarn_perm[lo:hi]:
                nd = nodes[p]
                yarns.setdefault(nd[0][1], []).append(nd)
        new["yarns"] = yarns
        new["_max_ts"] = int(res.max_ts[d])
        out.append(new)
    return out


def list_weave(ct, node=None, more=None):
    """list.cljc:20-34 -- every arity is the full GPU reweave;
    like the reference, a node that is not in ::nodes leaves ct unchanged."""
    if node is not None and node[0] not in ct["nodes"]:
        return ct
    return weave_lists([ct])[0]


def refresh_caches(weave_fn, ct):
    """shared.cljc:259-266: yarns (spin), lamport-ts (refresh-ts) and the weave
    all come from the one GPU call."""
    out = weave_fn(ct)
    out = dict(out)
    out["lamport_ts"] = out.get("_max_ts", ct["lamport_ts"])
    return out


def insert(weave_fn, ct, node, more=None):
    """shared.cljc:151-184 (same validations, same ex-info causes)."""
    nodes = [node] + list(more or [])
    if len({(n[0][0], n[0][1]) for n in nodes}) > 1:
        raise CauseError("All nodes must belong to the same tx.", {"txs"})
    existing = ct["nodes"].get(node[0])
    if existing is not None:
        if (node[1], node[2]) == existing:
            return ct
        raise CauseError("This node is already in the tree and can't be changed.",
                         {"append-only", "edits-not-allowed"})
    is_key = isinstance(node[1], (str, Keyword))
    if not is_key and node[1] not in ct["nodes"]:
        raise CauseError("The cause of this node is not in the tree.", {"cause-must-exist"})
    out = dict(ct)
    if node[0][0] > ct["lamport_ts"]:
        out["lamport_ts"] = node[0][0]
    nm = dict(ct["nodes"])
    for n in nodes:
        nm[n[0]] = (n[1], n[2])
    out["nodes"] = nm
    woven = weave_fn(out, node, more)
    woven = dict(woven)
    woven["lamport_ts"] = out["lamport_ts"]
    return woven


class _Tokens:
    """Value identity for the merge's body check (equal values <=> equal token)."""

    def __init__(self):
        self.t = {}

    def __call__(self, v):
        try:
            key = ("h", type(v).__name__, v)
            hash(key)
        except TypeError:
            key = ("r", repr(v))
        return self.t.setdefault(key, len(self.t))


def merge_lists(pairs):
    """s/merge-trees (shared.cljc:300-314) for many (ct1, ct2) list pairs in ONE
    GPU call (cw_merge_lists): the union of the two ::nodes maps, deduplicated,
    then the full reweave.  Same checks and ex-info causes as the
    reference; see include/causeweave.h for the one divergence (the reference
    can also throw :cause-must-exist because of its hash-map insertion order)."""
    for ct1, ct2 in pairs:
        if ct1["type"] != ct2["type"]:
            raise CauseError("Causal type missmatch. Merge not allowed.", {"type-missmatch"})
        if ct1["uuid"] != ct2["uuid"]:
            raise CauseError("Causal UUID missmatch. Merge not allowed.", {"uuid-missmatch"})
    da = [[(i, b[0], b[1]) for i, b in ct1["nodes"].items()] for ct1, _ in pairs]
    db = [[(i, b[0], b[1]) for i, b in ct2["nodes"].items()] for _, ct2 in pairs]
    pk = pack.pack_lists([a + b for a, b in zip(da, db)])  # one site ranking per pair
    tok = _Tokens()
    ia, ib = [], []
    for d, (a, b) in enumerate(zip(da, db)):
        lo = int(pk.offsets[d])
        ia.append(np.arange(lo, lo + len(a)))
        ib.append(np.arange(lo + len(a), lo + len(a) + len(b)))
    ia = np.concatenate(ia) if ia else np.zeros(0, np.int64)
    ib = np.concatenate(ib) if ib else np.zeros(0, np.int64)
    vals = np.array([tok(n[2]) for d in pk.docs for n in d.nodes], np.uint64)
    off_a = np.zeros(len(pairs) + 1, np.uint64)
    off_a[1:] = np.cumsum([len(a) for a in da])
    off_b = np.zeros(len(pairs) + 1, np.uint64)
    off_b[1:] = np.cumsum([len(b) for b in db])
    side = lambda idx, off: (off, pk.id_key[idx], pk.cause_key[idx], pk.kind[idx], vals[idx])
    res = weaver().merge_lists(side(ia, off_a), side(ib, off_b), pk.layout)
    vis = res.weave.visible()
    out = []
    for d, ((ct1, ct2), a, b) in enumerate(zip(pairs, da, db)):
        st = int(res.weave.status[d])
        if st & abi.STATUS_DUP:
            raise CauseError("This node is already in the tree and can't be changed.",
                             {"append-only", "edits-not-allowed"})
        if st & abi.STATUS_ORPHAN:
            raise CauseError("The cause of this node is not in the tree.", {"cause-must-exist"})
        if st:
            raise CauseError(f"document outside the weave's domain (status {st})", {"weave-domain"})
        lo, hi = int(res.offsets[d]), int(res.offsets[d + 1])
        src = res.src[lo:hi]
        node_of = lambda s: a[s] if s < len(a) else b[s - len(a)]
        merged = [node_of(int(s)) for s in src]
        new = dict(ct1)
        new["nodes"] = {n[0]: (n[1], n[2]) for n in merged}
        new["weave"] = [merged[p] for p in res.weave.weave_perm[lo:hi]]
        new["_visible"] = [bool(v) for v in vis[lo:hi]]
        yarns = {}
        for p in res.weave.yarn_perm[lo:hi]:
            nd = merged[p]
            yarns.setdefault(nd[0][1], []).append(nd)
        new["yarns"] = yarns
        # insert fast-forwards ::lamport-ts to every newly inserted node (shared.cljc:179-181)
        fresh = [merged[i][0][0] for i, s in enumerate(src) if s >= len(a)]
        new["lamport_ts"] = max([ct1["lamport_ts"]] + fresh)
        new["_max_ts"] = int(res.weave.max_ts[d])
        out.append(new)
    return out


def merge_trees(weave_fn, ct1, ct2):
    """shared.cljc:300-314 (lists; the weave-fn is the GPU weave)."""
    return merge_lists([(ct1, ct2)])[0]


def insert_bulk(ct, nodes):
    """Many s/insert calls (shared.cljc:151-184) in causal order, as one GPU
    merge of ``nodes`` into ``ct``."""
    ct2 = dict(ct)
    ct2["nodes"] = {n[0]: (n[1], n[2]) for n in nodes}
    return merge_trees(list_weave, ct, ct2)


def weft_lists(items):
    """s/weft (shared.cljc:268-293) for many (ct, ids-to-cut-yarns) list pairs in
    ONE GPU call (cw_weft_lists): time travel to the cut, then the full reweave.
    A cut id that is not a node keeps its site's whole yarn plus the
    one-element node ``(id,)`` (``(new-node [id nil])``), last in that yarn."""
    docs = [[(i, b[0], b[1]) for i, b in ct["nodes"].items()] for ct, _ in items]
    cuts = []
    for ct, ids in items:
        last = {}
        for i in ids:  # (assoc-in [::yarns site] ..): the last id of a site wins
            if i != ROOT_ID:
                last[i[1]] = i
        cuts.append(last)
    pk = pack.pack_lists(docs, min_site_bits=1,  # cw_weft_lists indexes cuts by site rank
                         extra_ids=[list(c.values()) for c in cuts])
    lay = pk.layout
    S = 1 << lay.site_bits
    cut = np.zeros(len(items) << lay.site_bits, np.uint64)
    for d, (last, pd) in enumerate(zip(cuts, pk.docs)):
        for site, i in last.items():
            cut[d * S + pd.site_rank[site]] = lay.pack(i[0], pd.site_rank[site], i[2])
    res = weaver().weft_lists(pk.offsets, pk.id_key, pk.cause_key, pk.kind, lay, cut)
    vis = res.weave.visible()
    out = []
    for d, ((ct, ids), nodes, last, pd) in enumerate(zip(items, docs, cuts, pk.docs)):
        st = int(res.weave.status[d])
        if st & (abi.STATUS_DUP | abi.STATUS_INTERNAL):
            raise CauseError(f"weft outside the weave's domain (status {st})", {"weave-domain"})
        lo, hi = int(res.offsets[d]), int(res.offsets[d + 1])
        # the [id] nodes come after the kept nodes, in site-rank order
        bogus = iter(sorted((i for i in last.values() if i not in ct["nodes"]),
                            key=lambda i: pd.site_rank[i[1]]))
        kept = [nodes[s] if s != 0xFFFFFFFF else (next(bogus),) for s in res.src[lo:hi]]
        new = new_list_ct(site_id=ct["site_id"], uuid=ct["uuid"])
        new["nodes"] = {n[0]: tuple(n[1:]) for n in kept}
        new["weave"] = [kept[p] for p in res.weave.weave_perm[lo:hi]]
        new["_visible"] = [bool(v) for v in vis[lo:hi]]
        yarns = {}
        for p in res.weave.yarn_perm[lo:hi]:
            yarns.setdefault(kept[p][0][1], []).append(kept[p])
        for y in yarns.values():  # (conj yarn-prefix [id]): the [id] node is last
            y.sort(key=lambda n: len(n) == 1)
        new["yarns"] = yarns
        new["lamport_ts"] = max(i[0] for i in ids if i != ROOT_ID)
        out.append(new)
    return out


def weft(ct, ids):
    """(c/weft causal-list ids) -- list.cljc:165-166 over shared.cljc:268-293."""
    return weft_lists([(ct, ids)])[0]


def append(weave_fn, ct, cause, value):
    """shared.cljc:186-192"""
    ct2 = dict(ct)
    ct2["lamport_ts"] = ct["lamport_ts"] + 1
    return insert(weave_fn, ct2, new_node(ct2["lamport_ts"], ct2["site_id"], cause, value))


def list_conj(ct, v):
    """list.cljc:36-40"""
    return append(list_weave, ct, ct["weave"][-1][0], v)


def list_cons(v, ct):
    """list.cljc:42-43"""
    return append(list_weave, ct, ROOT_ID, v)


def causal_list_to_list(ct):
    """list.cljc:68-72 (rendered flags from the GPU, hide? list.cljc:48-55)."""
    return [n for n, v in zip(ct["weave"], ct["_visible"]) if v]


def causal_list_to_edn(ct):
    """list.cljc:57-66: (peek node) of every rendered node, nested causal
    values materialised (s/causal->edn, list.cljc:64-66)"""
    return [causal_to_edn(n[-1]) for n in causal_list_to_list(ct)]


def count(ct):
    """list.cljc:77"""
    return len(causal_list_to_list(ct))


# ------------------------------------------------------------------------- maps
# map.cljc: the map interface over cw_weave_maps.  A map ct's ``weave`` is
# {key: key weave (root first)}; ``_active`` is {key: active node or BLANK}.
BLANK = Keyword("causal.collections.map", "blank")   # ::blank, map.cljc:52


def new_map_ct(site_id=None, uuid=None, rng=random):
    """map.cljc:12-19"""
    return {"type": "map", "lamport_ts": 0, "uuid": uuid or _uid(rng, 21),
            "site_id": site_id or new_site_id(rng), "nodes": {}, "yarns": {}, "weave": {},
            "_active": {}}


def _unpack_id(key, layout, rank):
    if key == 0:
        return ROOT_ID  # the virtual root packs to 0 (pack.pack_maps)
    inv = {r: s for s, r in rank.items()}
    ts = key >> layout.ts_shift
    site = (key >> layout.site_shift) & ((1 << layout.site_bits) - 1)
    tx = key & ((1 << layout.tx_bits) - 1)
    return (ts, inv[site], tx)


def weave_maps(cts):
    """Full reweave of many map cts in ONE GPU call (c.map/weave 1-arity,
    map.cljc:21-28, for each); also computes active-node per key."""
    docs = [[(i, b[0], b[1]) for i, b in ct["nodes"].items()] for ct in cts]
    pm = pack.pack_maps(docs)
    res = weaver().weave_maps(pm.offsets, pm.id_key, pm.cause, pm.cause_is_id, pm.kind,
                              pm.token_bits, pm.layout.key_bits)
    out = []
    segs_of = {}
    for s, d in enumerate(res.seg_coll.tolist()):
        segs_of.setdefault(d, []).append(s)
    for d, (ct, nodes) in enumerate(zip(cts, docs)):
        st = int(res.status[d])
        # non-Lamport causes and causes that are not nodes are the literal
        # fold's (the library's fused map path); a repeated id, a key token
        # out of range or an internal check are not a ::nodes map it weaves
        if st & (abi.STATUS_DUP | abi.STATUS_MAP_KEY | abi.STATUS_INTERNAL):
            raise CauseError(f"map outside the weave's domain (status {st})", {"weave-domain"})
        weave, active = {}, {}
        for s in segs_of.get(d, []):
            k = int(res.seg_key[s])
            if k == pack.NIL:
                key = None
            elif k >> 63:
                key = _unpack_id(k & ((1 << 63) - 1), pm.layout, pm.ranks[d])
            else:
                key = pm.keys[k]
            # nodes are woven as [id cause-in-weave v] (map.cljc:35-41)
            weave[key] = [ROOT_NODE] + [
                (nodes[p][0], nodes[p][1] if pack.valid_id(nodes[p][1]) else ROOT_ID, nodes[p][2])
                for p in res.key_weave(s)[1:]]
            a = int(res.seg_active[s])
            active[key] = BLANK if a < 0 else (nodes[a][0], key, nodes[a][2])
        new = dict(ct)
        new["weave"] = weave
        new["_active"] = active
        out.append(new)
    return out


def map_weave(ct, node=None, more=None):
    """map.cljc:21-45 -- every arity is the full GPU reweave."""
    if node is not None and node[0] not in ct["nodes"]:
        return ct
    return weave_maps([ct])[0]


def active_node(ct, k):
    """map.cljc:47-59 (computed on the GPU with the weave)."""
    return ct["_active"].get(k, BLANK)


def map_get(ct, k):
    """map.cljc:61-66"""
    n = active_node(ct, k)
    return None if n is BLANK else n[2]


def map_count(ct):
    """map.cljc:68-73"""
    return sum(1 for n in ct["_active"].values() if n is not BLANK)


def map_assoc(ct, k, v):
    """map.cljc:75-81"""
    if v != map_get(ct, k):
        return append(map_weave, ct, k, v)
    return ct


def map_dissoc(ct, k):
    """map.cljc:83-89"""
    v = map_get(ct, k)
    if v is not None and v is not False:
        return append(map_weave, ct, k, HIDE)
    return ct


def causal_map_to_edn(ct):
    """map.cljc:94-103: the active value of every key, nested causal values
    materialised (s/causal->edn, map.cljc:101)."""
    return {n[1]: causal_to_edn(n[2]) for n in ct["_active"].values() if n is not BLANK}


def causal_map_to_list(ct):
    """map.cljc:105-109"""
    return [n for n in ct["_active"].values() if n is not BLANK]
