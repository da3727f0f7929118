"""Host mirror of CausalBase materialisation, with the
weaves and the history sort on the MI355X.

A causal base (base/core.cljc) keeps nested collections flat: every nested
list or map is its own causal collection and the parent holds a ref keyword
``:causal.collection.ref/<uuid>``.  What touches node data here goes through the
C ABI in batches:

  * ``cb_to_edn`` (base/core.cljc:92-96, with the ref resolution of :83-90):
    every collection is rewoven in ONE cw_weave_lists call (all lists) and ONE
    cw_weave_maps call (all maps), then the refs are resolved on the host;
  * ``history`` (the ``::history`` sorted log, :107-115): the reverse paths
    ``[id uuid]`` of every insertion sorted by id with cw_sort_keys (the
    reference keeps the vector sorted by one binary-search insertion each).

The transaction bookkeeping (``transact_``, ``flatten_value``, ``map_to_nodes``,
``list_to_nodes``, :117-268) is host logic that only builds nodes; it follows
the reference clause by clause and defers the weave: collections are woven
when materialised (insertion in any causal order equals the full
reweave), with the insert-time checks of s/insert kept.
"""
from __future__ import annotations

import random

import numpy as np

from . import abi, causal as C, pack

REF_NS = "causal.collection.ref"      # base/core.cljc:57


class Char(str):
    """A Clojure character (``\\a``): one element of a string woven as a list."""

    __slots__ = ()

    def __repr__(self):
        return "\\" + str.__str__(self)


def _no_weave(ct, node=None, more=None):
    return ct


def new_cb(rng=random):
    """base/core.cljc:39-53"""
    return {"lamport_ts": 1, "uuid": C._uid(rng, 21), "site_id": C.new_site_id(rng),
            "history": [], "root_uuid": None, "collections": {}, "_rng": rng}


def uuid_to_ref(uuid):
    return C.Keyword(REF_NS, uuid)      # :59-60


def is_ref(v):
    return isinstance(v, C.Keyword) and v.ns == REF_NS     # :65-66


def ref_to_uuid(ref):
    return ref.name                     # :68-69


def _is_map(v):
    return isinstance(v, dict)


def _seqable(v):
    """clojure.core/seqable? for the values a transaction carries (nil is
    seqable; a character is not)."""
    if isinstance(v, Char):
        return False
    return v is None or isinstance(v, (str, list, tuple))


def new_node(cb, tx_index, cause, value):
    """:100-105 -> (tx_index + 1, node)"""
    return tx_index + 1, ((cb["lamport_ts"], cb["site_id"], tx_index or 0), cause, value)


def _insert(cb, uuid, nodes):
    """:107-115 -- proto/insert into the collection (s/insert's checks; the weave
    is deferred to materialisation) and the reverse paths into the history."""
    if not nodes:
        return cb
    cb = dict(cb)
    cols = dict(cb["collections"])
    cols[uuid] = C.insert(_no_weave, cols[uuid], nodes[0], nodes[1:])
    cols[uuid]["_dirty"] = True
    cb["collections"] = cols
    cb["history"] = cb["history"] + [(n[0], uuid) for n in nodes]
    return cb


def add_collection_for(cb, value, is_root=False):
    """:117-126 -> (cb, uuid or None)"""
    rng = cb.get("_rng", random)
    if _is_map(value):
        ct = C.new_map_ct(site_id=cb["site_id"], rng=rng)
    elif _seqable(value):
        ct = C.new_list_ct(site_id=cb["site_id"], rng=rng)
    else:
        return cb, None
    cb = dict(cb)
    cb["collections"] = dict(cb["collections"], **{ct["uuid"]: ct})
    if is_root:
        cb["root_uuid"] = ct["uuid"]
    return cb, ct["uuid"]


def map_to_nodes(cb, tx_index, m):
    """:130-138 -> (cb, tx_index, nodes)"""
    nodes = []
    for k, v in m.items():
        cb, tx_index, fv = flatten_value(cb, tx_index, v, preserve_strings=True)
        tx_index, node = new_node(cb, tx_index, k, fv)
        nodes.append(node)
    return cb, tx_index, nodes


def _elements(value, is_string):
    if value is None:
        return []
    if is_string:
        return [Char(ch) for ch in value]
    return list(value)


def list_to_nodes(cb, tx_index, value, cause=None):
    """:140-156 -> (cb, tx_index, nodes, last_node_id).  A string in a list of
    values is spliced into the same list, char by char."""
    is_string = isinstance(value, str) and not isinstance(value, Char)
    nodes = []
    cause = cause if cause is not None else C.ROOT_ID
    for v in _elements(value, is_string):
        if not is_string and isinstance(v, str) and not isinstance(v, Char):
            cb, tx_index, more, cause = list_to_nodes(cb, tx_index, v, cause)
            nodes += more
        else:
            cb, tx_index, fv = flatten_value(cb, tx_index, v, preserve_strings=is_string)
            tx_index, node = new_node(cb, tx_index, cause, fv)
            nodes.append(node)
            cause = node[0]
    return cb, tx_index, nodes, cause


def _flatten_collection(cb, tx_index, value, node_fn):
    """:158-164"""
    cb, uuid = add_collection_for(cb, value)
    cb, tx_index, nodes = node_fn(cb, tx_index, value)[:3]
    cb = _insert(cb, uuid, nodes)
    return cb, tx_index, uuid_to_ref(uuid)


def flatten_value(cb, tx_index, value, preserve_strings=False):
    """:166-172 -> (cb, tx_index, flat value)"""
    if preserve_strings and isinstance(value, str) and not isinstance(value, Char):
        return cb, tx_index, value
    if _is_map(value):
        return _flatten_collection(cb, tx_index, value, map_to_nodes)
    if _seqable(value):
        return _flatten_collection(cb, tx_index, value, list_to_nodes)
    return cb, tx_index, value


def _value_to_nodes(cb, tx_index, cause, value):
    """:174-183"""
    if _is_map(value):
        return map_to_nodes(cb, tx_index, value)
    if _seqable(value):
        return list_to_nodes(cb, tx_index, value, cause)[:3]
    tx_index, node = new_node(cb, tx_index, cause, value)
    return cb, tx_index, [node]


def _handle_value(cb, uuid, cause, value, tx_index):
    """:185-205"""
    ct = cb["collections"][uuid]
    merge = (cause is None and _is_map(value) and ct["type"] == "map") or \
        (not _is_map(value) and _seqable(value) and ct["type"] == "list")
    if merge:
        cb, tx_index, nodes = _value_to_nodes(cb, tx_index, cause, value)
        return _insert(cb, uuid, nodes), tx_index
    cb, tx_index, fv = flatten_value(cb, tx_index, value, preserve_strings=ct["type"] == "map")
    tx_index, node = new_node(cb, tx_index, cause, fv)
    return _insert(cb, uuid, [node]), tx_index


def transact_(cb, tx):
    """:238-268 -- tx = [(uuid, cause, value), ...]; uuid None makes a root."""
    tx_index = 0
    for uuid, cause, value in tx:
        if uuid is not None and cb["root_uuid"] is None:               # :219-221
            raise C.CauseError("Please transact a root collection first by setting uuid "
                               "and cause to nil", set())
        if uuid is not None and uuid not in cb["collections"]:          # :222-224
            raise C.CauseError("Collection with provided uuid not found", set())
        if uuid is None and not (_is_map(value) or isinstance(value, (list, tuple))):
            raise C.CauseError("Root node must satisfy the coll? predicate", set())
        if uuid is None:                                                # :207-212
            cb, uuid = add_collection_for(cb, value, is_root=True)
        cb, tx_index = _handle_value(cb, uuid, cause, value, tx_index)
    cb = dict(cb)
    cb["lamport_ts"] = cb["lamport_ts"] + 1
    return cb


# ------------------------------------------------------------ on the GPU ----
def weave_all(cb):
    """Reweave every collection changed since the last call: all lists in one
    cw_weave_lists call, all maps in one cw_weave_maps call."""
    cols = cb["collections"]
    lists = [u for u, ct in cols.items() if ct["type"] == "list" and ct.get("_dirty")]
    maps = [u for u, ct in cols.items() if ct["type"] == "map" and ct.get("_dirty")]
    if not lists and not maps:
        return cb
    new = dict(cols)
    if lists:
        for u, ct in zip(lists, C.weave_lists([cols[u] for u in lists])):
            new[u] = dict(ct, _dirty=False)
    if maps:
        for u, ct in zip(maps, C.weave_maps([cols[u] for u in maps])):
            new[u] = dict(ct, _dirty=False)
    out = dict(cb)
    out["collections"] = new
    return out


def get_collection(cb, uuid_or_ref=None):
    """:72-79"""
    key = uuid_or_ref if uuid_or_ref is not None else cb["root_uuid"]
    if key is None:
        return None
    return cb["collections"].get(ref_to_uuid(key) if is_ref(key) else key)


def _edn(cb, v, seen):
    """s/causal->edn (shared.cljc:320-328) with the ref resolution of
    Keyword's causal->edn (base/core.cljc:83-90); a ref met twice on one path
    raises instead of recursing forever (the reference's TODO at :88)."""
    if is_ref(v):
        u = ref_to_uuid(v)
        if u in seen:
            raise C.CauseError("collections reference each other", {"ref-cycle"})
        ct = cb["collections"].get(u)
        return None if ct is None else _ct_edn(cb, ct, seen | {u})
    return v


def _ct_edn(cb, ct, seen):
    if ct["type"] == "list":             # list.cljc:57-66
        return [_edn(cb, n[2], seen) for n in C.causal_list_to_list(ct)]
    return {n[1]: _edn(cb, n[2], seen) for n in C.causal_map_to_list(ct)}   # map.cljc:94-103


def cb_to_edn(cb):
    """base/core.cljc:92-96 -> (edn, cb with every collection woven)."""
    cb = weave_all(cb)
    root = get_collection(cb)
    if root is None:
        return None, cb
    return _ct_edn(cb, root, {root["uuid"]}), cb


def history(cb):
    """The ::history log: [(id, uuid)] sorted by id (vector compare of
    util.cljc:4-10), sorted on the GPU (cw_sort_keys)."""
    hist = cb["history"]
    if not hist:
        return []
    sites = sorted({i[1] for i, _ in hist}, key=pack.java_str_key)
    rank = {s: r for r, s in enumerate(sites)}
    ts_bits = max(1, max(i[0] for i, _ in hist).bit_length())
    tx_bits = max(1, max(i[2] for i, _ in hist).bit_length())
    site_bits = max(1, (len(sites) - 1).bit_length())
    if ts_bits + site_bits + tx_bits > 63:
        raise ValueError("history ids do not pack into 63 bits")
    keys = np.array([(i[0] << (site_bits + tx_bits)) | (rank[i[1]] << tx_bits) | i[2]
                     for i, _ in hist], np.uint64)
    _, order = C.weaver().sort_keys(keys, ts_bits + site_bits + tx_bits)
    return [hist[j] for j in order]
