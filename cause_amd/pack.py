"""Host-side marshalling for the weave C-ABI: site interning and id packing.

The GPU path works on order-preserving packed 64-bit ids:

    key = ts << (site_bits + tx_bits) | site_rank << tx_bits | tx

so that ``key(a) < key(b)`` iff ``(compare a b) < 0`` for ids ``[ts site tx]``
(util.cljc:4-10; ids are ``::s/id`` tuples, shared.cljc:31-40).  Site-ids are
ranked per document in Java ``String.compareTo`` order (UTF-16 code units), over
every site that appears in a node id *or* a cause id of that document, so a
cause pointing at an absent node still packs to a distinct, correctly ordered
key (it is then reported as an orphan by the GPU, never matched by accident).

Kinds (shared.cljc:21): 0 normal value, 1 ``:causal/hide``, 2 ``:causal/h.hide``,
3 ``:causal/h.show``; bit 2 flags the root node ``[[0 "0" 0] nil nil]``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

NIL = (1 << 64) - 1          # Clojure nil as a cause (root), CW_NIL in causeweave.h
NON_ID_CAUSE = NIL - 1       # a list node whose cause is not an id (never matches)

KIND_NORMAL, KIND_HIDE, KIND_HHIDE, KIND_HSHOW, KIND_ROOT = 0, 1, 2, 3, 4


def _special_names():
    return {("causal", "hide"): KIND_HIDE, ("causal", "h.hide"): KIND_HHIDE,
            ("causal", "h.show"): KIND_HSHOW}


_SPECIAL = _special_names()
ROOT_ID = (0, "0", 0)


def kind_of(value) -> int:
    """Value class of a node value: keywords with ns/name attributes
    (``causal/hide`` ...) are special (shared.cljc:21); anything else is normal."""
    ns = getattr(value, "ns", None)
    name = getattr(value, "name", None)
    if ns is not None and name is not None:
        return _SPECIAL.get((ns, name), KIND_NORMAL)
    return KIND_NORMAL


def java_str_key(s: str) -> bytes:
    """String.compareTo order: compare UTF-16 code units."""
    return s.encode("utf-16-be")


def is_id(x) -> bool:
    return isinstance(x, tuple) and len(x) == 3 and isinstance(x[1], str)


@dataclass(frozen=True)
class KeyLayout:
    """Bit layout of packed ids (shared by every document of a batch)."""

    ts_bits: int
    site_bits: int
    tx_bits: int

    @property
    def tx_shift(self) -> int:
        return 0

    @property
    def site_shift(self) -> int:
        return self.tx_bits

    @property
    def ts_shift(self) -> int:
        return self.tx_bits + self.site_bits

    @property
    def key_bits(self) -> int:
        return self.ts_bits + self.site_bits + self.tx_bits

    def pack(self, ts: int, site_rank: int, tx: int) -> int:
        return (ts << self.ts_shift) | (site_rank << self.site_shift) | tx


class KeyRangeError(ValueError):
    """Ids do not fit a K64 key (< 2^63; CW_STATUS_KEY_RANGE): use the K128
    layout (pack_lists_k128 / cw_weave_lists_k128), or they fit neither."""


def _bits(v: int) -> int:
    return max(int(v).bit_length(), 0)


def intern_sites(ids) -> dict:
    """Order-preserving site ranks for one document (String.compareTo order)."""
    sites = sorted({i[1] for i in ids}, key=java_str_key)
    return {s: r for r, s in enumerate(sites)}


@dataclass
class PackedDoc:
    id_key: np.ndarray     # uint64 [n]
    cause_key: np.ndarray  # uint64 [n]
    kind: np.ndarray       # uint8  [n]
    nodes: list            # the input nodes, in the packed order
    site_rank: dict


def layout_for(docs, extra_ids=None) -> KeyLayout:
    """Smallest layout that holds every id and id-cause of ``docs``
    (each doc: iterable of nodes ``(id, cause, value)``), plus ``extra_ids[d]``
    (ids that must pack in document d without being nodes, e.g. weft cuts)."""
    mts = msite = mtx = 0
    for d, nodes in enumerate(docs):
        ids = [n[0] for n in nodes] + [n[1] for n in nodes if is_id(n[1])]
        ids += list(extra_ids[d]) if extra_ids else []
        sites = {i[1] for i in ids}
        msite = max(msite, len(sites) - 1 if sites else 0)
        for ts, _, tx in ids:
            if ts < 0 or tx < 0:
                raise KeyRangeError("negative ts/tx-index")
            mts = max(mts, ts)
            mtx = max(mtx, tx)
    lay = KeyLayout(_bits(mts), _bits(msite), _bits(mtx))
    if lay.key_bits > 63:
        raise KeyRangeError(f"ids need {lay.key_bits} bits (> 63)")
    return lay


def pack_doc(nodes, layout: KeyLayout, extra_ids=()) -> PackedDoc:
    """Pack one document's nodes (``(id, cause, value)`` tuples, any order;
    weft's one-element ``(id,)`` node has cause nil and its id as value)."""
    nodes = list(nodes)
    ids = [n[0] for n in nodes] + [n[1] for n in nodes if len(n) > 1 and is_id(n[1])]
    ids += list(extra_ids)
    rank = intern_sites(ids)
    n = len(nodes)
    idk = np.empty(n, np.uint64)
    ck = np.empty(n, np.uint64)
    kd = np.empty(n, np.uint8)
    for i, nd in enumerate(nodes):
        nid = nd[0]
        cause, value = (nd[1], nd[-1]) if len(nd) > 1 else (None, nid)
        idk[i] = layout.pack(nid[0], rank[nid[1]], nid[2])
        if cause is None:
            ck[i] = NIL
        elif is_id(cause):
            ck[i] = layout.pack(cause[0], rank[cause[1]], cause[2])
        else:
            ck[i] = NON_ID_CAUSE
        k = kind_of(value)
        if nid == ROOT_ID and cause is None and value is None:
            k |= KIND_ROOT
        kd[i] = k
    return PackedDoc(idk, ck, kd, nodes, rank)


@dataclass
class PackedBatch:
    offsets: np.ndarray    # uint64 [D+1]
    id_key: np.ndarray     # uint64 [N]
    cause_key: np.ndarray  # uint64 [N]
    kind: np.ndarray       # uint8  [N]
    layout: KeyLayout
    docs: list             # PackedDoc per document


def pack_lists(docs, min_site_bits: int = 0, extra_ids=None) -> PackedBatch:
    """Pack a batch of list documents (each an iterable of nodes incl. root);
    ``extra_ids[d]``: ids that must pack in document d without being nodes."""
    docs = [list(d) for d in docs]
    lay = layout_for(docs, extra_ids)
    if lay.site_bits < min_site_bits:
        lay = KeyLayout(lay.ts_bits, min_site_bits, lay.tx_bits)
    packed = [pack_doc(d, lay, extra_ids[j] if extra_ids else ()) for j, d in enumerate(docs)]
    off = np.zeros(len(docs) + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs], dtype=np.uint64)
    cat = lambda f, dt: (np.concatenate([getattr(p, f) for p in packed]) if packed
                         else np.zeros(0, dt))
    return PackedBatch(off, cat("id_key", np.uint64), cat("cause_key", np.uint64),
                       cat("kind", np.uint8), lay, packed)


SITE_ID_LENGTH = 13  # shared.cljc:29


def valid_id(x) -> bool:
    """``(spec/valid? ::s/id x)`` (shared.cljc:31-40): [nat site-id nat] with a
    13-character site-id or "0".  A map cause that is not a valid id is a key
    (map.cljc:31)."""
    if not (isinstance(x, tuple) and len(x) == 3):
        return False
    ts, site, tx = x
    nat = lambda v: isinstance(v, int) and not isinstance(v, bool) and v >= 0
    return nat(ts) and nat(tx) and isinstance(site, str) and (
        len(site) == SITE_ID_LENGTH or site == "0")


@dataclass
class PackedMaps:
    offsets: np.ndarray      # uint64 [D+1]
    id_key: np.ndarray       # uint64 [N]
    cause: np.ndarray        # uint64 [N] packed id or key token
    cause_is_id: np.ndarray  # uint8  [N]
    kind: np.ndarray         # uint8  [N]
    layout: KeyLayout
    token_bits: int
    keys: list               # token -> key value
    docs: list               # nodes per collection, in the packed order
    ranks: list              # site rank table per collection


def pack_maps(docs) -> PackedMaps:
    """Pack a batch of map collections (each an iterable of ``(id, cause, value)``
    nodes; maps have no root node of their own).  Keys get batch-wide tokens in
    first-appearance order.  The virtual root [[0 "0" 0] nil nil] packs to 0 and
    so does a cause naming it; every other id packs by its site's rank in
    String.compareTo order, which may put site-ids such as " a " before "0"
    (list_test.cljc:85-96): an id with ts >= 1 still packs above 0, and only an
    id -- a node's or an id cause -- that itself sorts before the root id (ts 0)
    is refused (it would pack onto the root id)."""
    docs = [list(d) for d in docs]
    lay = layout_for([[(n[0], n[1] if valid_id(n[1]) else None, n[2]) for n in d]
                      + [((0, "0", 0), None, None)] for d in docs])
    tok = {}
    off = np.zeros(len(docs) + 1, np.uint64)
    N = sum(len(d) for d in docs)
    idk, ck = np.empty(N, np.uint64), np.empty(N, np.uint64)
    ci, kd = np.empty(N, np.uint8), np.empty(N, np.uint8)
    ranks = []
    j = 0
    for d, nodes in enumerate(docs):
        ids = [n[0] for n in nodes] + [n[1] for n in nodes if valid_id(n[1])] + [ROOT_ID]
        rank = intern_sites(ids)
        ranks.append(rank)
        pk = lambda i: 0 if i == ROOT_ID else lay.pack(i[0], rank[i[1]], i[2])
        for nid, cause, value in nodes:
            if nid[0] == 0 and java_str_key(nid[1]) < java_str_key("0"):
                raise KeyRangeError(f"map node id {nid} sorts before the root id")
            idk[j] = pk(nid)
            if valid_id(cause):
                # a cause id [0 s tx] with s before "0" would pack onto the root
                # id (or out of order): refused like such a node id
                if cause[0] == 0 and java_str_key(cause[1]) < java_str_key("0"):
                    raise KeyRangeError(f"map cause id {cause} sorts before the root id")
                ck[j] = pk(cause)
                ci[j] = 1
            elif cause is None:  # the nil key (cause_is_id = 2, include/causeweave.h)
                ck[j] = 0
                ci[j] = 2
            else:
                ck[j] = tok.setdefault(cause, len(tok))
                ci[j] = 0
            kd[j] = kind_of(value)
            j += 1
        off[d + 1] = j
    token_bits = max(1, _bits(max(len(tok) - 1, 0)))
    return PackedMaps(off, idk, ck, ci, kd, lay, token_bits, list(tok), docs, ranks)


# ---------------------------------------------------------------- K128 ids ----
# K128 = ts:64 | site_rank:32 | tx:32, as two u64 words per id
# (include/causeweave.h, cw_list_batch_k128): hi = ts, lo = site_rank << 32 | tx.
# (hi, lo) compared as one unsigned 128-bit number is (compare a b), util.cljc:4-10.
NIL2 = (NIL, NIL)               # a nil cause
NON_ID_CAUSE2 = (NIL, NIL - 1)  # a cause that is not an id (never matches one)


def pack_k128(ts: int, site_rank: int, tx: int):
    if not (0 <= ts < 1 << 64 and 0 <= site_rank < 1 << 32 and 0 <= tx < 1 << 32):
        raise KeyRangeError(f"id ({ts}, site rank {site_rank}, {tx}) does not fit K128")
    return ts, (site_rank << 32) | tx


@dataclass
class PackedBatchK128:
    offsets: np.ndarray    # uint64 [D+1]
    id_key: np.ndarray     # uint64 [N, 2] (hi, lo)
    cause_key: np.ndarray  # uint64 [N, 2]
    kind: np.ndarray       # uint8  [N]
    docs: list             # PackedDoc per document (id_key / cause_key [n, 2])


def pack_lists_k128(docs) -> PackedBatchK128:
    """Pack a batch of list documents (nodes incl. root, any order) as K128 ids;
    site-ids ranked per document in String.compareTo order like pack_lists."""
    docs = [list(d) for d in docs]
    packed = []
    for nodes in docs:
        ids = [n[0] for n in nodes] + [n[1] for n in nodes if len(n) > 1 and is_id(n[1])]
        rank = intern_sites(ids)
        n = len(nodes)
        idk = np.empty((n, 2), np.uint64)
        ck = np.empty((n, 2), np.uint64)
        kd = np.empty(n, np.uint8)
        for i, nd in enumerate(nodes):
            nid = nd[0]
            cause, value = (nd[1], nd[-1]) if len(nd) > 1 else (None, nid)
            idk[i] = pack_k128(nid[0], rank[nid[1]], nid[2])
            if cause is None:
                ck[i] = NIL2
            elif is_id(cause):
                ck[i] = pack_k128(cause[0], rank[cause[1]], cause[2])
            else:
                ck[i] = NON_ID_CAUSE2
            k = kind_of(value)
            if nid == ROOT_ID and cause is None and value is None:
                k |= KIND_ROOT
            kd[i] = k
        packed.append(PackedDoc(idk, ck, kd, nodes, rank))
    off = np.zeros(len(docs) + 1, np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs], dtype=np.uint64)
    cat = lambda f, shape, dt: (np.concatenate([getattr(p, f) for p in packed]) if packed
                                else np.zeros(shape, dt))
    return PackedBatchK128(off, cat("id_key", (0, 2), np.uint64), cat("cause_key", (0, 2), np.uint64),
                           cat("kind", (0,), np.uint8), packed)
