"""Full-size documents for the parity tests (test inputs only).

A config-2 document is *dirty* when some non-special node's cause is a special
node (a hide, h.hide or h.show): the conj-style causes of list.cljc:36-40
(``cause = the last weave node``) make them.  In a dirty document the plain
preorder of the cause tree is not the weave: the node must skip to after its
special cause's run (weave-later? clause A, shared.cljc:208-212), which is what
the fast path's effective tree restates.  Clean documents exercise
only the plain preorder.
"""
from __future__ import annotations

import numpy as np

from cause_amd import gen


def dirty_docs(off, idk, ck, kd) -> np.ndarray:
    """bool[D]: the document holds a non-special node with a special cause."""
    D = len(off) - 1
    out = np.zeros(D, bool)
    for d in range(D):
        a, b = int(off[d]), int(off[d + 1])
        i, c, k = idk[a:b], ck[a:b], kd[a:b] & 3
        order = np.argsort(i, kind="stable")
        si = i[order]
        has = c != np.uint64((1 << 64) - 1)
        pos = np.searchsorted(si, c[has])
        pos = np.minimum(pos, len(si) - 1)
        found = si[pos] == c[has]
        ck_kind = np.zeros(has.sum(), np.uint8)
        ck_kind[found] = k[order[pos[found]]]
        out[d] = bool(((k[has] == 0) & (ck_kind != 0)).any())
    return out


def config2_mixed(n_dirty: int, n_clean: int, scan: int = 256):
    """Full 50,001-node config-2 documents: the first n_dirty dirty and n_clean
    clean ones among the first ``scan`` of the bench workload, interleaved."""
    spec = gen.CONFIG2
    off, idk, ck, kd = gen.generate(spec, 0, scan)
    dirty = dirty_docs(off, idk, ck, kd)
    pick_d = list(np.flatnonzero(dirty)[:n_dirty])
    pick_c = list(np.flatnonzero(~dirty)[:n_clean])
    if len(pick_d) < n_dirty or len(pick_c) < n_clean:
        raise RuntimeError(f"not enough dirty/clean documents in {scan}: "
                           f"{dirty.sum()} dirty, {(~dirty).sum()} clean")
    picks = [x for pair in zip(pick_d, pick_c) for x in pair]
    picks += pick_d[len(pick_c):] + pick_c[len(pick_d):]
    n = spec.doc_size
    sel = np.concatenate([np.arange(p * n, (p + 1) * n) for p in picks])
    noff = np.arange(len(picks) + 1, dtype=np.uint64) * np.uint64(n)
    return noff, idk[sel], ck[sel], kd[sel], dirty[picks], spec.layout()
