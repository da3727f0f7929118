"""Config 5 at full size, bit-exact: ONE list of 2,000,040,001 nodes through
the giant-document path (wide links, the multi-level list ranking), compared
position by position with the CPU oracle.

The list is 40,000 full config-2 documents (50,001 nodes each, generated in
parallel) hung under one global root: document k's ids get the high bits k+1
(ids stay unique and order-preserving inside every document), its root becomes
a normal node caused by the global root [0 "0" 0].  In the reference's fold
(shared.cljc:194-241) the global root's children are the documents' roots,
woven newest first, each followed by its own weave, because no node of one
document is caused by a node of another -- so the expected weave is the
concatenation of the 40,000 per-document weaves in descending document order,
which the oracle computes document by document (METHOD_EFF, pinned to the
literal fold by tests/test_fullsize_literal.py).  A document root renders
unless its first child is a hide.

~200 GB of HBM and ~70 GB of host memory; about a minute on the GPU box.
"""
import numpy as np
import pytest

import oracle
from cause_amd import abi, gen, pack

pytestmark = pytest.mark.gpu

DOCS = 40_000


def test_config5_full_size_giant_list_bit_exact():
    import torch

    props = torch.cuda.get_device_properties(0)
    if props.total_memory < 250e9:
        pytest.skip("needs a 288 GB MI355X")
    spec = gen.CONFIG2
    n = spec.doc_size
    off, idk, ck, kd = gen.generate(spec, 0, DOCS, nthreads=16)
    kb = spec.layout().key_bits
    # expected: per-document weaves (before the ids are changed)
    perm_d, vis_d, st_d = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=16)
    assert not st_d.any()
    # the giant list: document k's ids under the high bits k + 1, its root a
    # normal node caused by the global root (key 0), the global root last
    N = DOCS * n + 1
    hi = (np.arange(DOCS, dtype=np.uint64) + np.uint64(1)) << np.uint64(kb)
    hi = np.repeat(hi, n)
    nil = ck == np.uint64(pack.NIL)
    idk |= hi
    ck |= hi
    ck[nil] = 0
    kd &= np.uint8(3)
    idk = np.append(idk, np.uint64(0))
    ck = np.append(ck, np.uint64(pack.NIL))
    kd = np.append(kd, np.uint8(pack.KIND_ROOT))
    del hi, nil
    lay = pack.KeyLayout(kb + 16 - spec.layout().site_bits - spec.layout().tx_bits,
                         spec.layout().site_bits, spec.layout().tx_bits)
    with abi.Weaver(0) as w:
        res = w.weave_lists(np.array([0, N], np.uint64), idk, ck, kd, lay, yarns=False)
    assert res.status[0] == 0, res.status
    del idk, ck
    # expected weave: the global root, then documents D-1 .. 0, each its weave
    want = np.empty(N, np.uint32)
    want[0] = N - 1
    p = perm_d.reshape(DOCS, n).astype(np.uint32)
    p += (np.arange(DOCS, dtype=np.uint32) * np.uint32(n))[:, None]
    want[1:] = p[::-1].reshape(-1)
    del p
    bad = np.flatnonzero(res.weave_perm != want)
    assert bad.size == 0, (bad.size, bad[:5], res.weave_perm[bad[:5]], want[bad[:5]])
    # rendered bits: the per-document bits, each document root rendered unless
    # its first child (weave position 1) is a hide or h.hide
    v = vis_d.reshape(DOCS, n).copy()
    first = perm_d.reshape(DOCS, n)[:, 1]
    k1 = kd[:-1].reshape(DOCS, n)[np.arange(DOCS), first]
    v[:, 0] = ~((k1 == pack.KIND_HIDE) | (k1 == pack.KIND_HHIDE)) & 1
    want_vis = np.concatenate([[0], v[::-1].reshape(-1)]).astype(np.uint8)
    got_vis = res.visible()
    assert np.array_equal(got_vis, want_vis)
    assert res.visible_count[0] == int(want_vis.sum())
