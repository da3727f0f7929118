"""Streamed batches (cause_amd/stream.py) against the
oracle and against direct cw_weave_lists calls: every streamed batch must be
bit-identical to weaving it alone, whatever the pipeline depth, and ragged
batches (different document counts and sizes per batch) must reuse the slots
correctly."""
import dataclasses

import numpy as np
import pytest

import oracle
from cause_amd import abi, gen, stream

pytestmark = pytest.mark.gpu


def _batch(spec, i, docs):
    d0 = sum(docs[:i])
    return gen.generate(spec, d0, d0 + docs[i], nthreads=4)


@pytest.mark.parametrize("depth,k32,perm16", [(2, False, False), (3, False, False),
                                              (2, True, False), (2, True, True)])
def test_stream_matches_direct_and_oracle(depth, k32, perm16):
    import torch

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=700)
    docs = [40, 17, 40, 1, 33, 40, 25]      # ragged: the slots see every size
    batches = [_batch(spec, i, docs) for i in range(len(docs))]
    max_nodes = max(len(b[1]) for b in batches)

    def fill(i, views):
        off, idk, ck, kd = batches[i]
        n = len(idk)
        if k32:
            idk, ck = abi.narrow_k32(idk, ck)
        views[0][:n], views[1][:n], views[2][:n] = idk, ck, kd
        return off

    got = {}

    def consume(o):
        got[o.index] = (o.weave_perm.copy(), o.visible_bits.copy(), o.visible_count.copy(),
                        o.max_ts.copy(), o.status.copy())

    with abi.Weaver(0) as w:
        s = stream.BatchStreamer(w, "cuda:0", max_nodes, max(docs), spec.layout(), depth=depth,
                                 k32=k32, perm16=perm16)
        st = s.run(len(docs), fill, consume)
        del s
        torch.cuda.synchronize()
    assert sorted(got) == list(range(len(docs)))
    assert st.batches == len(docs) and st.nodes == sum(len(b[1]) for b in batches)
    assert len(st.weave_ms) == len(docs) and st.wall_s > 0

    with abi.Weaver(0) as ref:
        for i, (off, idk, ck, kd) in enumerate(batches):
            r = ref.weave_lists(off, idk, ck, kd, spec.layout(), yarns=False)
            perm, bits, vc, mt, sta = got[i]
            np.testing.assert_array_equal(perm, r.weave_perm)
            np.testing.assert_array_equal(bits, r.visible_bits)
            np.testing.assert_array_equal(vc, r.visible_count)
            np.testing.assert_array_equal(mt, r.max_ts)
            np.testing.assert_array_equal(sta, r.status)
            assert not sta.any()
    # and the oracle on two whole batches
    for i in (1, 3):
        off, idk, ck, kd = batches[i]
        want_perm, want_vis, want_st = oracle.batch_lists(off, idk, ck, kd,
                                                          method=oracle.METHOD_EFF)
        perm, bits, *_ = got[i]
        np.testing.assert_array_equal(perm, want_perm)
        vis = np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(perm)]
        np.testing.assert_array_equal(vis, want_vis)


def test_stream_rejects_oversized_batch():
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=100)
    off, idk, ck, kd = gen.generate(spec, 0, 8, nthreads=2)

    def fill(i, views):
        return np.arange(10, dtype=np.uint64) * 101      # 9 documents > max_docs
    with abi.Weaver(0) as w:
        s = stream.BatchStreamer(w, "cuda:0", len(idk), 8, spec.layout())
        with pytest.raises(ValueError):
            s.run(1, fill)


def test_stream_close_returns_the_weaver():
    """After close() the Weaver is synchronous on its own stream again: a host
    call right after sees finished results (the streamer used to
    keep the Weaver on its private stream in async mode)."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=2000)
    off, idk, ck, kd = gen.generate(spec, 0, 6, nthreads=2)

    def fill(i, views):
        n = len(idk)
        views[0][:n], views[1][:n], views[2][:n] = idk, ck, kd
        return off

    with abi.Weaver(0) as w:
        with stream.BatchStreamer(w, "cuda:0", len(idk), 6, spec.layout()) as s:
            s.run(2, fill)
        r = w.weave_lists(off, idk, ck, kd, spec.layout(), yarns=False)
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    np.testing.assert_array_equal(r.weave_perm, perm)
    assert not r.status.any()
