"""cw_weave_lists_k32 (narrow keys) against cw_weave_lists (K64) on the same
batches: the K32 words are the K64 keys of batches whose ids fit 32 bits, so
every output -- weave order, rendered bits, counts, ::lamport-ts, yarns and
status -- must be identical, through the fast path, the exact path (documents
outside the domain), the giant path (one 100k-node list) and both memory
spaces.  The K64 path itself is pinned to the oracle by test_gpu_parity.py and
test_gpu_exact.py; here one batch per case is also checked against the oracle.
"""
import random

import numpy as np
import pytest

import oracle
from cause_amd import abi, gen, pack
from oracle import causal_ref as R
from tests import outdomain as X
from tests import refgen as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def weaver():
    with abi.Weaver(0) as w:
        yield w


def _same(a, b):
    for f in ("weave_perm", "visible_bits", "visible_count", "max_ts", "status", "yarn_perm"):
        x, y = getattr(a, f), getattr(b, f)
        if x is None or y is None:
            assert x is None and y is None, f
            continue
        np.testing.assert_array_equal(x, y, err_msg=f)


def _both_ways(w, off, idk, ck, kd, lay):
    import torch

    want = w.weave_lists(off, idk, ck, kd, lay)
    i32, c32 = abi.narrow_k32(idk, ck)
    got = w.weave_lists_k32(off, i32, c32, kd, lay)
    _same(got, want)
    # device memory
    dev = torch.device("cuda", 0)
    N, D = len(idk), len(off) - 1
    t = lambda x: torch.from_numpy(x.view(np.int32) if x.dtype == np.uint32 else x).to(dev)
    gi, gc, gk = t(i32), t(c32), t(kd)
    outs = {"weave_perm": torch.empty(max(N, 1), dtype=torch.int32, device=dev),
            "visible_bits": torch.zeros((N + 31) // 32 + 1, dtype=torch.int32, device=dev),
            "visible_count": torch.empty(max(D, 1), dtype=torch.int32, device=dev),
            "max_ts": torch.empty(max(D, 1), dtype=torch.int64, device=dev),
            "status": torch.empty(max(D, 1), dtype=torch.int32, device=dev)}
    w.weave_lists_k32_device(off, gi.data_ptr(), gc.data_ptr(), gk.data_ptr(), lay,
                             {k: v.data_ptr() for k, v in outs.items()})
    torch.cuda.synchronize()
    np.testing.assert_array_equal(outs["weave_perm"][:N].cpu().numpy().view(np.uint32),
                                  want.weave_perm)
    np.testing.assert_array_equal(outs["status"][:D].cpu().numpy().view(np.uint32), want.status)
    np.testing.assert_array_equal(outs["visible_count"][:D].cpu().numpy().view(np.uint32),
                                  want.visible_count)
    np.testing.assert_array_equal(outs["max_ts"][:D].cpu().numpy().view(np.uint64), want.max_ts)
    nb = (N + 31) // 32
    np.testing.assert_array_equal(outs["visible_bits"][:nb].cpu().numpy().view(np.uint32),
                                  want.visible_bits)
    # 16-bit weave_perm (documents below 2^16 nodes)
    if N and int(np.diff(off).max()) < 65536:
        p16 = torch.empty(N, dtype=torch.int16, device=dev)
        w.weave_lists_k32_device(off, gi.data_ptr(), gc.data_ptr(), gk.data_ptr(), lay,
                                 dict({k: v.data_ptr() for k, v in outs.items()},
                                      weave_perm=p16.data_ptr()), perm16=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(p16.cpu().numpy().view(np.uint16), want.weave_perm)
    return want


def test_config2_documents(weaver):
    spec = gen.CONFIG2
    off, idk, ck, kd = gen.generate(spec, 0, 12, nthreads=8)
    want = _both_ways(weaver, off, idk, ck, kd, spec.layout())
    assert not want.status.any()
    p, v, s = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    np.testing.assert_array_equal(want.weave_perm, p)
    # the generator's K32 words are the narrowed K64 keys
    _, i32, c32, k2 = gen.generate(spec, 0, 12, nthreads=8, k32=True)
    a, b = abi.narrow_k32(idk, ck)
    assert np.array_equal(i32, a) and np.array_equal(c32, b) and np.array_equal(k2, kd)


def test_out_of_domain_documents_take_the_exact_path(weaver):
    rng = random.Random(32)
    docs = []
    for steps in (6, 20, 80):
        for _ in range(8):
            nodes, _ = G.random_history(rng, steps)
            docs.append(X.corrupt([R.ROOT_NODE] + nodes, rng, X.KINDS, rate=0.2))
            docs.append([R.ROOT_NODE] + nodes)
    docs.append([])                              # an empty document
    b = pack.pack_lists(docs)
    assert b.layout.key_bits <= 31
    want = _both_ways(weaver, b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    assert (want.status != 0).any()
    p, v, s = oracle.batch_lists(b.offsets, b.id_key, b.cause_key, b.kind,
                                 method=oracle.METHOD_LITERAL)
    np.testing.assert_array_equal(want.weave_perm, p)


def test_one_giant_list(weaver):
    spec = gen.CONFIG1
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=1)
    _both_ways(weaver, off, idk, ck, kd, spec.layout())


def test_golden_vectors(weaver):
    z = np.load("tests/golden/packed_vectors.npz")
    names = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_offsets")})
    done = 0
    for nm in names:
        idk = z[nm + "_id_key"]
        if idk.size and int(idk.max()) >= abi.NIL32:
            continue
        lay = pack.KeyLayout(*[int(x) for x in z[nm + "_layout"]])
        res = _both_ways(weaver, z[nm + "_offsets"], idk, z[nm + "_cause_key"], z[nm + "_kind"], lay)
        np.testing.assert_array_equal(res.weave_perm, z[nm + "_weave_perm"])
        done += 1
    assert done


def test_perm16_rejects_large_documents(weaver):
    import torch

    off = np.array([0, 70_000], np.uint64)
    dev = torch.device("cuda", 0)
    z = torch.zeros(70_000, dtype=torch.int32, device=dev)
    o = {k: torch.zeros(70_000, dtype=torch.int32, device=dev).data_ptr()
         for k in ("weave_perm", "visible_bits", "visible_count", "max_ts", "status")}
    with pytest.raises(abi.WeaveError):
        weaver.weave_lists_k32_device(off, z.data_ptr(), z.data_ptr(), z.data_ptr(),
                                      pack.KeyLayout(17, 0, 0), o, perm16=True)


def test_narrow_rejects_wide_keys():
    with pytest.raises(ValueError):
        abi.narrow_k32(np.array([0, 1 << 33], np.uint64), np.array([pack.NIL, 0], np.uint64))
    i, c = abi.narrow_k32(np.array([0, 5], np.uint64), np.array([pack.NIL, 0], np.uint64))
    assert c[0] == abi.NIL32 and c[1] == 0 and i.dtype == np.uint32
