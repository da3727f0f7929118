"""Synthetic workload generators (input only, libcauseweave_gen.so): shapes,
determinism per document (any shard regenerates the same documents) and the
domain properties the benches rely on, checked with the CPU oracle."""
import dataclasses

import numpy as np

import oracle
from cause_amd import gen


def test_list_generator_shards_reproduce():
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=500)
    off, i, c, k = gen.generate(spec, 0, 6, nthreads=3)
    off2, i2, c2, k2 = gen.generate(spec, 4, 6, nthreads=1)
    n = spec.doc_size
    np.testing.assert_array_equal(i[4 * n:], i2)
    np.testing.assert_array_equal(c[4 * n:], c2)
    np.testing.assert_array_equal(k[4 * n:], k2)
    for d in range(6):
        ids, cs = i[d * n:(d + 1) * n], c[d * n:(d + 1) * n]
        assert len(np.unique(ids)) == n
        idset = set(ids.tolist())
        assert all(x == 2**64 - 1 or (x in idset) for x in cs.tolist())
        nonroot = cs != np.uint64(2**64 - 1)
        assert (cs[nonroot] < ids[nonroot]).all()  # lamport: causes are older
    _, st = oracle.list_weave(i[:n], c[:n], k[:n], oracle.METHOD_LITERAL)
    assert st == 0


def test_map_generator_shape_and_domain():
    spec = gen.CONFIG4
    lay, tb = spec.layout()
    assert tb == 8 and lay.site_bits == 4
    off, i, c, ci, k = gen.generate_maps(spec, 0, 200, nthreads=4)
    assert len(i) == 200 * 100
    _, i2, c2, ci2, k2 = gen.generate_maps(spec, 150, 200, nthreads=1)
    np.testing.assert_array_equal(i[150 * 100:], i2)
    np.testing.assert_array_equal(c[150 * 100:], c2)
    assert (c[ci == 0] < 256).all()
    kinds = np.bincount(k, minlength=4) / len(k)
    assert 0.05 < kinds[1] < 0.11 and 0.04 < kinds[2] < 0.08 and 0.03 < kinds[3] < 0.08
    for d in range(200):
        s = slice(d * 100, (d + 1) * 100)
        ids = {int(x): j for j, x in enumerate(i[s])}
        assert len(ids) == 100
        for j in np.flatnonzero(ci[s]):
            cj = ids[int(c[s][j])]
            assert ci[s][cj] == 0 and k[s][cj] == 0  # undo/redo target a value write
            assert c[s][j] < i[s][j]
    nk, npos, sk, sa = oracle.map_weave(i[:100], c[:100], ci[:100], k[:100], 0)
    assert set(sk.tolist()) == set(c[:100][ci[:100] == 0].tolist())
    assert (npos >= 1).all()


def test_map_generator_bad_fraction():
    spec = gen.MapSpec(nodes_per_coll=200, p_bad=0.05, seed=3)
    off, i, c, ci, k = gen.generate_maps(spec, 0, 20, nthreads=2)
    bad = 0
    for d in range(20):
        s = slice(d * 200, (d + 1) * 200)
        ids = {int(x): j for j, x in enumerate(i[s])}
        bad += sum(1 for j in np.flatnonzero(ci[s]) if ci[s][ids[int(c[s][j])]])
    assert bad > 50
