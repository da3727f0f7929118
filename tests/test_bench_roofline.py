"""bench.py's roofline arithmetic (CPU): SURVEY 8(d)'s B_io and the achieved
rate over all timed launches (round 5 divided the bytes by the steps once,
which reported a fifth of the rate over five steps)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_b_io_matches_survey():
    assert bench.b_io_bytes(8, 4) == pytest.approx(21.125)   # u64 keys, u32 weave_perm
    assert bench.b_io_bytes(4, 2) == pytest.approx(11.125)   # config 3: u32 keys, u16 weave_perm


def test_achieved_counts_every_launch():
    # five steps of one 12 ms launch each over 5e8 nodes at 21.125 B/node
    n, b = 500_010_000, bench.b_io_bytes(8, 4)
    gbs = bench.achieved_gbs(n * b, 5, 5 * 12.0)
    assert gbs == pytest.approx(n * b / 12e-3 / 1e9)
    assert gbs / bench.HBM_PEAK_GBS == pytest.approx(0.11, abs=0.005)
    assert bench.achieved_gbs(1.0, 3, 0.0) == 0.0


def test_sample_check_catches_a_wrong_document():
    """The bench line's parity check on the timed path (check_snapshot_lists):
    zero mismatches on the oracle's own outputs laid out as the device writes
    them (doc-local weave_perm, one batch-wide render bitmap), one mismatch
    when a sampled document's order is disturbed."""
    import dataclasses

    import numpy as np
    import torch

    import oracle
    from cause_amd import gen

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=700)
    off, idk, ck, kd = gen.generate(spec, 0, 9, nthreads=2)
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    N, D = len(idk), len(off) - 1
    bits = np.packbits(np.concatenate([vis, np.zeros((-N) % 32, np.uint8)]), bitorder="little")
    t_perm = torch.from_numpy(perm.view(np.int32).copy())
    t_bits = torch.from_numpy(bits.view(np.int32).copy())
    vc = np.array([vis[int(off[d]):int(off[d + 1])].sum() for d in range(D)], np.int32)
    t_vc, t_st = torch.from_numpy(vc), torch.from_numpy(st.view(np.int32).copy())
    docs = bench.sample_docs(D, 4)
    assert list(docs) == [0, 3, 5, 8]
    snap = bench.snapshot_lists(off, docs, t_perm, t_bits, t_vc, t_st)
    assert bench.check_snapshot_lists(off, idk, ck, kd, snap) == (4, 0)
    lo = int(off[5])
    t_perm[lo + 1], t_perm[lo + 2] = t_perm[lo + 2].clone(), t_perm[lo + 1].clone()
    snap = bench.snapshot_lists(off, docs, t_perm, t_bits, t_vc, t_st)
    assert bench.check_snapshot_lists(off, idk, ck, kd, snap) == (4, 1)
