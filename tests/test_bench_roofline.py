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
