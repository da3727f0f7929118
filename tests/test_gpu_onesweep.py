"""The one-sweep radix sort (cause_amd/csrc/onesweep.hip) behind cw_sort_keys /
cw_sort_keys32 and every one-array sort of the library (config 5's id sort,
list.cljc:28 / shared.cljc:128; the giant tree's cross-tile children):
bit-exact against numpy's stable argsort, under every tile geometry, at sizes
around the tile and chunk boundaries, with duplicates (stability), one
bucket only (the longest look-back chains), nearly sorted keys and 64-bit
keys (8 passes); and equal to the histogram-scan-scatter passes it replaces."""
import numpy as np
import pytest

from cause_amd import abi

pytestmark = pytest.mark.gpu


def _keys(kind, n, bits, seed):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 1 << bits, n, dtype=np.uint64) if bits < 64 else \
            rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    if kind == "few":  # 7 distinct values: long runs, stability everywhere
        v = rng.integers(0, 7, n, dtype=np.uint64) & np.uint64((1 << min(bits, 3)) - 1)
        return v << np.uint64(max(bits - 3, 0))
    if kind == "one":  # every key in one bucket of every pass
        return np.full(n, (1 << bits) - 1 if bits < 64 else 2**64 - 1, np.uint64)
    if kind == "sorted":  # ids of a list arrive nearly in order
        k = np.arange(n, dtype=np.uint64) * np.uint64(3)
        sw = rng.integers(0, n, n // 50)
        k[sw] = k[(sw + 7) % n]
        return k & np.uint64((1 << bits) - 1) if bits < 64 else k
    raise ValueError(kind)


def _check(w, k, bits):
    ko, io = w.sort_keys(k, bits)
    order = np.argsort(k, kind="stable")
    assert np.array_equal(ko, k[order])
    assert np.array_equal(io, order.astype(np.uint32))


@pytest.mark.parametrize("geom", ["1", "2", "3", "4", "5", "6"])
def test_onesweep_geometries(monkeypatch, geom):
    monkeypatch.setenv("CW_ONESWEEP", geom)
    with abi.Weaver(0) as w:
        for n, bits, kind in ((1 << 16, 17, "random"), ((1 << 16) + 1, 9, "few"),
                              (8 * 4096 * 3 + 17, 35, "random"), (8 * 8192 + 8191, 20, "one"),
                              (1_000_003, 33, "sorted"), (3_000_001, 35, "random"),
                              (200_000, 64, "random"), (123_457, 1, "few")):
            _check(w, _keys(kind, n, bits, n + bits), bits)


def test_onesweep_equals_the_hist_scan_scatter_passes(monkeypatch):
    k = _keys("random", 2_500_000, 35, 5)
    monkeypatch.setenv("CW_ONESWEEP", "0")
    with abi.Weaver(0) as w:
        ref = w.sort_keys(k, 35)
    monkeypatch.delenv("CW_ONESWEEP")  # the default geometry
    with abi.Weaver(0) as w:
        w.reset_kernel_stats()
        w.set_profiling(True)
        got = w.sort_keys(k, 35)
        w.set_profiling(False)
        st = w.kernel_stats()
        for _ in range(3):  # the look-back words are reused across calls (epochs)
            again = w.sort_keys(k, 35)
            assert np.array_equal(again[1], ref[1])
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    # 4 passes; the ranged default counts each pass's input (one histogram
    # launch a pass), the single-chain geometries all passes at once
    assert st["ksort_scatter"][0] == 4 and st["ksort_hist"][0] == 4


@pytest.mark.parametrize("geom", ["1", "4", "5"])
def test_onesweep_keys32(monkeypatch, geom):
    import torch

    monkeypatch.setenv("CW_ONESWEEP", geom)
    rng = np.random.default_rng(3)
    with abi.Weaver(0) as w:
        for n, bits in ((70_000, 32), (1_000_001, 21)):
            k = rng.integers(0, 1 << bits, n, dtype=np.uint64).astype(np.uint32)
            dev = torch.device("cuda", 0)
            kin = torch.from_numpy(k.view(np.int32)).to(dev)
            ko = torch.empty_like(kin)
            io = torch.empty(n, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            w.sort_keys32_device(kin.data_ptr(), n, bits, ko.data_ptr(), io.data_ptr())
            order = np.argsort(k, kind="stable")
            assert np.array_equal(ko.cpu().numpy().view(np.uint32), k[order])
            assert np.array_equal(io.cpu().numpy().view(np.uint32), order.astype(np.uint32))
