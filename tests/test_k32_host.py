"""Host side of the K32 boundary (no GPU): narrowing K64 keys to the u32 words
of cw_weave_lists_k32, and the generator's K32 output."""
import numpy as np
import pytest

from cause_amd import abi, gen, pack


def test_narrow_maps_nil_and_rejects_wide_keys():
    i, c = abi.narrow_k32(np.array([0, 5, 9], np.uint64), np.array([pack.NIL, 0, 5], np.uint64))
    assert i.dtype == np.uint32 and c.dtype == np.uint32
    assert list(c) == [abi.NIL32, 0, 5] and list(i) == [0, 5, 9]
    with pytest.raises(ValueError):
        abi.narrow_k32(np.array([0, 1 << 33], np.uint64), np.array([pack.NIL, 0], np.uint64))
    with pytest.raises(ValueError):
        abi.narrow_k32(np.array([0], np.uint64), np.array([abi.K32_RESERVED], np.uint64))
    # the non-id cause (NIL - 1) keeps its place at the top
    _, c = abi.narrow_k32(np.array([0], np.uint64), np.array([pack.NON_ID_CAUSE], np.uint64))
    assert c[0] == abi.NIL32 - 1


def test_generator_k32_words_are_the_narrowed_keys():
    off, idk, ck, kd = gen.generate(gen.CONFIG2, 3, 6, nthreads=2)
    off2, i32, c32, kd2 = gen.generate(gen.CONFIG2, 3, 6, nthreads=2, k32=True)
    a, b = abi.narrow_k32(idk, ck)
    assert np.array_equal(off, off2) and np.array_equal(kd, kd2)
    assert np.array_equal(i32, a) and np.array_equal(c32, b)
    with pytest.raises(ValueError):
        gen.generate(gen.CONFIG2, 0, 1, out=(idk, ck, kd), k32=True)
