"""K128 packing (host side, no GPU): the (hi, lo) pair of every id compares
like clojure.core/compare on [ts site tx] (util.cljc:4-10, restated as
causal_ref.id_key), for ids that do not fit the K64 layout."""
import random

import numpy as np
import pytest

from cause_amd import pack
from oracle import causal_ref as R


def _as_int(pair):
    return (int(pair[0]) << 64) | int(pair[1])


def test_k128_order_is_compare():
    rng = random.Random(5)
    sites = [R.new_site_id(rng) for _ in range(300)] + ["0", " a ", "A~aaaaaaaaaaa", "zz"]
    ids = [(rng.choice([0, 1, 1 << 40, (1 << 63) - 1, rng.randrange(1 << 63)]),
            rng.choice(sites), rng.choice([0, 1, (1 << 32) - 1, rng.randrange(1 << 32)]))
           for _ in range(3000)] + [R.ROOT_ID]
    nodes = [(i, R.ROOT_ID if i != R.ROOT_ID else None, "v" if i != R.ROOT_ID else None)
             for i in set(ids)]
    b = pack.pack_lists_k128([nodes])
    keys = [_as_int(p) for p in b.id_key]
    order_k = sorted(range(len(nodes)), key=lambda j: keys[j])
    order_r = sorted(range(len(nodes)), key=lambda j: R.id_key(nodes[j][0]))
    assert order_k == order_r
    # causes pack like the ids they name; nil is (NIL, NIL); the root is flagged
    root = [j for j, n in enumerate(nodes) if n[0] == R.ROOT_ID][0]
    assert tuple(b.cause_key[root]) == pack.NIL2 and b.kind[root] & pack.KIND_ROOT
    assert all(tuple(b.cause_key[j]) == tuple(b.id_key[root]) for j in range(len(nodes)) if j != root)


def test_k64_refuses_what_k128_takes():
    big = [R.ROOT_NODE, (((1 << 62), "aaaaaaaaaaaaa", 1 << 20), R.ROOT_ID, "x")]
    with pytest.raises(pack.KeyRangeError):
        pack.pack_lists([big])
    b = pack.pack_lists_k128([big])
    assert b.id_key.shape == (2, 2) and int(b.id_key[1][0]) == 1 << 62


def test_k128_limits_and_non_id_causes():
    with pytest.raises(pack.KeyRangeError):
        pack.pack_k128(1 << 64, 0, 0)
    with pytest.raises(pack.KeyRangeError):
        pack.pack_k128(0, 0, 1 << 32)
    b = pack.pack_lists_k128([[R.ROOT_NODE, ((1, "aaaaaaaaaaaaa", 0), "a-key", "x")], []])
    assert tuple(b.cause_key[1]) == pack.NON_ID_CAUSE2
    assert list(b.offsets) == [0, 2, 2]
    assert b.id_key.dtype == np.uint64


def test_map_packing_takes_sites_before_zero():
    """Site-ids that sort before "0" (list_test.cljc:85-96) pack in maps: the
    virtual root and causes naming it pack to 0, every other id above it."""
    nodes = [((1, " a ", 0), "k", "x"), ((2, " f ", 0), (1, " a ", 0), R.HIDE),
             ((3, "0", 1), R.ROOT_ID, "y")]
    pm = pack.pack_maps([nodes])
    assert pm.ranks[0][" a "] == 0 and pm.ranks[0]["0"] > 0
    assert (pm.id_key > 0).all()
    assert pm.cause[2] == 0 and pm.cause_is_id[2] == 1
    order = np.argsort(pm.id_key)
    assert [nodes[j][0] for j in order] == sorted((n[0] for n in nodes), key=R.id_key)
    with pytest.raises(pack.KeyRangeError):
        pack.pack_maps([[((0, " a ", 0), "k", "x")]])


def test_map_cause_id_before_the_root_is_refused():
    """An id cause [0 s tx] whose site sorts before "0" would pack onto the
    root id 0 (and a cause naming it would weave under the root): refused like
    a node id that sorts before the root."""
    site = "-" * 13  # a valid ::s/id site (13 chars) that sorts before "0"
    with pytest.raises(pack.KeyRangeError):
        pack.pack_maps([[((1, "0", 0), (0, site, 0), "x")]])
    # the same site with ts >= 1 packs above the root
    pm = pack.pack_maps([[((1, site, 0), "k", "x"), ((2, "0", 0), (1, site, 0), R.HIDE)]])
    assert pm.cause[1] > 0 and pm.cause_is_id[1] == 1
