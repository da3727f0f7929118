"""GPU parity of cw_weave_maps (c.map/weave 1-arity + active-node, map.cljc:26-59)
against the C oracle's literal fold (oracle/weave_oracle.c or_map_fold_literal,
pinned to the Python restatement and map_test.cljc in test_oracle.py).

Compared per collection and key: the key weave (node order, root first) and
the active node (LWW, -1 = ::blank), including the reference's quirky keys
(a key that is an id, or nil).  Collections the library flags
(duplicate ids) are out of domain: the flag itself is checked against the
host's own reading.  Every other collection -- nodes caused by the root id, by
nil or by an absent id, causes with larger ids than their nodes -- must match
the literal fold on every path.
"""
import random

import numpy as np
import pytest

import oracle
from cause_amd import abi, gen

pytestmark = pytest.mark.gpu

NO_ROOT = 0xFFFFFFFF
ID_KEY = 1 << 63
NIL = (1 << 64) - 1


@pytest.fixture(scope="module", params=["fused", "small", "pipeline"])
def weaver(request):
    """Every way of weaving key weaves: the one-kernel pack path (k_map_pack,
    collections of <= 2048 nodes), one wave per tiny key weave after the
    general sorts (k_small_weave, LDS pack sorts; CW_MAP_FUSED=0) and the full
    list pipeline (CW_MAP_SMALL=0, global radix passes)."""
    import os

    # "pipeline" also sorts with the global radix passes instead of the LDS packs
    knobs = {"fused": {"CW_MAP_FUSED": "1"},
             "small": {"CW_MAP_FUSED": "0", "CW_MAP_SMALL": "1", "CW_PACK_SORT": "1"},
             "pipeline": {"CW_MAP_FUSED": "0", "CW_MAP_SMALL": "0", "CW_PACK_SORT": "0"}}[request.param]
    old = {k: os.environ.get(k) for k in knobs}
    os.environ.update(knobs)
    try:
        w = abi.Weaver(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    w.fused = request.param == "fused"
    yield w
    w.close()


def oracle_maps(off, idk, ck, ci, kd):
    """Per collection: {key: (active, [input idx in weave order])}, keys in the
    ABI's form (token, ID_KEY | id, or NIL).  Tokens go to the oracle with bit
    63 set so they can never equal a packed id (a keyword is never a vector)."""
    out = []
    tok = np.uint64(1 << 63)
    for d in range(len(off) - 1):
        a, b = int(off[d]), int(off[d + 1])
        c = oracle.map_causes(ck[a:b], ci[a:b])
        nk, npos, sk, sa = oracle.map_weave(idk[a:b], c, ci[a:b], kd[a:b], 0)

        def api(k):
            if k == NIL:
                return NIL
            return k & ~ID_KEY if k & ID_KEY else ID_KEY | k

        order = np.lexsort((npos, nk))
        groups = {}
        for j in order:
            groups.setdefault(int(nk[j]), []).append(int(j))
        out.append({api(int(k)): (int(act), groups.get(int(k), [])) for k, act in zip(sk, sa)})
    return out


def gpu_maps(res, D):
    out = [dict() for _ in range(D)]
    for s in range(len(res.seg_key)):
        kw = res.key_weave(s)
        assert kw[0] == NO_ROOT, "key weave must start at its root"
        out[int(res.seg_coll[s])][int(res.seg_key[s])] = (int(res.seg_active[s]),
                                                           [int(x) for x in kw[1:]])
    return out


def expected_flags(off, idk, ck, ci):
    """Host reading of the map domain: duplicate ids (::nodes is a map)."""
    flags = np.zeros(len(off) - 1, np.uint32)
    for d in range(len(off) - 1):
        a, b = int(off[d]), int(off[d + 1])
        if len(set(idk[a:b].tolist())) != b - a:
            flags[d] |= abi.STATUS_DUP
    return flags


def check(weaver, off, idk, ck, ci, kd, token_bits, key_bits=0, flags=None):
    """Every collection without a flag is compared with the literal map fold on
    every path: key weaves with nodes caused by the root id, by nil or by an
    absent id, or with non-Lamport causes, are folded literally
    (CW_STATUS_NON_LAMPORT stays as information)."""
    res = weaver.weave_maps(off, idk, ck, ci, kd, token_bits, key_bits)
    D = len(off) - 1
    if flags is None:
        flags = expected_flags(off, idk, ck, ci)
    np.testing.assert_array_equal(res.status & (abi.STATUS_MAP_KEY | abi.STATUS_DUP), flags)
    got, want = gpu_maps(res, D), oracle_maps(off, idk, ck, ci, kd)
    for d in range(D):
        if flags[d]:
            continue
        assert int(res.status[d]) & ~abi.STATUS_NON_LAMPORT == 0, (d, res.status[d])
        assert got[d] == want[d], f"collection {d}"
    # key weaves come per collection in ascending key order
    sc, sk = res.seg_coll.astype(np.uint64), res.seg_key
    assert np.all((sc[1:] > sc[:-1]) | ((sc[1:] == sc[:-1]) & (sk[1:] > sk[:-1])))
    return res


def test_config4_shape(weaver):
    spec = gen.CONFIG4
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 3000, nthreads=8)
    res = check(weaver, off, idk, ck, ci, kd, tb)
    assert (res.status == 0).all()


def test_large_collections_few_keys(weaver):
    # long key weaves: few keys, many writes and id-caused undo/redo per key
    spec = gen.MapSpec(nodes_per_coll=20_000, n_keys=5, zipf_s=0.5, seed=11)
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 6, nthreads=6)
    check(weaver, off, idk, ck, ci, kd, tb)


def test_pack_limit_collections_long_key_weaves(weaver):
    """Collections at the fused path's pack limit (2048 nodes) with 3 keys:
    key weaves of hundreds of nodes woven inside one pack, next to a pack of
    many tiny collections."""
    spec = gen.MapSpec(nodes_per_coll=2048, n_keys=3, zipf_s=0.5, seed=12)
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 5, nthreads=5)
    small = gen.MapSpec(nodes_per_coll=3, seed=13)
    _, tb2 = small.layout()
    o2, i2, c2, ci2, k2 = gen.generate_maps(small, 0, 700, nthreads=4)
    cat = lambda a, b: np.concatenate([a, b])
    off2 = np.concatenate([off, off[-1] + o2[1:]])
    check(weaver, off2, cat(idk, i2), cat(ck, c2), cat(ci, ci2), cat(kd, k2), max(tb, tb2))


def test_many_keys(weaver):
    spec = gen.MapSpec(nodes_per_coll=3000, n_keys=60_000, zipf_s=0.2, seed=12)
    _, tb = spec.layout()
    assert tb == 16
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 20, nthreads=8)
    check(weaver, off, idk, ck, ci, kd, tb)


def test_f8c_id_keys(weaver):
    """a node whose cause node is itself id-caused lands in a weave
    keyed by that id, appended there as an orphan."""
    spec = gen.MapSpec(nodes_per_coll=60, p_bad=0.05, seed=13)
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 400, nthreads=8)
    res = check(weaver, off, idk, ck, ci, kd, tb)
    assert (res.status == 0).all()
    n_id = int(((res.seg_key & np.uint64(ID_KEY)) != 0).sum())
    assert 50 < n_id < len(res.seg_key)


def test_ragged_and_empty_collections(weaver):
    rng = np.random.default_rng(5)
    parts = []
    sizes = [0, 1, 2, 0, 5, 100, 4097, 1, 0, 9000, 33]
    for d, n in enumerate(sizes):
        if n == 0:
            parts.append((np.zeros(0, np.uint64),) * 2 + (np.zeros(0, np.uint8),) * 2)
            continue
        spec = gen.MapSpec(nodes_per_coll=n, n_keys=int(rng.integers(1, 300)), seed=100 + d)
        _, tb = spec.layout()
        _, i, c, ci, k = gen.generate_maps(spec, d, d + 1, nthreads=1)
        parts.append((i, c, ci, k))
    off = np.zeros(len(sizes) + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    idk, ck, ci, kd = (np.concatenate([p[j] for p in parts]) for j in range(4))
    res = check(weaver, off, idk, ck, ci, kd, 9)
    assert res.status[0] == 0 and res.status[3] == 0


def test_absent_causes_nil_key_and_flags(weaver):
    spec = gen.MapSpec(nodes_per_coll=50, seed=14)
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 5, nthreads=1)
    idk, ck, ci = idk.copy(), ck.copy(), ci.copy()
    # collection 1: id causes that are not in the collection -> the nil key
    for j in (50 + np.flatnonzero(ci[50:100] == 0)[:3]):
        ci[j], ck[j] = 1, (1 << 40) | 3
    # collection 2: a duplicated id
    idk[101] = idk[100]
    # collection 3: a node caused by the root id
    j = 150 + int(np.flatnonzero(ci[150:200] == 0)[0])
    ci[j], ck[j] = 1, 0
    res = check(weaver, off, idk, ck, ci, kd, tb)
    assert res.status[2] & abi.STATUS_DUP
    assert res.status[3] == 0  # the literal fold of the nil key weave, on every path
    assert res.status[0] == 0 and res.status[1] == 0 and res.status[4] == 0
    nil = np.flatnonzero((res.seg_coll == 1) & (res.seg_key == np.uint64(NIL)))
    assert len(nil) == 1 and len(res.key_weave(int(nil[0]))) == 4


def test_assoc_after_dissoc_quirk(weaver):
    """assoc :a 1, dissoc :a, assoc :a 2 => {} (map.cljc:50-52)."""
    s = 1  # site bits = 1, one site of rank 1
    ids = np.array([(1 << s) | 1, (2 << s) | 1, (3 << s) | 1, (4 << s) | 1], np.uint64)
    cause = np.array([0, 0, 0, 1], np.uint64)        # key tokens :a = 0, :b = 1
    cis = np.zeros(4, np.uint8)
    kind = np.array([0, 1, 0, 0], np.uint8)          # 1, hide, 2 on :a; :b -> value
    res = check(weaver, np.array([0, 4], np.uint64), ids, cause, cis, kind, 1)
    got = gpu_maps(res, 1)[0]
    assert got[0][0] == -1          # :a stays hidden
    assert got[0][1] == [1, 2, 0]   # root, hide, 2 (newest value skips the hide), 1
    assert got[1] == (3, [3])


def test_random_small_maps_match_oracle(weaver):
    rng = random.Random(21)
    offs, I, Cs, CI, K = [0], [], [], [], []
    for d in range(300):
        n = rng.randint(1, 40)
        nodes, values = [], []
        for m in range(n):
            t = m + 1
            site = rng.randint(1, 3)
            idv = (t << 2) | site
            r = rng.random()
            if r < 0.55 or not values:
                nodes.append((idv, rng.randint(0, 5), 0, 0))
                values.append(idv)
            elif r < 0.7:
                nodes.append((idv, rng.randint(0, 5), 0, 1))
            else:  # mostly undo/redo of a value; sometimes any earlier node (F8c keys)
                pool = values if rng.random() < 0.8 else [x[0] for x in nodes]
                nodes.append((idv, rng.choice(pool), 1, rng.choice([1, 2, 3, 0])))
        rng.shuffle(nodes)
        for x in nodes:
            I.append(x[0]); Cs.append(x[1]); CI.append(x[2]); K.append(x[3])
        offs.append(len(I))
    check(weaver, np.array(offs, np.uint64), np.array(I, np.uint64), np.array(Cs, np.uint64),
          np.array(CI, np.uint8), np.array(K, np.uint8), 3)


def literal_histories(rng, n_colls, n_lo, n_hi, t_max=None):
    """Map collections the reference folds with nodes that are not children of
    their causes in id order: nodes caused by the root id [0 "0" 0] or by nil
    (the nil key, next to nodes whose cause is absent, and children of those),
    and undo/redo nodes whose cause has a larger id or is the node itself (a
    self-caused id X makes the id key weave X hold X's children and
    grandchildren with their causes)."""
    offs, I, Cs, CI, K = [0], [], [], [], []
    for d in range(n_colls):
        n = rng.randint(n_lo, n_hi)
        nodes = []
        ids = rng.sample(range(1, t_max or 7 * n_hi), n)
        for m, t in enumerate(ids):
            idv = (t << 2) | rng.randint(1, 3)
            r = rng.random()
            if r < 0.45:                   # a value or hide under a key
                nodes.append([idv, rng.randint(0, 3), 0, rng.choice([0, 0, 0, 1])])
            elif r < 0.55:                 # caused by the root id
                nodes.append([idv, 0, 1, rng.choice([0, 1, 2, 3])])
            elif r < 0.6:                  # a nil cause (cause_is_id = 2)
                nodes.append([idv, 0, 2, rng.choice([0, 0, 1])])
            elif r < 0.7:                  # an absent cause
                nodes.append([idv, ((1 << 40) + rng.randint(0, 99)) << 2 | 1, 1,
                              rng.choice([0, 2, 3])])
            else:                          # undo / redo of any node (older or newer)
                nodes.append([idv, None, 1, rng.choice([1, 2, 3, 0])])
        for x in nodes:
            if x[1] is None:
                x[1] = x[0] if rng.random() < 0.04 else rng.choice(nodes)[0]
        rng.shuffle(nodes)
        for x in nodes:
            I.append(x[0]); Cs.append(x[1]); CI.append(x[2]); K.append(x[3])
        offs.append(len(I))
    return (np.array(offs, np.uint64), np.array(I, np.uint64), np.array(Cs, np.uint64),
            np.array(CI, np.uint8), np.array(K, np.uint8))


def test_literal_key_weaves_root_id_nil_and_non_lamport_causes(weaver):
    """Small collections of literal_histories: the fused path folds those key
    weaves literally in LDS, the general paths through exact.hip; all must
    match the oracle's literal map fold exactly."""
    off, idk, ck, ci, kd = literal_histories(random.Random(23), 400, 2, 30, t_max=200)
    res = check(weaver, off, idk, ck, ci, kd, 2)
    assert (res.status & abi.STATUS_NON_LAMPORT).any()


def self_cause_collections():
    """Hand-made collections around a self-caused id X (cause = id), which the
    reference's new-node spec forbids (shared.cljc:98) but a ::nodes map handed
    to the 1-arity weave can hold.  Returns the batch and the expected key
    weave ID|X of collection 0 (input indices after the root)."""
    t = lambda ts, site=1: (ts << 2) | site
    X, C, C2, G = t(5), t(9), t(13), t(17)
    colls = [
        # X->X, two children of X, a grandchild through C: the key weave X is
        # root, X, C2, C, G (weave-node: C2 lands right after X, before C)
        [(X, X, 1, 0), (C, X, 1, 0), (C2, X, 1, 0), (G, C, 1, 0)],
        # the same shuffled, with an older child of X (E < X: placed before
        # the node it causes), hides of G and C2, a plain key and a nil key
        [(G, C, 1, 0), (t(3), X, 1, 0), (C2, X, 1, 0), (X, X, 1, 2), (C, X, 1, 0),
         (t(20), G, 1, 1), (t(21), C2, 1, 2), (t(2), 1, 0, 0), (t(22), t(2), 1, 0),
         (t(23), t(99), 1, 0)],
        # a two-cycle X<->Y: neither is self-caused, every id key weave chains
        [(X, C, 1, 0), (C, X, 1, 0), (t(30), X, 1, 0), (t(31), C, 1, 3), (t(32), t(30), 1, 0)],
        # a self-caused special, children of several kinds, great-grandchildren
        # (key = a grandchild's cause, not X) and an absent X sibling
        [(X, X, 1, 1), (C, X, 1, 3), (C2, X, 1, 0), (G, C2, 1, 0), (t(18), G, 1, 2),
         (t(19, 2), C2, 1, 1), (t(24), t(19, 2), 1, 0), (t(25, 3), X, 1, 0)],
    ]
    offs, cols = [0], ([], [], [], [])
    for nodes in colls:
        for x in nodes:
            for k in range(4):
                cols[k].append(x[k])
        offs.append(len(cols[0]))
    return (np.array(offs, np.uint64), np.array(cols[0], np.uint64), np.array(cols[1], np.uint64),
            np.array(cols[2], np.uint8), np.array(cols[3], np.uint8)), (ID_KEY | X, [0, 2, 1, 3])


def test_self_caused_id_key(weaver):
    """the id key weave of a self-caused id X folds X, its
    children and grandchildren by their real causes (map.cljc:30-45,
    shared.cljc:225-241), on the fused, small and pipeline paths."""
    (off, idk, ck, ci, kd), (xkey, xweave) = self_cause_collections()
    res = check(weaver, off, idk, ck, ci, kd, 2)
    got = gpu_maps(res, len(off) - 1)
    assert got[0][xkey][1] == xweave
    assert res.status[0] & abi.STATUS_NON_LAMPORT  # X's cause is X: folded literally
    assert res.status[2] == 0  # a two-cycle stays chained, nothing to flag
    # the same collections amid a batch of clean ones (packs, tiles, chunks)
    spec = gen.MapSpec(nodes_per_coll=60, p_bad=0.05, seed=31)
    _, tb = spec.layout()
    o2, i2, c2, ci2, k2 = gen.generate_maps(spec, 0, 300, nthreads=4)
    cat = lambda a, b: np.concatenate([a, b])
    off3 = np.concatenate([o2, o2[-1] + off[1:]])
    check(weaver, off3, cat(i2, idk), cat(c2, ck), cat(ci2, ci), cat(k2, kd), max(2, tb))


@pytest.mark.parametrize("n_lo,n_hi,colls", [(3000, 6000, 4), (15000, 20000, 2)])
def test_large_literal_collections(weaver, n_lo, n_hi, colls):
    """Collections past the fused path's pack (> 2048 nodes: the general path
    on every weaver) with root-id, nil, absent and non-Lamport causes."""
    off, idk, ck, ci, kd = literal_histories(random.Random(n_lo), colls, n_lo, n_hi)
    res = check(weaver, off, idk, ck, ci, kd, 2)
    assert (res.status & abi.STATUS_NON_LAMPORT).any()
    nil = res.seg_key == np.uint64(NIL)
    assert nil.sum() == colls  # one nil key weave per collection (absent, root-id, nil causes)


def test_repeat_calls_identical(weaver):
    spec = gen.CONFIG4
    _, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 10, 510, nthreads=8)
    a = weaver.weave_maps(off, idk, ck, ci, kd, tb)
    # a list call in between replaces the cached tables
    loff, li, lc, lk = gen.generate(gen.GenSpec(nodes_per_doc=300, n_sites=3), 0, 5)
    weaver.weave_lists(loff, li, lc, lk, gen.GenSpec(nodes_per_doc=300, n_sites=3).layout())
    b = weaver.weave_maps(off, idk, ck, ci, kd, tb)
    for f in ("seg_offsets", "seg_coll", "seg_key", "seg_active", "seg_perm", "status"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f))


def test_device_memory_call_matches_host(weaver):
    """cw_weave_maps with CW_MEM_DEVICE (what bench.py --config 4 times) gives
    the host-memory call's key weaves and active nodes."""
    import torch

    spec = gen.CONFIG4
    lay, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 500, nthreads=8)
    host = weaver.weave_maps(off, idk, ck, ci, kd, tb, lay.key_bits)
    dev = torch.device("cuda", 0)
    g = [torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
         for x in (idk, ck, ci, kd)]
    N, D = len(idk), len(off) - 1
    o = {"seg_offsets": torch.zeros(N + 1, dtype=torch.int64, device=dev),
         "seg_coll": torch.zeros(N, dtype=torch.int32, device=dev),
         "seg_key": torch.zeros(N, dtype=torch.int64, device=dev),
         "seg_active": torch.zeros(N, dtype=torch.int64, device=dev),
         "seg_perm": torch.zeros(2 * N, dtype=torch.int32, device=dev),
         "status": torch.zeros(D, dtype=torch.int32, device=dev)}
    S = weaver.weave_maps_device(off, [x.data_ptr() for x in g], tb, lay.key_bits,
                                 {k: v.data_ptr() for k, v in o.items()}, N)
    assert S == len(host.seg_key)
    np.testing.assert_array_equal(o["seg_offsets"][:S + 1].cpu().numpy().view(np.uint64),
                                  host.seg_offsets)
    np.testing.assert_array_equal(o["seg_key"][:S].cpu().numpy().view(np.uint64), host.seg_key)
    np.testing.assert_array_equal(o["seg_active"][:S].cpu().numpy(), host.seg_active)
    np.testing.assert_array_equal(o["seg_perm"][:N + S].cpu().numpy().view(np.uint32),
                                  host.seg_perm)
    np.testing.assert_array_equal(o["status"].cpu().numpy().view(np.uint32), host.status)


def test_device_calls_with_a_changed_layout_are_rechecked(weaver):
    """Device-memory calls take the previous call's pack table on trust when
    the collection count and a few offsets agree, and compare the whole layout
    while the kernel runs: a layout that differs elsewhere (two neighbouring
    collections trading nodes) is woven again from a fresh table."""
    import torch

    spec = gen.CONFIG4
    lay, tb = spec.layout()
    off, idk, ck, ci, kd = gen.generate_maps(spec, 0, 6000, nthreads=8)
    D, N = len(off) - 1, len(idk)
    # the same nodes, collections 10 and 11 re-split: every node of 11 joins 10
    # except its last one (the offsets at D, D/2 and D/3 stay)
    off2 = off.copy()
    off2[11] = off[12] - 1
    dev = torch.device("cuda", 0)
    g = [torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
         for x in (idk, ck, ci, kd)]

    def call(o_off):
        o = {"seg_offsets": torch.zeros(N + 1, dtype=torch.int64, device=dev),
             "seg_coll": torch.zeros(N, dtype=torch.int32, device=dev),
             "seg_key": torch.zeros(N, dtype=torch.int64, device=dev),
             "seg_active": torch.zeros(N, dtype=torch.int64, device=dev),
             "seg_perm": torch.zeros(2 * N, dtype=torch.int32, device=dev),
             "status": torch.zeros(D, dtype=torch.int32, device=dev)}
        S = weaver.weave_maps_device(o_off, [x.data_ptr() for x in g], tb, lay.key_bits,
                                     {k: v.data_ptr() for k, v in o.items()}, N)
        return S, {k: v.cpu().numpy() for k, v in o.items()}

    for o_off in (off, off2, off2, off):
        S, h = call(o_off)
        host = weaver.weave_maps(o_off, idk, ck, ci, kd, tb, lay.key_bits)
        assert S == len(host.seg_key)
        np.testing.assert_array_equal(h["seg_offsets"][:S + 1].view(np.uint64), host.seg_offsets)
        np.testing.assert_array_equal(h["seg_coll"][:S].view(np.uint32), host.seg_coll)
        np.testing.assert_array_equal(h["seg_key"][:S].view(np.uint64), host.seg_key)
        np.testing.assert_array_equal(h["seg_active"][:S], host.seg_active)
        np.testing.assert_array_equal(h["seg_perm"][:N + S].view(np.uint32), host.seg_perm)
        np.testing.assert_array_equal(h["status"].view(np.uint32), host.status)
