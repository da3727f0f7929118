"""The distributed giant-list weave (cause_amd/giant.py, BASELINE config 5) on
CPU: gloo ranks, the kernels replaced by the numpy/oracle double
tests/giant_cpu_ops.py.  Each rank holds a random share of one list's nodes in
random order; the gathered weave must equal the oracle's weave of the whole
list (global input index = rank offset + local index)."""
import dataclasses
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from cause_amd import gen, giant


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def make_list(n, seed):
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n, seed=seed)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=1)
    return spec, idk, ck, kd


def shares(N, W, seed, empty_rank=None):
    """A random split of 0..N-1 into W shares (random order inside each)."""
    rng = np.random.default_rng(seed)
    owner = rng.integers(0, W, N)
    if empty_rank is not None:
        owner[owner == empty_rank] = (empty_rank + 1) % W
    return [rng.permutation(np.flatnonzero(owner == r)) for r in range(W)]


def _worker(rank, world, port, n, seed, samples, empty_rank, tree, q, opts=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.giant_cpu_ops import CpuOps

        spec, idk, ck, kd = make_list(n, seed)
        sh = shares(len(idk), world, seed, empty_rank)[rank]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
        lay = spec.layout()
        res = giant.weave_distributed(CpuOps(), t(idk[sh]), t(ck[sh]),
                                      torch.from_numpy(kd[sh].copy()), lay.key_bits,
                                      ts_shift=lay.ts_shift, samples=samples, tree=tree,
                                      **(opts or {}))
        if (opts or {}).get("out") == "sharded":
            q.put(("part", rank, res.pos_base, res.weave_perm.numpy().copy(),
                   res.visible_bits.numpy().copy(), res.visible_count, res.status, res.n_total,
                   res.max_ts))
        elif rank == 0:
            q.put((res.weave_perm.numpy().copy(), res.visible_count, res.status, res.n_total,
                   res.max_ts))
        q.put(("own", rank, res.n_owned))
        if rank == 0:
            q.put(("rk", res.ranking))
    finally:
        dist.destroy_process_group()


def run(world, n, seed, samples=64, empty_rank=None, tree="auto", **opts):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker,
                      args=(r, world, port, n, seed, samples, empty_rank, tree, q, opts))
          for r in range(world)]
    for p in ps:
        p.start()
    sharded = opts.get("out") == "sharded"
    got, owned, parts = None, {}, []
    for _ in range(2 * world + 1 if sharded else world + 2):
        m = q.get(timeout=120)
        if isinstance(m[0], str) and m[0] == "part":
            parts.append(m)
        elif isinstance(m[0], str) and m[0] == "rk":
            run.ranking = m[1]
        elif isinstance(m[0], str):
            owned[m[1]] = m[2]
        else:
            got = m
    if sharded:
        # the slices in position order: weave_perm and render bits of the whole list
        parts.sort(key=lambda m: m[2])
        N = parts[0][7]
        pos = 0
        for m in parts:
            assert m[2] == pos and (m[2] % 32 == 0)
            pos += len(m[3])
        assert pos == N and len({m[5] for m in parts}) == 1
        st = 0
        for m in parts:
            st |= m[6]
        wp = np.concatenate([m[3] for m in parts])
        bits = np.concatenate([np.unpackbits(m[4].view(np.uint8), bitorder="little")[:len(m[3])]
                               for m in parts])
        got = (wp, parts[0][5], st, N, parts[0][8], bits)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return got, owned


@pytest.mark.parametrize("tree", ["dist", "root"])
@pytest.mark.parametrize("world,n,seed,empty", [(2, 3000, 11, None), (3, 5000, 12, None),
                                                (4, 2000, 13, 2)])
def test_distributed_weave_matches_oracle(world, n, seed, empty, tree):
    """tree="dist": effective parents, sibling runs and threads rank by rank
    (dist.hip's numpy double); "root": the whole tree on rank 0."""
    (wp, vcount, status, N, max_ts), owned = run(world, n, seed, empty_rank=empty, tree=tree)
    spec, idk, ck, kd = make_list(n, seed)
    assert N == len(idk) and sum(owned.values()) == N
    perm, vis, st = oracle.batch_lists(np.array([0, N], np.uint64), idk, ck, kd,
                                       method=oracle.METHOD_EFF)
    # global input index -> node of the whole list
    sh = np.concatenate(shares(N, world, seed, empty))
    assert status == 0 and not st.any()
    assert np.array_equal(sh[wp.view(np.uint32)], perm)
    assert vcount == int(vis.sum())
    assert max_ts == int(idk.max()) >> spec.layout().ts_shift
    # the sample sort balances the owners
    assert max(owned.values()) < 2.0 * N / world


@pytest.mark.parametrize("world,n,seed,empty,k,out", [
    (1, 3000, 21, None, 16, "root"), (2, 4000, 22, None, 16, "root"),
    (3, 5000, 23, None, 4, "sharded"), (4, 3000, 24, 1, 16, "sharded"),
    (2, 2500, 25, None, 1, "root"), (2, 2500, 26, None, 1000, "sharded")])
def test_ruling_set_ranking_matches_oracle(world, n, seed, empty, k, out):
    """The list ranked where it lies (giant._rank_ruling, dist.hip k_rs_*'s numpy
    double): rulers every ~k nodes walk their sublists, walkers crossing ranks
    travel as all-to-all messages, the ruler links are ranked on rank 0, and the
    weave lands on rank 0 or spread by position.  k = 1 (every node a ruler)
    and k = 1000 (a few long walks) bound the density."""
    got, owned = run(world, n, seed, empty_rank=empty, tree="dist", ranking="ruling",
                     out=out, ruler_k=k)
    wp, vcount, status, N = got[:4]
    spec, idk, ck, kd = make_list(n, seed)
    perm, vis, st = oracle.batch_lists(np.array([0, N], np.uint64), idk, ck, kd,
                                       method=oracle.METHOD_EFF)
    sh = np.concatenate(shares(N, world, seed, empty))
    assert status == 0 and not st.any()
    assert np.array_equal(sh[wp.view(np.uint32)], perm)
    assert vcount == int(vis.sum())
    if out == "sharded":
        assert np.array_equal(got[5], vis)


def test_ruling_set_rounds_and_messages_at_w8():
    """A config-5 list over 8 ranks (DESIGN.md §6 study): every crossing step
    of the list is one walker message -- ~0.4 per node at W = 8 -- and the
    rounds are the most crossings of any sublist (K = 16: ~50-120 at this
    size), with the weave still the oracle's."""
    n, seed = 20_000, 27
    got, owned = run(8, n, seed, tree="dist", ranking="ruling")
    wp, vcount, status, N = got[:4]
    spec, idk, ck, kd = make_list(n, seed)
    perm, vis, st = oracle.batch_lists(np.array([0, N], np.uint64), idk, ck, kd,
                                       method=oracle.METHOD_EFF)
    sh = np.concatenate(shares(N, 8, seed))
    assert status == 0 and np.array_equal(sh[wp.view(np.uint32)], perm)
    info = run.ranking
    assert info["ruler_k"] == 16 and 0.04 < info["rulers"] / N < 0.09, info
    assert 0.3 < info["messages"] / N < 0.5, info
    assert 20 < info["rounds"] < 200, info
    # one host readback a round: the all_gather of the bucket sizes is both the
    # exchange's split sizes and the termination test
    assert info["syncs_per_round"] <= 1.0, info


def _dup_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.giant_cpu_ops import CpuOps

        spec, idk, ck, kd = make_list(3000, 31)
        sh = shares(len(idk), world, 31)[rank]
        if rank == 1:  # rank 1 also holds a copy of a node rank 0 owns
            sh = np.concatenate([sh, shares(len(idk), world, 31)[0][:1]])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
        lay = spec.layout()
        res = giant.weave_distributed(CpuOps(), t(idk[sh]), t(ck[sh]),
                                      torch.from_numpy(kd[sh].copy()), lay.key_bits,
                                      ts_shift=lay.ts_shift, samples=64)
        if rank == 0:
            q.put(res.status)
    finally:
        dist.destroy_process_group()


def test_distributed_weave_flags_an_id_held_by_two_ranks():
    """The same id on two ranks is a duplicate of the one ::nodes map
    (shared.cljc:166-171): the owner sees it repeated and the root's status has
    CW_STATUS_DUP, as the single-GPU path reports."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    status = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert status & 2  # CW_STATUS_DUP


def test_choose_splitters_weighted():
    s = np.arange(100, dtype=np.int64)
    w = np.ones(100)
    assert list(giant.choose_splitters(s, w, 4)) == [24, 49, 74]
    # a rank with 10x the nodes but the same number of samples weighs 10x
    s2 = np.concatenate([np.arange(0, 50), np.arange(50, 100)]).astype(np.int64)
    w2 = np.concatenate([np.full(50, 10.0), np.full(50, 1.0)])
    assert giant.choose_splitters(s2, w2, 2)[0] < 50
    assert len(giant.choose_splitters(np.zeros(0, np.int64), np.zeros(0), 3)) == 0


def _orphan_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.giant_cpu_ops import CpuOps

        class Ops(CpuOps):
            linked = 0

            def weave_linked(self, *a):
                Ops.linked += 1
                return super().weave_linked(*a)

        spec, idk, ck, kd = make_list(2000, 41)
        ck = ck.copy()
        ck[7] = idk.max() + np.uint64(5)   # a cause that is no node: an orphan
        sh = shares(len(idk), world, 41)[rank]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
        lay = spec.layout()
        res = giant.weave_distributed(Ops(), t(idk[sh]), t(ck[sh]), torch.from_numpy(kd[sh].copy()),
                                      lay.key_bits + 1, ts_shift=lay.ts_shift, samples=64,
                                      tree="dist")
        if rank == 0:
            q.put((res.status, Ops.linked))
    finally:
        dist.destroy_process_group()


def test_distributed_tree_leaves_out_of_domain_lists_to_the_root():
    """A list with an orphan cause is outside the fast path's domain: every rank's
    cw_dist_check sees it and the list goes to the rank-0 weave (and its exact
    path) instead of the tree by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_orphan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    status, linked = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert status & 4 and linked == 0  # CW_STATUS_ORPHAN, no cw_weave_linked


def test_config5_list_order_crosses_ranks():
    """Why the list ranking stays on the gathering GPU: in a
    config-5 list the preorder successor of a node lies on another rank of the
    id order for ~21% of the nodes at W = 2 and ~42% at W = 8 (30% of causes
    are uniformly random earlier nodes, whose newest child follows them), so
    rank-local sublists would be a few nodes long and a distributed ranking
    pays O(N) cross-rank messages."""
    spec, idk, ck, kd = make_list(200_000, 5)
    off = np.array([0, len(idk)], np.uint64)
    p, _, _ = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF)
    rank = np.empty(len(idk), np.int64)
    rank[np.argsort(idk, kind="stable")] = np.arange(len(idk))
    r = rank[p.astype(np.int64)]
    N = len(idk)
    frac = {W: np.count_nonzero(np.diff(r * W // N)) / N for W in (2, 8)}
    assert 0.15 < frac[2] < 0.3 and 0.35 < frac[8] < 0.5, frac
