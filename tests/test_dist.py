"""Multi-rank document sharding on CPU (gloo, world_size 2).

Each rank weaves its own contiguous document shard (here with the CPU oracle:
no GPU in this container; on the GPU box the same shard goes through
cw_weave_lists) and the ranks combine only bookkeeping: a MAX of times and a
SUM of counters.  The combined result must equal weaving the whole batch in
one process.
"""
import dataclasses
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from cause_amd import gen, shard

SPEC = dataclasses.replace(gen.CONFIG2, nodes_per_doc=400)
DOCS_PER_RANK = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = shard.doc_range(rank, world, docs_per_rank=DOCS_PER_RANK)
        off, idk, ck, kd = gen.generate(SPEC, b, e, nthreads=2)
        perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=2)
        checksum = int((perm.astype(np.uint64) * np.arange(1, len(perm) + 1, dtype=np.uint64)).sum()
                       % np.uint64(2**61 - 1))
        nodes, visible, bad = shard.reduce_sum([len(idk), int(vis.sum()), int(st.sum())], dist)
        t = shard.reduce_max_time(0.5 + rank, dist)
        cs = shard.reduce_sum([checksum], dist)[0]
        if rank == 0:
            out.put((nodes, visible, bad, t, cs))
    finally:
        dist.destroy_process_group()


def test_doc_range_weak_and_strong():
    assert [shard.doc_range(r, 4, docs_per_rank=10) for r in range(4)] == \
        [(0, 10), (10, 20), (20, 30), (30, 40)]
    parts = [shard.doc_range(r, 3, total_docs=10) for r in range(3)]
    assert parts == [(0, 4), (4, 7), (7, 10)]
    with pytest.raises(ValueError):
        shard.doc_range(0, 2)


def test_two_rank_gloo_sharding_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    nodes, visible, bad, t, cs = q.get(timeout=10)
    # the same documents in one process
    off, idk, ck, kd = gen.generate(SPEC, 0, world * DOCS_PER_RANK, nthreads=2)
    perm, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=2)
    assert nodes == len(idk)
    assert visible == int(vis.sum())
    assert bad == 0
    assert t == 1.5  # MAX over ranks (0.5, 1.5)
    # checksums are per shard; recompute them shard by shard here
    want = 0
    n_per = SPEC.doc_size * DOCS_PER_RANK
    for r in range(world):
        p = perm[r * n_per:(r + 1) * n_per].astype(np.uint64)
        want += int((p * np.arange(1, len(p) + 1, dtype=np.uint64)).sum() % np.uint64(2**61 - 1))
    assert cs == want
