"""Benchmark: nodes woven/s for BASELINE.json configs[1] on MI355X.

Workload (per GPU, weak scaling): 10,000 independent CausalLists of 50,001
nodes each (root + 50,000 nodes from 8 sites: 10% hides, 2% h.shows, 5%
conj-style causes), node order shuffled inside each
document.  One step = one full reweave of the GPU's whole batch through the C
ABI (cw_weave_lists, device memory): sorted ids, parents, weave order, rendered
bits and counts per document.  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--docs", type=int, default=10_000, help="documents per GPU")
    ap.add_argument("--nodes", type=int, default=50_000, help="non-root nodes per document")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="budget of the cpu_baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-refresh", action="store_true",
                    help="skip the refresh_caches (yarns) steps: PMC passes count the weave alone")
    ap.add_argument("--no-h2d", action="store_true", help="skip the PCIe-inclusive pass")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="BASELINE.json configs[config-1]: 2 = the headline batch "
                         "(default), 1 = one 100k-node list (latency; replicas on N GPUs), "
                         "3 = --stream-docs documents streamed from host memory in --docs "
                         "batches (sharded over N GPUs), "
                         "4 = CausalMap collections (10^6 x 100 nodes per GPU), "
                         "5 = one giant list (--giant nodes; replicas on N GPUs)")
    ap.add_argument("--stream-docs", type=int, default=1_000_000,
                    help="--config 3: documents in the whole job (all GPUs)")
    ap.add_argument("--depth", type=int, default=2, help="--config 3: pipeline slots")
    ap.add_argument("--tree", default="auto", choices=["auto", "dist", "root"],
                    help="--config 5 --dist: the tree rank by rank (dist) or on rank 0 (root); "
                         "auto = dist for N > 1")
    ap.add_argument("--keys", type=int, default=64, choices=[32, 64],
                    help="configs 1/2/5: key words of the resident inputs (32 = cw_weave_lists_k32)")
    ap.add_argument("--k64", action="store_true",
                    help="--config 3: stream 8-byte keys (cw_weave_lists) instead of K32")
    ap.add_argument("--no-prestaged", action="store_true",
                    help="--config 3: skip the pass with the inputs pre-staged in host memory")
    ap.add_argument("--giant", type=int, default=1 << 26, help="--config 5: nodes in the list")
    ap.add_argument("--ranking", default="auto", choices=["auto", "ruling", "root"],
                    help="--config 5 --dist with the tree by rank: list ranking by a ruling set "
                         "where the list lies (ruling) or on rank 0 (root); auto = ruling for N > 1")
    ap.add_argument("--out", default="root", choices=["root", "sharded"],
                    help="--config 5 --dist --ranking ruling: the weave on rank 0, or spread "
                         "over the ranks by weave position")
    ap.add_argument("--ruler-k", type=int, default=16,
                    help="--config 5 --ranking ruling: one ruler per ~K nodes")
    ap.add_argument("--colls", type=int, default=1_000_000, help="--config 4: collections per GPU")
    ap.add_argument("--dist", action="store_true",
                    help="--config 5 on one GPU through the distributed path (sample sort, "
                         "exchange, gather; always taken when N > 1)")
    ap.add_argument("--cache", default=None,
                    help="configs 1/2/5: save the generated input under this directory, or load "
                         "it from there when present (several profiler passes, one generation)")
    ap.add_argument("--check", action="store_true",
                    help="after timing, every rank compares its outputs with the CPU oracle "
                         "(configs 2, 3 and 4; the JSON line gets a 'check' object)")
    ap.add_argument("--check-docs", type=int, default=256,
                    help="without --check: the last timed step's outputs of this many documents "
                         "(configs 1/2/5; collections for config 4) spread over the batch are "
                         "compared with the oracle after timing (0: off)")
    return ap.parse_args()


def launch_ranks(a) -> int:
    """`python bench.py --gpus N` without a launcher: start N ranks (one process
    per GPU) through torch.distributed.run as a CHILD process, before this
    process touches the GPU, and return its exit code.  Rank 0 prints the line."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def _k64(*keys):
    """K32 words -> the K64 keys they stand for (reserved top words sign-extend);
    K64 keys pass through."""
    out = []
    for x in keys:
        if x.dtype == np.uint32:
            x = np.where(x >= 0xFFFFFFF0, x.view(np.int32).astype(np.int64).view(np.uint64),
                         x.astype(np.uint64))
        out.append(x)
    return out


def check_lists(off, idk, ck, kd, perm, bits, vcount, status):
    """--check: this rank's config-2 outputs vs the oracle (effective-tree
    preorder in C, itself pinned to the literal fold by the tests): mismatching
    documents."""
    import oracle

    want, vis, st = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=16)
    got = perm.cpu().numpy().view(np.uint32)
    gvis = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:len(got)]
    gst = status.cpu().numpy().view(np.uint32)
    gvc = vcount.cpu().numpy().view(np.uint32)
    bad = 0
    for d in range(len(off) - 1):
        lo, hi = int(off[d]), int(off[d + 1])
        ok = (gst[d] == st[d] and np.array_equal(got[lo:hi], want[lo:hi]) and
              np.array_equal(gvis[lo:hi], vis[lo:hi]) and int(gvc[d]) == int(vis[lo:hi].sum()))
        bad += 0 if ok else 1
    return bad


def sample_docs(D, k):
    """k document indices spread evenly over [0, D) (all of them if D <= k)."""
    if D <= k:
        return np.arange(D, dtype=np.int64)
    return np.unique(np.linspace(0, D - 1, k).round().astype(np.int64))


def snapshot_lists(off, docs, perm, bits, vcount, status):
    """Device outputs of the sampled documents, copied to the host right after
    the timed steps (so later untimed calls cannot be what gets checked)."""
    snap = []
    for d in docs:
        lo, hi = int(off[d]), int(off[d + 1])
        w0, w1 = lo >> 5, (hi + 31) >> 5
        snap.append((int(d), perm[lo:hi].cpu().numpy().view(np.uint32).copy(),
                     bits[w0:w1].cpu().numpy().view(np.uint32).copy(),
                     int(vcount[d].item()), int(status[d].item())))
    return snap


def check_snapshot_lists(off, idk, ck, kd, snap):
    """The timed step's outputs of the sampled documents vs the oracle
    (effective-tree preorder + visibility in C, pinned to the literal fold by
    tests/test_fullsize_literal.py) -> (documents checked, mismatches)."""
    import oracle

    sizes = [int(off[d + 1] - off[d]) for d, *_ in snap]
    sub_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    sel = np.concatenate([np.arange(int(off[d]), int(off[d + 1])) for d, *_ in snap])
    want, vis, st = oracle.batch_lists(sub_off, idk[sel], ck[sel], kd[sel],
                                       method=oracle.METHOD_EFF, nthreads=16)
    bad = 0
    for j, (d, gp, gb, gvc, gst) in enumerate(snap):
        lo, hi = int(off[d]), int(off[d + 1])
        a, b = int(sub_off[j]), int(sub_off[j + 1])
        allbits = np.unpackbits(gb.view(np.uint8), bitorder="little")
        gvis = allbits[lo - ((lo >> 5) << 5):][:hi - lo]
        ok = (gst == st[j] and np.array_equal(gp, want[a:b]) and
              np.array_equal(gvis, vis[a:b]) and gvc == int(vis[a:b].sum()))
        bad += 0 if ok else 1
    return len(snap), bad


def check_maps(off, idk, ck, ci, kd, o, S, colls=None):
    """This rank's config-4 key weaves and active nodes vs the literal
    c.map/weave fold (oracle/weave_oracle.c), for every collection or only
    `colls` -> (mismatching collections, collections checked)."""
    import oracle

    h = {k: v.cpu().numpy() for k, v in o.items()}
    so, sc, sk = h["seg_offsets"].view(np.uint64), h["seg_coll"].view(np.uint32), h["seg_key"].view(np.uint64)
    sa, sp, gst = h["seg_active"], h["seg_perm"].view(np.uint32), h["status"].view(np.uint32)
    D = len(off) - 1
    todo = range(D) if colls is None else [int(c) for c in colls]
    want_set = set(todo)
    got = [dict() for _ in range(D)]
    for s in range(S):
        c = int(sc[s])
        if c not in want_set:
            continue
        kw = sp[int(so[s]):int(so[s + 1])]
        got[c][int(sk[s])] = (int(sa[s]), kw[1:].tolist() if kw[0] == 0xFFFFFFFF else None)
    tok, idk_bit, nil = np.uint64(1 << 63), 1 << 63, (1 << 64) - 1
    bad = 0
    for d in todo:
        a, b = int(off[d]), int(off[d + 1])
        c = oracle.map_causes(ck[a:b], ci[a:b])
        nk, npos, skk, saa = oracle.map_weave(idk[a:b], c, ci[a:b], kd[a:b], 0)
        order = np.lexsort((npos, nk))
        groups = {}
        for j in order:
            groups.setdefault(int(nk[j]), []).append(int(j))
        api = lambda k: nil if k == nil else (k & ~idk_bit if k & idk_bit else idk_bit | k)
        want = {api(int(k)): (int(act), groups.get(int(k), [])) for k, act in zip(skk, saa)}
        bad += 0 if (gst[d] == 0 and got[d] == want) else 1
    return bad, len(todo)


class heartbeat:
    """Prints a progress line to stderr every `every` seconds while a long host
    step (the generator of a giant list) runs."""

    def __init__(self, what, every=30.0):
        import threading

        self.what, self.every, self.stop = what, every, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(self.every):
            print(f"[bench] {self.what}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self.t.join()


def b_io_bytes(key_bytes, perm_bytes):
    """SURVEY 8(d)'s algorithmic bytes per node of the weave: id + cause keys
    and the kind byte in, weave_perm and one visible bit out."""
    return key_bytes + key_bytes + 1 + perm_bytes + 1 / 8


def achieved_gbs(bytes_per_launch, launches, ms_total):
    """GB/s of a kernel over the timed steps: its bytes per launch times the
    launches, over the summed launch time (launches and ms both over ALL the
    timed steps, as cw_get_kernel_stats reports them)."""
    return bytes_per_launch * launches / (ms_total / 1e3) / 1e9 if ms_total > 0 else 0.0


def pmc_traffic(kernel, workload, default_size):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, scripts/pmc_traffic.py: FETCH_SIZE doubled per
    MI355X_MICROARCH.md), only when they were measured on THIS library build
    (cw_build_id) and this workload at its default size.  -> (bytes or None, note)."""
    from cause_amd import abi

    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not default_size:
        return None, "no PMC pass at this size"
    if not os.path.exists(path):
        return None, "profiles/pmc_traffic.json missing"
    t = json.load(open(path))
    bid = abi.build_id()
    if t.get("build_id") != bid:
        return None, (f"stale counters: measured on build {t.get('build_id')}, "
                      f"this library is build {bid}")
    entry = t.get("workloads", {}).get(workload, {}).get(kernel)
    if not entry:
        return None, f"no PMC pass of kernel {kernel} on {workload}"
    return entry["bytes"], (f"rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE per launch, "
                            f"{workload}, build {bid}")


def cpu_baseline_prefix(idk, ck, kd, prefix):
    """Config 5: the literal fold is quadratic, so it runs on the id-order prefix
    of `prefix` nodes of the same list (causally closed: causes are older)."""
    import oracle

    if len(idk) > prefix:  # the prefix without sorting the whole list
        thr = np.partition(idk, prefix - 1)[prefix - 1]
        sel = np.flatnonzero(idk <= thr)
        o = sel[np.argsort(idk[sel], kind="stable")][:prefix]
    else:
        o = np.argsort(idk, kind="stable")
    t0 = time.perf_counter()
    _, st = oracle.list_weave(idk[o], ck[o], kd[o], oracle.METHOD_LITERAL)
    t = time.perf_counter() - t0
    return {"value": prefix / t, "unit": "nodes/s", "cores": 1, "kind": "port",
            "sample": f"literal weave-node fold (shared.cljc:194-241) in C on the first {prefix:,} "
                      f"nodes (id order) of the same list, {t:.1f} s; the fold is quadratic, so "
                      f"the whole list would run far slower than this rate"}


def cpu_baseline(spec, budget_s, max_docs=64):
    """The reference algorithm (literal weave-node fold, oracle/weave_oracle.c,
    one core) on the first documents of this same workload, until ~budget_s."""
    import oracle

    done_nodes, t_total, ndocs = 0, 0.0, 0
    from cause_amd import gen

    while t_total < budget_s and ndocs < max_docs:
        off, idk, ck, kd = gen.generate(spec, ndocs, ndocs + 1, nthreads=1)
        t0 = time.perf_counter()
        _, st = oracle.list_weave(idk, ck, kd, oracle.METHOD_LITERAL)
        t_total += time.perf_counter() - t0
        done_nodes += len(idk)
        ndocs += 1
    return {"value": done_nodes / t_total, "unit": "nodes/s", "cores": 1, "kind": "port",
            "sample": f"{ndocs} documents x {spec.doc_size} nodes of the same workload, "
                      f"literal weave-node fold (shared.cljc:194-241, list.cljc:26-28) "
                      f"in C, {t_total:.1f} s"}


def cpu_baseline_parallel(spec, docs=2000, threads=16):
    """A stronger CPU reference point than the literal fold: the effective-tree
    preorder (oracle/weave_oracle.c) over `docs` documents of this
    workload on `threads` host threads (the box's CPU share)."""
    import oracle
    from cause_amd import gen

    off, idk, ck, kd = gen.generate(spec, 0, docs, nthreads=threads)
    t0 = time.perf_counter()
    oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF, nthreads=threads,
                       with_vis=True)
    t = time.perf_counter() - t0
    return {"value": len(idk) / t, "unit": "nodes/s", "cores": threads, "kind": "port",
            "sample": f"{docs} documents x {spec.doc_size} nodes of the same workload, "
                      f"effective-tree preorder + visibility (SURVEY F5/F6) in C on "
                      f"{threads} threads, {t:.2f} s"}


def cpu_baseline_maps(spec, budget_s):
    """The literal c.map/weave fold (oracle/weave_oracle.c or_map_fold_literal,
    map.cljc:21-59) on one core, collection by collection, until ~budget_s."""
    import oracle
    from cause_amd import gen

    done, t_total, colls = 0, 0.0, 0
    tok = np.uint64(1 << 63)
    while t_total < budget_s and colls < 200_000:
        off, idk, ck, ci, kd = gen.generate_maps(spec, colls, colls + 1000, nthreads=1)
        c = oracle.map_causes(ck, ci)
        t0 = time.perf_counter()
        for d in range(1000):
            a, b = int(off[d]), int(off[d + 1])
            oracle.map_weave(idk[a:b], c[a:b], ci[a:b], kd[a:b], 0)
        t_total += time.perf_counter() - t0
        done += len(idk)
        colls += 1000
    return {"value": done / t_total, "unit": "nodes/s", "cores": 1, "kind": "port",
            "sample": f"{colls} collections x {spec.nodes_per_coll} nodes of the same workload, "
                      f"literal map weave + active-node (map.cljc:21-59) in C, {t_total:.1f} s"}


def check_giant_dist(res, idk, ck, kd, world, rank, dist, N, sharded):
    """--check for --config 5 --dist: the weave (on rank 0, or its slices
    gathered there) against the oracle's weave of the whole list (rank r holds
    nodes r, r + world, ... of the generation order)."""
    import oracle

    parts = None
    if sharded:
        parts = [None] * world
        dist.all_gather_object(parts, (res.pos_base, res.weave_perm.cpu().numpy(),
                                       res.visible_bits.cpu().numpy()))
    if rank != 0:
        return
    if parts is not None:
        parts.sort(key=lambda p: p[0])
        wp = np.concatenate([p[1] for p in parts]).view(np.uint32)
        vis = np.concatenate([np.unpackbits(p[2].view(np.uint8), bitorder="little")[:len(p[1])]
                              for p in parts])
    else:
        wp = res.weave_perm.cpu().numpy().view(np.uint32)
        vis = np.unpackbits(res.visible_bits.cpu().numpy().view(np.uint8), bitorder="little")[:N]
    # global input index: rank r's local i is node r + i * world
    counts = [len(range(r, N, world)) for r in range(world)]
    start = np.concatenate([[0], np.cumsum(counts)[:-1]])
    r_of = np.repeat(np.arange(world), counts)
    node = r_of + (np.arange(N) - start[r_of]) * world
    perm, want_vis, st = oracle.batch_lists(np.array([0, N], np.uint64), idk, ck, kd,
                                            method=oracle.METHOD_EFF)
    ok = bool(np.array_equal(node[wp], perm)) and bool(np.array_equal(vis, want_vis))
    print(json.dumps({"check": "config5 dist", "nodes": N, "ok": ok}), flush=True)
    if not ok:
        raise SystemExit("config 5 --check: the weave differs from the oracle")


def main_giant_dist(a, world, rank, local, dist, torch, dev):
    """--config 5 on N GPUs: ONE list of --giant nodes whose nodes are spread
    over the ranks (rank r holds every N-th node of the generation order).
    One step = cause_amd.giant.weave_distributed: local sort, sample sort by
    all_to_all (RCCL), cause join at the owners, then (--tree dist, the
    default for N > 1) the tree rank by rank with all-to-all rounds and the
    successors gathered on rank 0 for the list ranking, or (--tree root) the
    rank-ordered arrays gathered on rank 0 and the whole tree + tour there.
    Strong scaling: the list is the same at every N."""
    import dataclasses

    from cause_amd import abi, gen, giant

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.giant)
    lay = spec.layout()
    tree_dist = a.tree == "dist" or (a.tree == "auto" and world > 1)
    ruling = tree_dist and (a.ranking == "ruling" or (a.ranking == "auto" and world > 1))
    t0 = time.time()
    with heartbeat("generating the input"):
        off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=16)
    t_gen = time.time() - t0
    N = len(idk)
    sel = slice(rank, N, world)
    g_id = torch.from_numpy(np.ascontiguousarray(idk[sel]).view(np.int64)).to(dev)
    g_ca = torch.from_numpy(np.ascontiguousarray(ck[sel]).view(np.int64)).to(dev)
    g_kd = torch.from_numpy(np.ascontiguousarray(kd[sel])).to(dev)
    if rank != 0 or (a.no_cpu and not a.check):
        del idk, ck, kd
        idk = ck = kd = None
    torch.cuda.synchronize()
    group = None
    if world == 1:  # one rank: a private gloo group only for the (empty) exchange bookkeeping
        import socket

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        store = dist.TCPStore("127.0.0.1", port, 1, True)
        dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    w = abi.Weaver(local)
    ops = giant.HipOps(w, dev)

    def step():
        return giant.weave_distributed(ops, g_id, g_ca, g_kd, lay.key_bits, ts_shift=lay.ts_shift,
                                       group=group, tree=a.tree, ranking=a.ranking, out=a.out,
                                       ruler_k=a.ruler_k)

    res = None
    for _ in range(a.warmup):
        res = step()
    torch.cuda.synchronize()
    if res is not None and res.status not in (None, 0):
        raise SystemExit(f"status {res.status}")
    if a.check and res is not None:
        with heartbeat("--check against the oracle"):
            check_giant_dist(res, idk, ck, kd, world, rank, dist, N, ruling and a.out == "sharded")
    w.reset_kernel_stats()
    w.set_profiling(True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    w.set_profiling(False)
    stats = w.kernel_stats()
    from cause_amd import shard

    dt_max = shard.reduce_max_time(dt, dist, dev) if world > 1 else dt
    value = N * a.steps / dt_max
    if rank == 0:
        name, (launches, ms, by) = max(stats.items(), key=lambda kv: kv[1][1])
        achieved = by / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        traffic, tnote = pmc_traffic(name, f"config5dist_w{world}", a.giant == 1 << 26)
        cpu = None
        if not a.no_cpu:  # after the GPU region, on rank 0 at every N
            cpu = cpu_baseline_prefix(idk, ck, kd, 100_000)
        line = {
            "metric": "nodes woven/sec (whole node) + % of HBM roofline at 1/2/4/8 MI355X",
            "value": value, "unit": "nodes/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt_max / a.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": (f"config5: one CausalList of {N:,} nodes spread over "
                                    f"{world} rank(s), distributed sample sort + "
                                    + (f"tree by rank + {'ruling-set ranking (K=%d, weave %s)' % (a.ruler_k, 'on rank 0' if a.out == 'root' else 'sharded by position') if ruling else 'list ranking on rank 0'}"
                                       if tree_dist else "tree on rank 0")),
                       "tree": a.tree, "ranking": a.ranking if tree_dist else None,
                       "out": a.out if tree_dist and ruling else "root",
                       "nodes_total": N, "sites": spec.n_sites, "p_hide": spec.p_hide,
                       "key_bits": lay.key_bits,
                       "parallelism": f"sample sort x{world} ({dist.get_backend()})"},
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_note": tnote,
                         "launches_per_step": launches / a.steps,
                         "kernel_ms_per_step": ms / a.steps},
            "cpu_baseline": cpu,
            "kernels_ms_per_step_rank0": {k: round(v[1] / a.steps, 4) for k, v in
                                          sorted(stats.items(), key=lambda kv: -kv[1][1])},
            "kernel_sum_ms_per_step_rank0": sum(v[1] for v in stats.values()) / a.steps,
            "nodes_owned_rank0": res.n_owned, "gen_s": t_gen, "ruling_set": res.ranking,
        }
        print(json.dumps(line), flush=True)
    w.close()


def main_maps(a, world, rank, local, dist, torch, dev):
    """--config 4: a batch of CausalMaps per GPU through cw_weave_maps (device memory)."""
    from cause_amd import abi, gen, shard

    spec = gen.CONFIG4
    lay, tb = spec.layout()
    d0, d1 = shard.doc_range(rank, world, docs_per_rank=a.colls)
    t0 = time.time()
    off, idk, ck, ci, kd = gen.generate_maps(spec, d0, d1, nthreads=16)
    t_gen = time.time() - t0
    N, D = len(idk), d1 - d0
    g = [torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
         for x in (idk, ck, ci, kd)]
    cap = N
    o = {"seg_offsets": torch.empty(cap + 1, dtype=torch.int64, device=dev),
         "seg_coll": torch.empty(cap, dtype=torch.int32, device=dev),
         "seg_key": torch.empty(cap, dtype=torch.int64, device=dev),
         "seg_active": torch.empty(cap, dtype=torch.int64, device=dev),
         "seg_perm": torch.empty(N + cap, dtype=torch.int32, device=dev),
         "status": torch.empty(D, dtype=torch.int32, device=dev)}
    ptrs = [x.data_ptr() for x in g]
    outs = {k: v.data_ptr() for k, v in o.items()}
    torch.cuda.synchronize()
    w = abi.Weaver(local)
    w.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def step():
        return w.weave_maps_device(off, ptrs, tb, lay.key_bits, outs, cap)

    for _ in range(a.warmup):
        S = step()
    torch.cuda.synchronize()
    if int(o["status"].max().item()) != 0:
        raise SystemExit(f"rank {rank}: collections out of domain")
    w.reset_kernel_stats()
    w.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        S = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    w.set_profiling(False)
    stats = w.kernel_stats()
    dt_max = shard.reduce_max_time(dt, dist, dev) if world > 1 else dt
    value = N * world * a.steps / dt_max
    name, (launches, ms, by) = max(stats.items(), key=lambda kv: kv[1][1])
    achieved = by / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    traffic, tnote = pmc_traffic(name, "config4", a.colls == 1_000_000)
    check = None
    if a.check or a.check_docs > 0:
        # --check: every collection; otherwise --check-docs collections spread
        # over the batch (the last timed step's outputs: nothing ran since)
        colls = None if a.check else sample_docs(D, a.check_docs)
        with heartbeat("--check against the oracle"):
            bad, nchk = check_maps(off, idk, ck, ci, kd, o, S, colls)
        tot = shard.reduce_sum([bad, nchk], dist, dev) if world > 1 else [bad, nchk]
        check = {"collections_checked": tot[1], "mismatches": tot[0],
                 "against": "literal c.map/weave fold + active-node (oracle, C)",
                 "what": "every collection" if a.check else
                         f"{a.check_docs} collections spread evenly over each rank's batch, "
                         f"outputs of the last timed step"}
    if rank == 0:
        # timed after the GPU region, on rank 0 at every N (the other ranks are done)
        cpu = cpu_baseline_maps(spec, a.cpu_seconds) if not a.no_cpu else None
        line = {
            "metric": "nodes woven/sec (whole node) + % of HBM roofline at 1/2/4/8 MI355X",
            "value": value, "unit": "nodes/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt_max / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "config4: CausalMap collections, key weaves + active-node",
                       "colls_per_gpu": D, "nodes_per_coll": spec.nodes_per_coll,
                       "nodes_per_gpu": N, "key_weaves_per_gpu": S, "keys": spec.n_keys,
                       "zipf_s": spec.zipf_s, "parallelism": f"collections sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_note": tnote,
                         "launches_per_step": launches / a.steps,
                         "kernel_ms_per_step": ms / a.steps},
            "cpu_baseline": cpu,
            "kernels_ms_per_step": {k: round(v[1] / a.steps, 4) for k, v in
                                    sorted(stats.items(), key=lambda kv: -kv[1][1])},
            "kernel_sum_ms_per_step": sum(v[1] for v in stats.values()) / a.steps,
            "gen_s": t_gen,
        }
        if cpu:
            line["speedup_vs_cpu_baseline"] = value / cpu["value"]
        if check:
            line["check"] = check
        print(json.dumps(line), flush=True)
    w.close()


def main_stream(a, world, rank, local, dist, torch, dev):
    """--config 3: --stream-docs documents, generated on the host into pinned
    memory and streamed through the GPU in --docs batches (cause_amd/stream.py:
    fill -> H2D -> weave -> D2H, --depth slots).  Documents are sharded
    contiguously over the ranks (total fixed: strong scaling, no collectives).
    value = device-resident rate (nodes / the weaves' own time, every batch);
    end_to_end = nodes / wall time of the whole pipeline (generation, PCIe both
    ways and the weave overlapped)."""
    from cause_amd import abi, gen, shard, stream
    import dataclasses

    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.nodes)
    layout = spec.layout()
    T, B, n = a.stream_docs, a.docs, spec.doc_size
    d0, d1 = rank * T // world, (rank + 1) * T // world
    nb = (d1 - d0 + B - 1) // B
    w = abi.Weaver(local)
    st_bad = [0]
    vis_total = [0]

    k32 = not a.k64

    def fill(i, views):
        b0 = d0 + i * B
        b1 = min(d1, b0 + B)
        off, *_ = gen.generate(spec, b0, b1, nthreads=16, out=views, k32=k32)
        return off

    def consume(o):
        st_bad[0] += int(np.count_nonzero(o.status))
        vis_total[0] += int(o.visible_count.sum(dtype=np.uint64))

    perm16 = k32 and n < 65536
    s = stream.BatchStreamer(w, dev, B * n, B, layout, depth=a.depth, k32=k32, perm16=perm16)
    s.run(min(a.warmup, nb), fill)          # warm-up batches (not timed)
    w.reset_kernel_stats()
    w.set_profiling(True)
    if world > 1:
        dist.barrier()
    with heartbeat(f"streaming {d1 - d0:,} documents in {nb} batches"):
        st = s.run(nb, fill, consume)
    if world > 1:
        dist.barrier()
    w.set_profiling(False)
    stats = w.kernel_stats()
    if st_bad[0]:
        raise SystemExit(f"rank {rank}: {st_bad[0]} documents out of domain")
    # the same pipeline with the inputs already in (pinned) host memory: each
    # slot keeps the batch generated into it first, and the batches cycle over
    # the slots (a weave never writes its inputs), so only PCIe and the weave run
    pre = None
    if not a.no_prestaged:
        filled = {}

        def fill_pre(i, views):
            j = i % a.depth
            if j not in filled:
                filled[j] = fill(j, views)
            return filled[j]

        s.run(a.depth, fill_pre)
        if world > 1:
            dist.barrier()
        st_pre = s.run(nb, fill_pre, lambda o: st_bad.__setitem__(
            0, st_bad[0] + int(np.count_nonzero(o.status))))
        if world > 1:
            dist.barrier()
        wall_pre = shard.reduce_max_time(st_pre.wall_s, dist, dev) if world > 1 else st_pre.wall_s
        pre = {"value": T * n / wall_pre,
               "unit": "nodes/s", "wall_s": wall_pre,
               "h2d_ms_per_batch": float(np.mean(st_pre.h2d_ms)),
               "weave_ms_per_batch": float(np.mean(st_pre.weave_ms)),
               "d2h_ms_per_batch": float(np.mean(st_pre.d2h_ms)),
               "note": f"inputs pre-staged in pinned host memory ({a.depth} distinct batches "
                       f"cycled over the slots), H2D + weave + D2H pipelined, no generation"}
        if st_bad[0]:
            raise SystemExit(f"rank {rank}: {st_bad[0]} documents out of domain")
    check = None
    if a.check:  # after timing: every streamed batch again, each compared with the oracle
        import oracle

        bad = [0, 0]

        def consume_check(o):
            b0 = d0 + o.index * B
            b1 = min(d1, b0 + B)
            off, idk, ck, kd = gen.generate(spec, b0, b1, nthreads=16)
            want, vis, wst = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_EFF,
                                                nthreads=16)
            got = o.weave_perm.astype(np.uint32)
            gvis = np.unpackbits(o.visible_bits.view(np.uint8), bitorder="little")[:len(got)]
            for dd in range(b1 - b0):
                lo, hi = int(off[dd]), int(off[dd + 1])
                ok = (o.status[dd] == wst[dd] and np.array_equal(got[lo:hi], want[lo:hi]) and
                      np.array_equal(gvis[lo:hi], vis[lo:hi]) and
                      int(o.visible_count[dd]) == int(vis[lo:hi].sum()))
                bad[0] += 0 if ok else 1
            bad[1] += b1 - b0

        with heartbeat("--check against the oracle"):
            s.run(nb, fill, consume_check)
        tot = shard.reduce_sum(bad, dist, dev) if world > 1 else bad
        check = {"documents_checked": tot[1], "mismatches": tot[0],
                 "against": "effective-tree preorder + visibility (oracle, C)"}
    t_dev = sum(st.weave_ms) / 1e3
    t_dev_max = shard.reduce_max_time(t_dev, dist, dev) if world > 1 else t_dev
    wall_max = shard.reduce_max_time(st.wall_s, dist, dev) if world > 1 else st.wall_s
    total = T * n
    name, (launches, ms, by) = max(stats.items(), key=lambda kv: kv[1][1])
    achieved_kernel = by / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    # SURVEY 8(d)'s bytes for the fused weave (as config 2): B_io per node of a
    # batch -- ids, causes, kinds in, weave_perm and the visible bit out
    b_io = b_io_bytes(4 if k32 else 8, 2 if perm16 else 4)
    whole = name == "weave"
    achieved = achieved_gbs(B * n * b_io if whole else by / max(launches, 1), launches, ms)
    # a config-3 batch has the config-2 batch's shape: the same kernels' counters
    traffic, tnote = pmc_traffic(name, "config2", B == 10_000 and a.nodes == 50_000)
    if rank == 0:
        cpu = None
        if not a.no_cpu:  # after the GPU region, on rank 0 at every N
            cpu = cpu_baseline(spec, a.cpu_seconds, max_docs=64)
        kw, pw = (4 if k32 else 8), (2 if perm16 else 4)
        pcie = total // world * (kw + kw + 1 + pw) + total // world // 8
        line = {
            "metric": "nodes woven/sec (whole node) + % of HBM roofline at 1/2/4/8 MI355X",
            "value": total / t_dev_max, "unit": "nodes/s", "n_gpus": world, "steps": nb,
            "warmup": min(a.warmup, nb), "ms_per_step": t_dev_max / nb * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (generated on the host per batch)",
            "config": {"workload": (f"config3: {T:,} CausalLists streamed from host memory in "
                                    f"{B:,}-document batches"),
                       "docs_total": T, "docs_per_batch": B, "nodes_per_doc": n,
                       "sites": spec.n_sites, "p_hide": spec.p_hide, "p_show": spec.p_show,
                       "p_conj": spec.p_conj, "key_bits": layout.key_bits,
                       "pipeline_depth": a.depth, "key_words": "u32 (cw_weave_lists_k32)" if k32
                       else "u64 (cw_weave_lists)", "weave_perm": "u16" if perm16 else "u32",
                       "parallelism": f"docs sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "frac_io": achieved / HBM_PEAK_GBS if whole else None,
                         "bytes_alg_per_node": b_io if whole else by / launches / (B * n),
                         "achieved_kernel_scratch": achieved_kernel,
                         "traffic": traffic, "traffic_note": tnote,
                         "launches_per_step": launches / nb,
                         "kernel_ms_per_step": ms / nb},
            "cpu_baseline": cpu,
            "end_to_end": {"value": total / wall_max, "unit": "nodes/s", "wall_s": wall_max,
                           "pcie_bytes_per_gpu": pcie,
                           "h2d_ms_per_batch": float(np.mean(st.h2d_ms)),
                           "weave_ms_per_batch": float(np.mean(st.weave_ms)),
                           "d2h_ms_per_batch": float(np.mean(st.d2h_ms)),
                           "host_fill_s_per_batch": st.fill_s / nb,
                           "note": "host generation (16 threads), H2D, weave and D2H "
                                   "pipelined over the slots; rank-0 figures"},
            "end_to_end_prestaged": pre,
            "visible_nodes": vis_total[0],
        }
        if cpu:
            line["speedup_vs_cpu_baseline"] = line["value"] / cpu["value"]
        if check:
            line["check"] = check
        print(json.dumps(line), flush=True)
    del s
    w.close()


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={world}: using {world} ranks",
              file=sys.stderr)
    # more ranks than GPUs (a rehearsal on a one-GPU box): ranks share devices
    # and the bookkeeping collectives go over gloo (RCCL needs a GPU per rank)
    ndev = torch.cuda.device_count()
    shared = world > max(ndev, 1)
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)  # before the process group: RCCL binds the current device
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo" if shared or not torch.cuda.is_available() else "nccl")

    if a.config == 5 and (world > 1 or a.dist):
        main_giant_dist(a, world, rank, local, dist, torch, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    if a.config == 3:
        main_stream(a, world, rank, local, dist, torch, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    if a.config == 4:
        main_maps(a, world, rank, local, dist, torch, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    from cause_amd import abi, gen, shard
    import dataclasses

    if a.config == 1:
        # one list; every rank weaves its own replica (the path does not shard)
        spec, D = gen.CONFIG1, 1
        d0, d1 = 0, 1
        workload = "config1: one CausalList of 100,000 inserts from 4 sites, full reweave"
    elif a.config == 5:
        # one giant list (config 5 scaled to one GPU: the 2e9-node list needs the
        # RCCL sample sort of DESIGN.md 8); every rank weaves its own replica
        spec, D = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.giant), 1
        d0, d1 = 0, 1
        workload = (f"config5 (scaled): one CausalList of {a.giant + 1:,} nodes, 8 sites, "
                    f"10% hides, full reweave on the giant-document path")
    else:
        spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=a.nodes)
        D = a.docs
        d0, d1 = shard.doc_range(rank, world, docs_per_rank=D)  # weak scaling, no data exchange
        workload = "config2: independent CausalLists, full reweave"
    layout = spec.layout()
    t0 = time.time()
    k32 = a.keys == 32
    tag = f"c{a.config}_n{spec.doc_size}_d{d0}-{d1}_k{a.keys}"
    cached = a.cache and all(os.path.exists(os.path.join(a.cache, f"{tag}_{x}.npy"))
                             for x in ("off", "id", "cause", "kind"))
    if cached:  # (PMC passes re-run the bench: generate a large input once a call)
        off, idk, ck, kd = (np.load(os.path.join(a.cache, f"{tag}_{x}.npy"))
                            for x in ("off", "id", "cause", "kind"))
    else:
        with heartbeat("generating the input"):
            off, idk, ck, kd = gen.generate(spec, d0, d1, nthreads=16, k32=k32)
        if a.cache:
            os.makedirs(a.cache, exist_ok=True)
            for x, arr in zip(("off", "id", "cause", "kind"), (off, idk, ck, kd)):
                np.save(os.path.join(a.cache, f"{tag}_{x}.npy"), arr)
    N = len(idk)
    t_gen = time.time() - t0
    kv = np.int32 if k32 else np.int64
    g_id = torch.from_numpy(idk.view(kv)).to(dev)
    g_ca = torch.from_numpy(ck.view(kv)).to(dev)
    g_kd = torch.from_numpy(kd).to(dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    bits = torch.empty((N + 31) // 32, dtype=torch.int32, device=dev)
    vcount = torch.empty(D, dtype=torch.int32, device=dev)
    max_ts = torch.empty(D, dtype=torch.int64, device=dev)
    status = torch.empty(D, dtype=torch.int32, device=dev)
    outs = {"weave_perm": perm.data_ptr(), "visible_bits": bits.data_ptr(),
            "visible_count": vcount.data_ptr(), "max_ts": max_ts.data_ptr(),
            "status": status.data_ptr()}
    torch.cuda.synchronize()

    w = abi.Weaver(local)
    w.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    w.set_async(True)

    call = w.weave_lists_k32_device if k32 else w.weave_lists_device

    def step():
        call(off, g_id.data_ptr(), g_ca.data_ptr(), g_kd.data_ptr(), layout, outs)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if int(status.max().item()) != 0:
        raise SystemExit(f"rank {rank}: documents out of domain: status max {status.max().item()}")

    # the dominant kernel: one step with events around every launch
    w.reset_kernel_stats()
    w.set_profiling(True)
    step()
    torch.cuda.synchronize()
    w.set_profiling(False)
    dom = max(w.kernel_stats().items(), key=lambda kv: kv[1][1])[0]
    # timed region: HIP events on the launch stream around the dominant
    # kernel's launches only (two events a launch: per-kernel events on every
    # launch cost a sub-millisecond one-list step a third of its time)
    w.reset_kernel_stats()
    w.set_profile_only(dom)
    w.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    w.set_profiling(False)
    w.set_profile_only(None)
    stats_dom = w.kernel_stats()
    # parity on the timed path: the last timed step's outputs of --check-docs
    # documents spread over the batch, copied out now and compared with the
    # oracle after every GPU measurement (outside the timed region)
    snap, snap_note = None, None
    if a.check_docs > 0 and not a.check:
        if a.config == 5 and N > (1 << 27):
            snap_note = (f"not checked in the bench: one {N:,}-node list is too large for the "
                         f"oracle in the bench's budget (tests/test_gpu_giant_full.py checks "
                         f"2,000,040,001 nodes position by position)")
        else:
            snap = snapshot_lists(off, sample_docs(D, a.check_docs), perm, bits, vcount, status)
    # the per-kernel breakdown (information): the same steps with events on
    # every launch
    w.reset_kernel_stats()
    w.set_profiling(True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt_allprof = time.perf_counter() - t1
    w.set_profiling(False)
    stats = w.kernel_stats()

    dt_max = shard.reduce_max_time(dt, dist, dev) if world > 1 else dt
    total_nodes = N * world * a.steps
    value = total_nodes / dt_max
    # the full reconstitute path (s/refresh-caches, shared.cljc:259-266: spin ->
    # refresh-ts -> weave-fn): the same steps with the yarns (yarn_perm, the id
    # order partitioned by site) asked for as well; `value` stays the weave's
    refresh = None
    if a.config in (2, 5) and not k32 and not a.no_refresh:
        yarn = torch.empty(N, dtype=torch.int32, device=dev)
        outs_y = dict(outs, yarn_perm=yarn.data_ptr())

        def step_y():
            call(off, g_id.data_ptr(), g_ca.data_ptr(), g_kd.data_ptr(), layout, outs_y)

        step_y()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step_y()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dty = time.perf_counter() - t0
        dty = shard.reduce_max_time(dty, dist, dev) if world > 1 else dty
        w.reset_kernel_stats()
        w.set_profiling(True)
        for _ in range(a.steps):
            step_y()
        torch.cuda.synchronize()
        w.set_profiling(False)
        ys = w.kernel_stats()
        yk = {k: v for k, v in ys.items() if k not in stats or k.startswith("yarn")}
        refresh = {"value": total_nodes / dty, "unit": "nodes/s", "ms_per_step": dty / a.steps * 1e3,
                   "note": "the weave step plus the yarns (yarn_perm: spin's id order partitioned "
                           "by site) and ::lamport-ts: s/refresh-caches in full",
                   "kernels_ms_per_step": {k: round(v[1] / a.steps, 4) for k, v in
                                           sorted(ys.items(), key=lambda kv: -kv[1][1])},
                   "yarn_kernels": {k: {"ms_per_step": round(v[1] / a.steps, 4),
                                        "alg_bytes_per_step": v[2] / a.steps,
                                        "achieved_gbs": round(v[2] / (v[1] / 1e3) / 1e9, 1)
                                        if v[1] > 0 else None} for k, v in yk.items()}}
        del yarn
    check = None
    if a.check:
        with heartbeat("--check against the oracle"):
            bad = check_lists(off, *_k64(idk, ck), kd, perm, bits, vcount, status)
        tot = shard.reduce_sum([bad, D], dist, dev) if world > 1 else [bad, D]
        check = {"documents_checked": tot[1], "mismatches": tot[0],
                 "against": "effective-tree preorder + visibility (oracle, C)",
                 "what": "every document of the batch, outputs of the last untimed step"}
    elif snap is not None:
        with heartbeat("sample check against the oracle"):
            nchk, bad = check_snapshot_lists(off, *_k64(idk, ck), kd, snap)
        tot = shard.reduce_sum([bad, nchk], dist, dev) if world > 1 else [bad, nchk]
        check = {"documents_checked": tot[1], "mismatches": tot[0],
                 "against": "effective-tree preorder + visibility (oracle, C)",
                 "what": (f"the last timed step's weave_perm, visible bits, visible_count and "
                          f"status of {a.check_docs} documents spread evenly over each rank's "
                          f"batch (fewer if the batch is smaller), copied out after timing")}
    elif snap_note:
        check = {"documents_checked": 0, "mismatches": None, "note": snap_note}

    # PCIe-inclusive rate (not the headline value): inputs from pinned host
    # buffers, the weave, weave_perm + visible bits back, serialised
    e2e = None
    if a.config == 2 and not a.no_h2d and world == 1:  # (N > 1: 8.5 GB pinned per rank)
        h_in = [torch.from_numpy(x).pin_memory() for x in
                (idk.view(np.int64), ck.view(np.int64), kd)]
        h_perm = torch.empty(N, dtype=torch.int32).pin_memory()
        h_bits = torch.empty((N + 31) // 32, dtype=torch.int32).pin_memory()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            for g, h in zip((g_id, g_ca, g_kd), h_in):
                g.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            step()
            torch.cuda.synchronize()
            h_perm.copy_(perm, non_blocking=True)
            h_bits.copy_(bits, non_blocking=True)
            torch.cuda.synchronize()
        dte = time.perf_counter() - t0
        dte = shard.reduce_max_time(dte, dist, dev) if world > 1 else dte
        e2e = {"value": total_nodes / dte, "unit": "nodes/s", "ms_per_step": dte / a.steps * 1e3,
               "bytes_per_step_pcie": N * (8 + 8 + 1 + 4) + (N + 31) // 32 * 4,
               "note": "inputs H2D from pinned host memory, weave, weave_perm and visible "
                       "bits D2H, serialised per step"}

    # dominant kernel = largest share of the measured kernel time, timed
    # inside the timed region
    name = dom
    launches, ms, by = stats_dom[dom]
    achieved_kernel = by / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    # SURVEY 8(d)'s headline algorithmic bytes: B_io per node = id + cause +
    # kind in, weave_perm + one visible bit out (21.125 B with u64 keys, 13.125
    # with u32).  The fused per-document kernel does the whole weave, so its
    # algorithmic bytes are B_io x the nodes of a launch; its own scratch
    # handoffs (achieved_kernel_scratch) are not algorithmic bytes.
    b_io = b_io_bytes(4 if k32 else 8, 4)
    whole = name == "weave"
    achieved = achieved_gbs(N * b_io, launches, ms) if whole else achieved_gbs(by / launches, launches, ms)
    kernel_ms_total = sum(v[1] for v in stats.values())
    # HBM bytes per launch of that kernel from the committed rocprofv3 PMC
    # passes (scripts/pmc_traffic.py; FETCH_SIZE doubled per MI355X_MICROARCH.md)
    # (config 5 has passes at its scaled default, 2^26 nodes, and at BASELINE's
    # full 2,000,000,001 nodes: workload "config5full")
    full5 = a.config == 5 and a.giant == 2_000_000_001
    traffic, tnote = pmc_traffic(name, "config5full" if full5 else f"config{a.config}",
                                 a.keys == 64 and (a.config == 1 or (a.config == 2 and a.docs == 10_000
                                                   and a.nodes == 50_000) or
                                                   (a.config == 5 and a.giant == 1 << 26) or full5))

    if rank == 0:
        cpu = None
        if not a.no_cpu:  # after the GPU region, on rank 0 at every N
            with heartbeat("cpu_baseline"):
                cpu = (cpu_baseline_prefix(*_k64(idk, ck), kd, 100_000) if a.config == 5 else
                       cpu_baseline(spec, a.cpu_seconds, max_docs=1 if a.config == 1 else 64))
        line = {
            "metric": "nodes woven/sec (whole node) + % of HBM roofline at 1/2/4/8 MI355X",
            "value": value, "unit": "nodes/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt_max / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": workload,
                       "docs_per_gpu": D, "nodes_per_doc": spec.doc_size,
                       "nodes_per_gpu": N, "sites": spec.n_sites, "p_hide": spec.p_hide,
                       "p_show": spec.p_show, "p_conj": spec.p_conj,
                       "key_bits": layout.key_bits,
                       "key_words": "u32 (cw_weave_lists_k32)" if k32 else "u64 (cw_weave_lists)",
                       "parallelism": (f"replicas x{world}" if a.config in (1, 5)
                                       else f"docs sharded x{world}")},
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "frac_io": achieved / HBM_PEAK_GBS if whole else None,
                         "bytes_alg_per_node": b_io if whole else by / launches / N,
                         "bytes_alg_note": ("B_io (SURVEY 8d): id + cause + kind in, weave_perm + "
                                            "visible bit out, per node of the launch" if whole else
                                            "the kernel's algorithmic bytes (DESIGN 5)"),
                         "achieved_kernel_scratch": achieved_kernel,
                         "frac_kernel_scratch": achieved_kernel / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_note": tnote,
                         "launches_per_step": launches / a.steps,
                         "kernel_ms_per_step": ms / a.steps},
            "frac_step_io": value * b_io / 1e9 / HBM_PEAK_GBS / world,
            "cpu_baseline": cpu,
            "kernels_ms_per_step": {k: round(v[1] / a.steps, 4) for k, v in
                                    sorted(stats.items(), key=lambda kv: -kv[1][1])},
            "kernel_gbs": {k: round(v[2] / (v[1] / 1e3) / 1e9, 1) for k, v in stats.items()
                           if v[1] > 0},
            "kernel_sum_ms_per_step": kernel_ms_total / a.steps,
            "ms_per_step_events_on_every_launch_rank0": dt_allprof / a.steps * 1e3,
            "end_to_end_pcie": e2e,
            "gen_s": t_gen,
            # device memory in use after the timed steps (inputs, outputs and the
            # library's scratch): the config-5 sizing
            "hbm_used_gib": round((lambda f, t: (t - f) / 2**30)(*torch.cuda.mem_get_info(dev)), 2),
        }
        if cpu:
            line["speedup_vs_cpu_baseline"] = value / cpu["value"]
        if check:
            line["check"] = check
        if refresh:
            line["refresh_caches"] = refresh
        if not a.no_cpu and a.config == 2:
            with heartbeat("cpu_baseline_parallel"):
                par = cpu_baseline_parallel(spec)
            line["cpu_baseline_parallel"] = par
            line["speedup_vs_cpu_parallel"] = value / par["value"]
        print(json.dumps(line), flush=True)
    w.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
