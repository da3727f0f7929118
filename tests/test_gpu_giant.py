"""The distributed giant-list weave on the GPU (cause_amd/giant.py, config 5).

1. Each building block behind the C ABI (cw_sort_keys, cw_partition_keys,
   cw_lookup_keys, cw_gather, cw_scatter32, cw_weave_ranked) against the CPU
   double tests/giant_cpu_ops.py on the same inputs, bit-exact.
2. weave_distributed with HipOps: one rank in this process, and two ranks as
   two worker processes sharing cuda:0 (gloo, host-staged exchange), against
   the oracle's weave of the whole list.
"""
import dataclasses
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
from cause_amd import abi, gen, giant
from tests.giant_cpu_ops import CpuOps

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ops():
    import torch

    with abi.Weaver(0) as w:
        yield giant.HipOps(w, "cuda:0")
        torch.cuda.synchronize()


def _t(a, dev="cuda:0"):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _i64(a):
    return np.ascontiguousarray(a, np.uint64).view(np.int64)


@pytest.mark.parametrize("n,bits", [(1, 5), (1000, 12), (5000, 40), (300_000, 33), (70_000, 63)])
def test_sort_keys(ops, n, bits):
    rng = np.random.default_rng(n)
    k = rng.integers(0, 1 << bits, n, dtype=np.uint64)  # duplicates: stability shows
    ko, io = ops.sort_keys(_t(_i64(k)), bits)
    rk, ri = CpuOps().sort_keys(__import__("torch").from_numpy(_i64(k)), bits)
    assert np.array_equal(ko.cpu().numpy(), rk.numpy())
    assert np.array_equal(io.cpu().numpy(), ri.numpy())


@pytest.mark.parametrize("m,ns", [(0, 3), (1, 0), (5000, 1), (100_000, 7), (200_000, 200)])
def test_partition(ops, m, ns):
    import torch

    rng = np.random.default_rng(m + ns)
    k = rng.integers(0, 1 << 40, m, dtype=np.uint64)
    k[: m // 10] = np.uint64(2**64 - 1)  # nil causes go to the last bucket
    sp = np.sort(rng.integers(0, 1 << 40, ns, dtype=np.uint64))
    perm, counts = ops.partition(_t(_i64(k)), torch.from_numpy(_i64(sp)))
    rp, rc = CpuOps().partition(torch.from_numpy(_i64(k)), torch.from_numpy(_i64(sp)))
    assert counts == rc
    assert np.array_equal(perm.cpu().numpy(), rp.numpy())


@pytest.mark.parametrize("n,m,base", [(0, 10, 0), (1, 5, 7), (10_000, 50_000, 0),
                                      (400_000, 100_000, 123_456)])
def test_lookup(ops, n, m, base):
    import torch

    rng = np.random.default_rng(n + m)
    s = np.unique(rng.integers(0, 1 << 36, n, dtype=np.uint64))
    q = rng.integers(0, 1 << 36, m, dtype=np.uint64)
    if len(s):
        hit = rng.integers(0, len(s), m // 2)
        q[: m // 2] = s[hit]
    got, gdup = ops.lookup(_t(_i64(s)), _t(_i64(q)), base)
    ref, rdup = CpuOps().lookup(torch.from_numpy(_i64(s)), torch.from_numpy(_i64(q)), base)
    assert np.array_equal(got.cpu().numpy(), ref.numpy())
    assert gdup == rdup == 0


@pytest.mark.parametrize("m", [0, 1000])
def test_lookup_reports_repeated_ids(ops, m):
    """An id held by two ranks meets itself at its owner after the sample sort:
    the owner's sorted run repeats it and cw_lookup_keys flags CW_STATUS_DUP
    (even with no queries to answer)."""
    import torch

    s = np.sort(np.random.default_rng(3).integers(0, 1 << 30, 5000, dtype=np.uint64))
    s[2500] = s[2499]
    q = s[:m].copy()
    got, dup = ops.lookup(_t(_i64(s)), _t(_i64(q)), 0)
    ref, rdup = CpuOps().lookup(torch.from_numpy(_i64(s)), torch.from_numpy(_i64(q)), 0)
    assert dup == rdup == abi.STATUS_DUP
    assert np.array_equal(got.cpu().numpy(), ref.numpy())


def test_gather_scatter(ops):
    rng = np.random.default_rng(5)
    n = 100_003
    idx = rng.permutation(n).astype(np.int32)
    for dt in (np.uint8, np.int32, np.int64):
        src = rng.integers(0, 100, n).astype(dt)
        got = ops.gather(_t(src), _t(idx)).cpu().numpy()
        assert np.array_equal(got, src[idx])
    src = rng.integers(0, 1 << 30, n).astype(np.int32)
    out = ops.scatter32(_t(src), _t(idx)).cpu().numpy()
    ref = np.empty_like(src)
    ref[idx] = src
    assert np.array_equal(out, ref)


def ranked_case(n, seed):
    """One list as (par, kind) in rank order, from the config-2 generator."""
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=n, seed=seed)
    off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=1)
    o = np.argsort(idk, kind="stable")
    rank = np.empty(len(o), np.int64)
    rank[o] = np.arange(len(o))
    ck_o = ck[o]
    pos = np.searchsorted(idk[o], ck_o)
    par = np.where(ck_o == np.uint64(2**64 - 1), 0xFFFFFFFF, pos).astype(np.uint32)
    return par.view(np.int32), kd[o].copy(), o.astype(np.int32)


@pytest.mark.parametrize("n,seed", [(1, 1), (50, 2), (20_000, 3), (600_000, 4)])
def test_weave_ranked(ops, n, seed):
    import torch

    par, kd, val = ranked_case(n, seed)
    got = ops.weave_ranked(_t(par), _t(kd), _t(val))
    ref = CpuOps().weave_ranked(torch.from_numpy(par), torch.from_numpy(kd), torch.from_numpy(val))
    assert int(got["status"][0]) == 0 == int(ref["status"][0])
    assert np.array_equal(got["weave_perm"].cpu().numpy(), ref["weave_perm"].numpy())
    assert int(got["visible_count"][0]) == int(ref["visible_count"][0])
    assert np.array_equal(got["visible_bits"].cpu().numpy(), ref["visible_bits"].numpy())


def test_weave_ranked_flags_orphans_and_roots(ops):
    par, kd, val = ranked_case(2000, 7)
    p = par.copy()
    p[100] = -1  # CW_NOT_FOUND
    got = ops.weave_ranked(_t(p), _t(kd), _t(val))
    assert int(got["status"][0]) & abi.STATUS_ORPHAN
    k = kd.copy()
    k[0] &= ~np.uint8(4)
    got = ops.weave_ranked(_t(par), _t(k), _t(val))
    assert int(got["status"][0]) & abi.STATUS_ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_inputs(n, seed, lo, hi):
    """The run [lo, hi) of a ranked list: (par, kind) of those ranks."""
    par, kd, val = ranked_case(n, seed)
    return par[lo:hi].copy(), kd[lo:hi].copy(), par, kd, val


def _same(a, b):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    b = b.cpu().numpy() if hasattr(b, "cpu") else np.asarray(b)
    if a.shape != b.shape:
        print("shapes", a.shape, b.shape)
        return False
    bad = np.flatnonzero((a != b).reshape(len(a), -1).any(axis=1)) if a.size else []
    if len(bad):
        print("differ at", bad[:5], a[bad[:5]], b[bad[:5]], "of", len(bad))
    return len(bad) == 0


@pytest.mark.parametrize("n,seed,lo,hi", [(30_000, 41, 0, 30_000), (30_000, 42, 9_000, 21_000),
                                          (5_000, 43, 4_000, 5_000)])
def test_dist_ops_match_the_double(ops, n, seed, lo, hi):
    """Every building block of the distributed tree (dist.hip) against its numpy
    restatement (tests/giant_cpu_ops.py) on one rank's run of a list."""
    import torch

    cpu = CpuOps()
    par, kd, fpar, fkd, _ = _dist_inputs(n, seed, lo, hi)
    T = torch.from_numpy
    assert ops.dist_check(_t(par), _t(kd), lo) == cpu.dist_check(T(par), T(kd), lo) == 0
    eff = ops.dist_eff(_t(par), _t(kd), lo)
    ceff = cpu.dist_eff(T(par), T(kd), lo)
    assert _same(eff, ceff)
    rng = np.random.default_rng(seed)
    q = rng.integers(lo, hi, 5000).astype(np.int64)
    assert _same(ops.dist_climb(_t(par), _t(kd), lo, _t(q)), cpu.dist_climb(T(par), T(kd), lo, T(q)))
    (k1, c1), (k2, c2) = ops.dist_pending(eff), cpu.dist_pending(ceff)
    assert _same(k1, k2) and c1 == c2
    # effective parents of the whole list from the full run: the group keys,
    # runs, records and links of a one-rank tree
    feff = cpu.dist_eff(T(fpar), T(fkd), 0)
    gk = cpu.dist_gkey(feff, T(fkd))
    assert _same(ops.dist_gkey(_t(feff.numpy()), _t(fkd)), gk)
    sk, si = cpu.sort_keys32(gk, 32)
    nsc, okey, rec = ops.dist_runs(_t(sk.numpy()), _t(si.numpy()), 0, _t(fkd))
    cnsc, cokey, crec = cpu.dist_runs(sk, si, 0, T(fkd))
    assert _same(nsc, cnsc) and _same(okey, cokey)
    heads = torch.from_numpy(cokey.numpy() != -1)
    assert _same(rec.cpu()[heads], crec[heads])
    rs = crec[heads].contiguous()
    rkey = ops.dist_rkey(_t(rs.numpy()))
    assert _same(rkey, cpu.dist_rkey(rs))
    rk, ri = cpu.sort_keys32(rkey.cpu(), 32)
    n = len(fpar)   # (the list has a root besides its n generated nodes)
    fs, fn = ops.zeros32(n), ops.zeros32(n)
    cfs, cfn = cpu.zeros32(n), cpu.zeros32(n)
    reply = ops.dist_link(_t(rk.numpy()), _t(ri.numpy()), _t(rs.numpy()), 0, n, fs, fn)
    creply = cpu.dist_link(rk, ri, rs, 0, n, cfs, cfn)
    assert _same(reply, creply) and _same(fs, cfs) and _same(fn, cfn)
    ops.dist_put(_t(rs.numpy()), reply, 0, nsc)
    cpu.dist_put(rs, creply, 0, cnsc)
    assert _same(nsc, cnsc)
    thr = ops.dist_thr(nsc, 0)
    cthr = cpu.dist_thr(cnsc, 0)
    assert _same(thr, cthr)
    # a run that starts mid-list: tiles counted from the run's start
    assert _same(ops.dist_thr(_t(cnsc.numpy()[lo:hi]), lo), cpu.dist_thr(cnsc[lo:hi], lo))
    succ = ops.dist_succ(_t(fkd), fs, fn, 0)
    csucc = cpu.dist_succ(T(fkd), cfs, cfn, 0)
    assert _same(succ, csucc)


@pytest.mark.parametrize("n,seed", [(1, 1), (50, 2), (20_000, 3), (600_000, 4)])
def test_weave_linked_equals_weave_ranked(ops, n, seed):
    """cw_weave_linked on the successors of the one-rank distributed tree gives
    cw_weave_ranked's weave of the same list."""
    import torch

    cpu = CpuOps()
    par, kd, val = ranked_case(n, seed)
    n = len(par)
    T = torch.from_numpy
    eff = ops.dist_eff(_t(par), _t(kd), 0)
    sk, si = ops.sort_keys32(ops.dist_gkey(eff, _t(kd)), 32)
    nsc, okey, rec = ops.dist_runs(sk, si, 0, _t(kd))
    heads = okey.cpu().numpy() != -1
    rs = _t(rec.cpu().numpy()[heads])
    rk, ri = ops.sort_keys32(ops.dist_rkey(rs), 32)
    fs, fn = ops.zeros32(n), ops.zeros32(n)
    reply = ops.dist_link(rk, ri, rs, 0, n, fs, fn)
    ops.dist_put(rs, reply, 0, nsc)
    succ, thr = ops.dist_succ(_t(kd), fs, fn, 0), ops.dist_thr(nsc, 0)
    got = ops.weave_linked(succ, thr, _t(val))
    want = ops.weave_ranked(_t(par), _t(kd), _t(val))
    ref = cpu.weave_linked(succ.cpu(), thr.cpu(), T(val))
    assert int(got["status"][0]) == 0 == int(want["status"][0])
    for k in ("weave_perm", "visible_count"):
        assert _same(got[k], want[k]) and _same(got[k], ref[k]), k
    nb = (n + 31) // 32
    assert _same(got["visible_bits"][:nb], want["visible_bits"][:nb])


def _one_rank_tree(ops, par, kd):
    """(succ, thr) of the one-rank distributed tree on the GPU."""
    n = len(par)
    eff = ops.dist_eff(_t(par), _t(kd), 0)
    sk, si = ops.sort_keys32(ops.dist_gkey(eff, _t(kd)), 32)
    nsc, okey, rec = ops.dist_runs(sk, si, 0, _t(kd))
    heads = okey.cpu().numpy() != -1
    rs = _t(rec.cpu().numpy()[heads])
    rk, ri = ops.sort_keys32(ops.dist_rkey(rs), 32)
    fs, fn = ops.zeros32(n), ops.zeros32(n)
    reply = ops.dist_link(rk, ri, rs, 0, n, fs, fn)
    ops.dist_put(rs, reply, 0, nsc)
    return ops.dist_succ(_t(kd), fs, fn, 0), ops.dist_thr(nsc, 0)


def _rows_sorted(t):
    a = t.cpu().numpy().view(np.uint32)
    return a[np.lexsort(a.T[::-1])] if len(a) else a


@pytest.mark.parametrize("n,seed,k,lo,hi", [(20_000, 3, 16, 0, None), (20_000, 5, 4, 7_000, 15_000),
                                            (300_000, 4, 16, 100_000, 250_000),
                                            (50, 2, 1, 0, None), (5_000, 6, 5000, 1_000, 4_000)])
def test_ruling_set_ops_match_the_double(ops, n, seed, k, lo, hi):
    """The ruling-set kernels (dist.hip k_rs_*) against their numpy restatement
    (tests/giant_cpu_ops.py) on a whole list and on one rank's run of it: node
    words, ruler list, one walk round (every node's {ruler, offset}, the links
    and the messages of walkers leaving the run), the ruler ranking, positions
    and the emit -- which must be cw_weave_linked's weave."""
    import torch

    cpu = CpuOps()
    T = torch.from_numpy
    par, kd, val = ranked_case(n, seed)
    N = len(par)
    hi = N if hi is None else hi
    succ, thr = _one_rank_tree(ops, par, kd)
    cs, ct = succ.cpu(), thr.cpu()
    seed32 = giant.RULER_SEED
    # one run [lo, hi) of the list (base lo); the rest of the list is "remote"
    word, rlist, nr = ops.rs_rulers(_t(cs.numpy()[lo:hi]), _t(ct.numpy()[lo:hi]), lo, k, seed32)
    cw, crl, cnr = cpu.rs_rulers(cs[lo:hi], ct[lo:hi], lo, k, seed32)
    assert nr == cnr and _same(word, cw) and _same(rlist.cpu()[:nr], crl[:nr])
    m = hi - lo
    rb = 0 if (lo == 0 and hi == N) else 7   # ruler indices of a later rank start higher
    own, links = ops.zeros32(2 * m), ops.zeros32(4 * max(nr, 1)).view(-1, 4)
    nl, st = ops.zeros32(1), ops.zeros32(1)
    out, key = ops.rs_walk(None, nr, rlist, rb, word, _t(ct.numpy()[lo:hi]), lo, own, links, nl, st)
    cown, clinks = cpu.zeros32(2 * m), cpu.zeros32(4 * max(cnr, 1)).view(-1, 4)
    cnl, cst = cpu.zeros32(1), cpu.zeros32(1)
    cout, ckey = cpu.rs_walk(None, cnr, crl, rb, cw, ct[lo:hi], lo, cown, clinks, cnl, cst)
    assert int(st[0]) == 0 == int(cst[0]) and int(nl[0]) == int(cnl[0])
    assert _same(own, cown) and _same(key, ckey)
    moved = ckey.numpy() != -1
    assert _same(out.cpu()[torch.from_numpy(moved)], cout[torch.from_numpy(moved)])
    assert np.array_equal(_rows_sorted(links[:int(nl[0])]), _rows_sorted(clinks[:int(cnl[0])]))
    if lo or hi != N:
        return
    # the whole list: one round ranks it
    assert not moved.any() and int(nl[0]) == nr
    pb = ops.rs_top(links[:nr], N, st)
    cpb = cpu.rs_top(clinks[:nr], N, cst)
    assert int(st[0]) == 0 == int(cst[0]) and _same(pb, cpb)
    rec, pk = ops.rs_pos(own, pb, succ, _t(val), keys=True)
    crec, cpk = cpu.rs_pos(cown, cpb, cs, T(val), keys=True)
    assert _same(rec, crec) and _same(pk, cpk)
    wp, bits, cnt = ops.rs_emit(rec, 0, N, st)
    want = ops.weave_linked(succ, thr, _t(val))
    assert int(st[0]) == 0
    assert _same(wp, want["weave_perm"]) and int(cnt[0]) == int(want["visible_count"][0])
    nb = (N + 31) // 32
    assert _same(bits[:nb], want["visible_bits"][:nb])


@pytest.mark.parametrize("m", [1, 2, 1000, (1 << 21) + 5, 3_000_000])
def test_ruling_set_top_level(ops, m):
    """cw_dist_rs_top on m ruler links in random list order (ruler 0 first),
    directly by pointer jumping (m <= 2^21) or in two levels (sub-rulers walk
    the ruler list): every ruler's position = the lengths before it."""
    import torch

    rng = np.random.default_rng(m)
    order = np.concatenate([[0], rng.permutation(np.arange(1, m))]).astype(np.uint32)
    ln = rng.integers(1, 40, m).astype(np.uint32)
    nxt = np.full(m, 0xFFFFFFFF, np.uint32)
    nxt[order[:-1]] = order[1:]
    links = np.stack([np.arange(m, dtype=np.uint32), nxt, ln, np.zeros(m, np.uint32)], 1)
    links = links[rng.permutation(m)]          # records arrive in any order
    want = np.zeros(m, np.uint64)
    want[order] = np.concatenate([[0], np.cumsum(ln[order].astype(np.uint64))[:-1]])
    total = int(ln.sum())
    st = ops.zeros32(1)
    pos = ops.rs_top(_t(np.ascontiguousarray(links)), total, st)
    assert int(st[0]) == 0
    assert np.array_equal(pos.cpu().numpy().view(np.uint32), want.astype(np.uint32))
    # a broken list (one link lost) is flagged, not ranked silently
    if m > 2:
        bad = links.copy()
        bad[bad[:, 0] == order[m // 2], 1] = 0xFFFFFFFF
        st = ops.zeros32(1)
        ops.rs_top(_t(np.ascontiguousarray(bad)), total, st)
        assert int(st[0]) & 32


@pytest.mark.parametrize("tree,ranking,out", [("root", "auto", "root"), ("dist", "root", "root"),
                                              ("dist", "ruling", "root"),
                                              ("dist", "ruling", "sharded")])
def test_distributed_one_rank_in_process(ops, tree, ranking, out):
    import torch
    import torch.distributed as dist

    from tests.test_giant_dist import make_list

    spec, idk, ck, kd = make_list(100_000, 21)
    rng = np.random.default_rng(0)
    sh = rng.permutation(len(idk))
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    g = dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        lay = spec.layout()
        res = giant.weave_distributed(ops, _t(_i64(idk[sh])), _t(_i64(ck[sh])), _t(kd[sh]),
                                      lay.key_bits, ts_shift=lay.ts_shift, tree=tree,
                                      ranking=ranking, out=out)
    finally:
        dist.destroy_process_group()
    perm, vis, st = oracle.batch_lists(np.array([0, len(idk)], np.uint64), idk, ck, kd,
                                       method=oracle.METHOD_EFF)
    assert res.status == 0
    assert np.array_equal(sh[res.weave_perm.cpu().numpy()], perm)
    assert res.visible_count == int(vis.sum())


@pytest.mark.parametrize("ranking,out", [("auto", "root"), ("root", "root"), ("ruling", "sharded")])
def test_distributed_two_ranks_share_the_gpu(tmp_path, ranking, out):
    """Two worker processes on cuda:0 (gloo: the exchange is staged on the host;
    with the nccl backend on distinct GPUs it runs over RCCL).  ranking auto =
    the ruling set at W = 2; "root" = the successors gathered on rank 0;
    out="sharded": each rank holds its 1/W of the weave positions."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "giant_worker.py"),
                                       str(tmp_path), ranking, out], env=e, cwd=ROOT))
    for p in procs:
        assert p.wait(timeout=300) == 0
    res = json.load(open(tmp_path / "rank0.json"))
    assert res["ok"], res
