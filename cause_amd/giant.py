"""One CausalList spread over several GPUs (BASELINE config 5: a single list of
2*10^9 nodes on 8 MI355X).

The reference weaves a list by `(sort ::nodes)` and a fold (list.cljc:26-28);
its nodes live in one hash map.  Here each rank (one process per GPU) holds an
arbitrary share of the node bag and the weave runs as

  1. local sort of the ids (cw_sort_keys);
  2. sample sort: weighted regular samples -> all_gather -> W-1 splitters;
     ids, causes, kinds and origins go to their owner rank (all_to_all, the
     only data exchange of the weave: RCCL over xGMI with the nccl backend);
  3. the owner sorts what it received: rank r owns a contiguous run of the
     global id order, so a node's global rank = owner base + local index;
  4. cause join (shared.cljc:175-178): cause ids travel to the rank owning
     them (cw_partition_keys + all_to_all), are looked up there
     (cw_lookup_keys) and the global ranks travel back (all_to_all);
  5. the tree rank by rank (_tree_distributed: all-to-all rounds between the
     dist.hip kernels) and the list ranking where the list lies
     (_rank_ruling: a ruling set whose walkers hop ranks as messages); the
     weave lands on one rank or spread by weave position.  Lists outside the
     fast path's domain (and tree="root") instead gather the rank-ordered
     (parent rank, kind, origin) arrays -- 9 bytes a node -- on one rank, which
     weaves the whole list there (cw_weave_ranked, with its exact path).

Every step that touches node data is a HIP kernel of libcauseweave behind the
C ABI; torch provides device memory, the collectives and tiny host-side
arithmetic on W-sized arrays (sample weights, splitters).  `ops` is the
kernel interface: HipOps in production; tests may pass a CPU double to check
the exchange logic with gloo on CPU.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

NOT_FOUND = 0xFFFFFFFF
STATUS_INTERNAL = 1 << 5   # CW_STATUS_INTERNAL
RULER_K = 16               # one ruler per ~16 nodes (DESIGN.md §6 study)
RULER_SEED = 0x2545F491


def _on_stream(f):
    """Run a HipOps method on the ops' stream (ordered after the caller's)."""
    def g(self, *a, **k):
        with self.stream_context():
            return f(self, *a, **k)
    g.__name__ = f.__name__
    return g


class HipOps:
    """The kernels of the distributed weave on one GPU (libcauseweave).

    The library and torch share one stream (a torch stream handed to the
    context; torch's default stream has no handle to hand over), so kernels,
    torch's allocations and the collectives are ordered without host syncs."""

    def __init__(self, weaver, device):
        self.w = weaver
        self.dev = torch.device(device)
        self.stream = torch.cuda.Stream(self.dev)
        weaver.set_stream(self.stream.cuda_stream)
        weaver.set_async(True)

    @contextlib.contextmanager
    def stream_context(self):
        cur = torch.cuda.current_stream(self.dev)
        if cur == self.stream:
            yield
            return
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            yield
        cur.wait_stream(self.stream)

    def _e(self, n, dtype):
        return torch.empty(n, dtype=dtype, device=self.dev)

    @_on_stream
    def sort_keys(self, keys, key_bits):
        n = keys.numel()
        ko, io = self._e(n, torch.int64), self._e(n, torch.int32)
        if n:
            self.w.sort_keys_device(keys.data_ptr(), n, key_bits, ko.data_ptr(), io.data_ptr())
        return ko, io

    @_on_stream
    def sort_keys32(self, keys, key_bits):
        n = keys.numel()
        ko, io = self._e(n, torch.int32), self._e(n, torch.int32)
        if n:
            self.w.sort_keys32_device(keys.data_ptr(), n, key_bits, ko.data_ptr(), io.data_ptr())
        return ko, io

    @_on_stream
    def partition(self, keys, splitters):
        m = keys.numel()
        perm = self._e(m, torch.int32)
        sp = splitters.to(self.dev)
        counts = self.w.partition_keys_device(keys.data_ptr() if m else 0, m,
                                              sp.data_ptr() if sp.numel() else 0, sp.numel(),
                                              perm.data_ptr() if m else 0)
        return perm, [int(x) for x in counts]

    @_on_stream
    def partition_dev(self, keys, splitters):
        """partition with the bucket sizes left on the device (int64 tensor of
        len(splitters) + 1): no host readback."""
        m = keys.numel()
        perm = self._e(m, torch.int32)
        sp = splitters.to(self.dev)
        counts = torch.empty(sp.numel() + 1, dtype=torch.int64, device=self.dev)
        self.w.partition_keys_dev(keys.data_ptr() if m else 0, m,
                                  sp.data_ptr() if sp.numel() else 0, sp.numel(),
                                  perm.data_ptr() if m else 0, counts.data_ptr())
        return perm, counts

    @_on_stream
    def lookup(self, sorted_keys, queries, base):
        """(global rank of each query or NOT_FOUND, CW_STATUS_DUP if the owner's
        sorted ids repeat one)."""
        m = queries.numel()
        out = self._e(m, torch.int32)
        st = torch.zeros(1, dtype=torch.int32, device=self.dev)
        if m or sorted_keys.numel():
            self.w.lookup_keys_device(sorted_keys.data_ptr() if sorted_keys.numel() else 0,
                                      sorted_keys.numel(), queries.data_ptr() if m else 0, m,
                                      base, out.data_ptr() if m else 0, st.data_ptr())
        return out, int(st.item())

    @_on_stream
    def gather(self, src, idx):
        m = idx.numel()
        out = self._e(m, src.dtype)
        if m:
            self.w.gather_device(src.data_ptr(), idx.data_ptr(), m, src.element_size(),
                                 out.data_ptr())
        return out

    @_on_stream
    def scatter32(self, src, idx):
        m = idx.numel()
        out = self._e(m, torch.int32)
        if m:
            self.w.scatter32_device(src.data_ptr(), idx.data_ptr(), m, out.data_ptr())
        return out

    @_on_stream
    def weave_ranked(self, par, kind, val):
        n = par.numel()
        o = {"weave_perm": self._e(n, torch.int32),
             "visible_bits": self._e((n + 31) // 32, torch.int32),
             "visible_count": self._e(1, torch.int32), "status": self._e(1, torch.int32)}
        self.w.weave_ranked_device(n, par.data_ptr(), kind.data_ptr(), val.data_ptr(),
                                   {k: t.data_ptr() for k, t in o.items()})
        return o

    # --- the distributed tree (dist.hip) ----------------------------------------
    @staticmethod
    def _p(t):
        return t.data_ptr() if t is not None and t.numel() else 0

    @_on_stream
    def dist_check(self, par, kind, base):
        st = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.w.dist("check", par.numel(), base, self._p(par), self._p(kind), st.data_ptr())
        return int(st.item())

    @_on_stream
    def dist_eff(self, par, kind, base):
        eff = self._e(par.numel(), torch.int32)
        self.w.dist("eff", par.numel(), base, self._p(par), self._p(kind), self._p(eff))
        return eff

    @_on_stream
    def dist_climb(self, par, kind, base, q):
        out = self._e(q.numel(), torch.int32)
        self.w.dist("climb", par.numel(), base, self._p(par), self._p(kind), self._p(q), q.numel(),
                    self._p(out))
        return out

    @_on_stream
    def dist_pending(self, w):
        """(partition keys of the eff words waiting on another rank, how many)."""
        keys = self._e(w.numel(), torch.int64)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.w.dist("pending", self._p(w), w.numel(), self._p(keys), cnt.data_ptr())
        return keys, int(cnt.item())

    @_on_stream
    def dist_gkey(self, eff, kind):
        key = self._e(eff.numel(), torch.int32)
        self.w.dist("gkey", self._p(eff), self._p(kind), eff.numel(), self._p(key))
        return key

    @_on_stream
    def dist_runs(self, skey, sidx, base, kind):
        n = skey.numel()
        nsc, okey = self._e(n, torch.int32), self._e(n, torch.int64)
        rec = self._e(n * 4, torch.int32)
        self.w.dist("runs", self._p(skey), self._p(sidx), n, base, self._p(kind), self._p(nsc),
                    self._p(okey), self._p(rec))
        return nsc, okey, rec.view(n, 4)

    @_on_stream
    def dist_rkey(self, rec):
        key = self._e(rec.shape[0], torch.int32)
        self.w.dist("rkey", self._p(rec), rec.shape[0], self._p(key))
        return key

    @_on_stream
    def dist_link(self, skey, sidx, rec, base, n, fcS, fcN):
        reply = self._e(rec.shape[0], torch.int32)
        self.w.dist("link", self._p(skey), self._p(sidx), rec.shape[0], self._p(rec), base, n,
                    self._p(fcS), self._p(fcN), self._p(reply))
        return reply

    @_on_stream
    def dist_put(self, rec, reply, base, nsc):
        self.w.dist("put", self._p(rec), self._p(reply), rec.shape[0], base, nsc.numel(), self._p(nsc))

    @_on_stream
    def dist_thr(self, nsc, base):
        thr = self._e(nsc.numel(), torch.int32)
        self.w.dist("thr", self._p(nsc), nsc.numel(), base, self._p(thr))
        return thr

    @_on_stream
    def dist_succ(self, kind, fcS, fcN, base):
        out = self._e(kind.numel(), torch.int32)
        self.w.dist("succ", self._p(kind), self._p(fcS), self._p(fcN), kind.numel(), base,
                    self._p(out))
        return out

    # --- the ruling-set list ranking (dist.hip) ------------------
    @_on_stream
    def rs_rulers(self, succ, thr, base, k, seed):
        """(node words int32 [n, 2], ruler list int32 [n], number of rulers)."""
        n = succ.numel()
        word, rlist = self._e(2 * n, torch.int32).view(n, 2), self._e(n, torch.int32)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.w.dist("rs_rulers", self._p(succ), self._p(thr), n, base, k, seed, self._p(word),
                    self._p(rlist), cnt.data_ptr())
        return word, rlist, int(cnt.item())

    @_on_stream
    def rs_walk(self, walkers, m, rlist, rbase, word, thr, base, own, links, nlinks, status):
        """One exchange round: (messages int32 [m, 4], their partition keys)."""
        out, key = self._e(m * 4, torch.int32).view(m, 4), self._e(m, torch.int64)
        self.w.dist("rs_walk", self._p(walkers), m, self._p(rlist), rbase, self._p(word),
                    self._p(thr), word.shape[0], base, self._p(own), self._p(links),
                    nlinks.data_ptr(), self._p(out), self._p(key), status.data_ptr())
        return out, key

    @_on_stream
    def rs_top(self, links, total, status):
        """Weave position of every ruler (int32 [m]) from all m links."""
        m = links.shape[0]
        pos = self._e(m, torch.int32)
        self.w.dist("rs_top", self._p(links), m, total, self._p(pos), status.data_ptr())
        return pos

    @_on_stream
    def rs_pos(self, own, pos_base, succ, val, keys=False):
        n = succ.numel()
        rec = self._e(2 * n, torch.int32).view(n, 2)
        key = self._e(n, torch.int64) if keys else None
        self.w.dist("rs_pos", self._p(own), self._p(pos_base), self._p(succ), self._p(val), n,
                    self._p(rec), self._p(key))
        return rec, key

    @_on_stream
    def rs_emit(self, rec, p0, length, status):
        """(weave_perm [length], visible_bits, visible_count [1]) of positions
        [p0, p0 + length) from the emit records."""
        perm = self._e(length, torch.int32)
        bits = self._e((length + 31) // 32, torch.int32)
        cnt = self._e(1, torch.int32)
        self.w.dist("rs_emit", self._p(rec), rec.shape[0], p0, length, self._p(perm),
                    self._p(bits), cnt.data_ptr(), status.data_ptr())
        return perm, bits, cnt

    @_on_stream
    def gather_rows(self, rec, idx):
        """rec[idx] for 16-byte rows (int32 [n, 4])."""
        m = idx.numel()
        out = self._e(m * 4, torch.int32).view(m, 4)
        if m:
            self.w.gather_device(rec.data_ptr(), idx.data_ptr(), m, 16, out.data_ptr())
        return out

    @_on_stream
    def scatter_into(self, dst, src, idx):
        """dst[idx[i]] = src[i] (4-byte elements, in place)."""
        if idx.numel():
            self.w.scatter32_device(src.data_ptr(), idx.data_ptr(), idx.numel(), dst.data_ptr())

    @_on_stream
    def zeros32(self, n):
        return torch.zeros(n, dtype=torch.int32, device=self.dev)

    @_on_stream
    def weave_linked(self, succ, thr, val):
        n = succ.numel()
        o = {"weave_perm": self._e(n, torch.int32),
             "visible_bits": self._e((n + 31) // 32, torch.int32),
             "visible_count": self._e(1, torch.int32), "status": self._e(1, torch.int32)}
        self.w.weave_linked_device(n, succ.data_ptr(), thr.data_ptr(), val.data_ptr(),
                                   {k: t.data_ptr() for k, t in o.items()})
        return o

    def sync(self):
        torch.cuda.synchronize(self.dev)


@dataclass
class GiantResult:
    """On the gathering rank: the weave of the whole list.  weave_perm[g] =
    global input index (rank offset + local index) of the node at weave
    position g; elsewhere None."""
    weave_perm: torch.Tensor | None
    visible_bits: torch.Tensor | None
    visible_count: int | None
    status: int | None
    n_total: int
    n_owned: int        # ids this rank owned after the sample sort
    max_ts: int
    pos_base: int = 0   # out="sharded": weave position of this rank's weave_perm[0]
    ranking: dict | None = None   # ruling set: rulers, exchange rounds, messages sent


def _a2a(t, send, recv, group):
    """all_to_all_single with split sizes; gloo works on host tensors."""
    if dist.get_world_size(group) == 1:
        return t
    out = torch.empty(sum(recv), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        o = out.cpu()
        dist.all_to_all_single(o, t.cpu(), recv, send, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, t, recv, send, group=group)
    return out


def _exchange_counts(send, group, device):
    W = len(send)
    if W == 1:
        return list(send)
    dev = "cpu" if dist.get_backend(group) == "gloo" else device
    s = torch.tensor(send, dtype=torch.int64, device=dev)
    r = torch.empty(W, dtype=torch.int64, device=dev)
    dist.all_to_all_single(r, s, group=group)
    return [int(x) for x in r.cpu()]


def _all_gather_ints(vals, group, device):
    dev = "cpu" if dist.get_backend(group) == "gloo" else device
    W = dist.get_world_size(group)
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    out = [torch.empty_like(t) for _ in range(W)]
    dist.all_gather(out, t, group=group)
    return [[int(x) for x in o.cpu()] for o in out]


def _gather_count_rows(counts, W, group):
    """Every rank's first W bucket sizes (a device or host int64 tensor) as a
    W x W host matrix: one all_gather and ONE readback -- both the exchange
    sizes of a ruling-set round and its termination test (all zero)."""
    c = counts[:W]
    if dist.get_backend(group) == "gloo" and c.is_cuda:
        c = c.cpu()
    out = [torch.empty_like(c) for _ in range(W)]
    dist.all_gather(out, c, group=group)
    return torch.stack(out).cpu().tolist()


def choose_splitters(samples, weights, W):
    """W-1 splitters from weighted samples (each stands for `weight` ids):
    splitter j = the first sample whose cumulative weight reaches j*N/W."""
    if W <= 1 or len(samples) == 0:
        return np.zeros(0, np.int64)
    o = np.argsort(samples, kind="stable")
    s, cw = samples[o], np.cumsum(weights[o])
    total = cw[-1]
    at = np.searchsorted(cw, np.arange(1, W) * total / W, side="left")
    return s[np.minimum(at, len(s) - 1)].astype(np.int64)


def weave_distributed(ops, id_key, cause_key, kind, key_bits, ts_shift=0, group=None,
                      root=0, samples=256, tree="auto", ranking="auto", out="root",
                      ruler_k=RULER_K) -> GiantResult:
    """Weave one list whose nodes are spread over the ranks of `group`.

    id_key / cause_key: int64 tensors holding the packed u64 keys (< 2^63);
    kind: uint8.  Every rank calls this; rank `root` receives the weave.
    tree: "dist" builds the tree rank by rank (_tree_distributed), "root" on
    the root alone (cw_weave_ranked), "auto" = dist for W > 1.  Lists outside
    the fast path's domain always take "root" (its exact path).
    ranking (tree "dist" only): "ruling" ranks the list where it lies
    (_rank_ruling, a ruler every ~ruler_k nodes), "root" gathers the
    successors on the root (cw_weave_linked); "auto" = ruling for W > 1.
    out (ranking "ruling" only): "root" -- the whole weave on the root;
    "sharded" -- rank j holds weave positions [pos_base, pos_base + len) (a
    contiguous 1/W of them, 32-aligned), visible_count is the list's total."""
    if key_bits > 63:
        raise ValueError("keys must be < 2^63 (int64 order)")
    if tree not in ("auto", "dist", "root"):
        raise ValueError("tree: auto, dist or root")
    if ranking not in ("auto", "ruling", "root"):
        raise ValueError("ranking: auto, ruling or root")
    if out not in ("root", "sharded"):
        raise ValueError("out: root or sharded")
    if ruler_k < 1:
        raise ValueError("ruler_k >= 1")
    ctx = getattr(ops, "stream_context", contextlib.nullcontext)
    with ctx():
        return _weave_distributed(ops, id_key, cause_key, kind, key_bits, ts_shift, group, root,
                                  samples, tree, ranking, out, ruler_k)


def _any(v, group, dev):
    return sum(x[0] for x in _all_gather_ints([v], group, dev))


def _tree_distributed(ops, par, kind, base, owns, group, dev):
    """(successor word, thread word) of this rank's nodes (global ranks
    [base, base + n)) -- the giant path's tree with the
    cross-rank steps as all-to-all rounds (dist.hip)."""
    W = len(owns)
    N = sum(owns)
    n = par.numel()
    starts = [sum(owns[:j]) for j in range(1, W)] + [N]
    split_t = torch.as_tensor(np.array(starts, np.int64), device=dev)
    # effective parents: climbs leave the run at most W - 1 times
    eff = ops.dist_eff(par, kind, base)
    for _ in range(W + 1):
        keys, waiting = ops.dist_pending(eff)
        if not _any(waiting, group, dev):
            break
        # the climbs that left the run go to the owner of the cause they reached
        perm, counts = ops.partition(keys, split_t)   # W + 1 buckets: the last stays
        send = counts[:W]
        idx = perm[:sum(send)]
        recv = _exchange_counts(send, group, dev)
        rq = _a2a(ops.gather(keys, idx), send, recv, group)
        ans = ops.dist_climb(par, kind, base, rq)
        ops.scatter_into(eff, _a2a(ans, recv, send, group), idx)
    else:
        raise RuntimeError("distributed tree: effective parents did not converge")
    # siblings: local runs of each (e, class), their records at the owner of e
    sk, si = ops.sort_keys32(ops.dist_gkey(eff, kind), 32)
    nsc, okey, rec = ops.dist_runs(sk, si, base, kind)
    del eff, sk, si
    perm, counts = ops.partition(okey, split_t)
    send = counts[:W]
    idx = perm[:sum(send)]
    rs = ops.gather_rows(rec, idx)
    recv = _exchange_counts(send, group, dev)
    rr = _a2a(rs.reshape(-1), [4 * x for x in send], [4 * x for x in recv], group).view(-1, 4)
    fcS, fcN = ops.zeros32(n), ops.zeros32(n)
    rk, ri = ops.sort_keys32(ops.dist_rkey(rr), 32)
    reply = ops.dist_link(rk, ri, rr, base, n, fcS, fcN)
    ops.dist_put(rs, _a2a(reply, recv, send, group), base, nsc)
    del rec, okey, perm, idx, rs, rr, rk, ri, reply
    # threads: chains resolved inside each tile; the rest is chased by the walk
    return ops.dist_succ(kind, fcS, fcN, base), ops.dist_thr(nsc, base)


def _bcast(t, src, group):
    """Broadcast from group rank src (gloo works on host tensors)."""
    if dist.get_world_size(group) == 1:
        return t
    g = dist.get_global_rank(group, src) if group is not None else src
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        c = t.cpu()
        dist.broadcast(c, g, group=group)
        t.copy_(c)
    else:
        dist.broadcast(t, g, group=group)
    return t


def _rank_ruling(ops, succ, thr, org, base, owns, group, dev, root, out, k, n_own, max_ts):
    """The list ranking where the list lies (dist.hip k_rs_*):
    rulers (global rank 0 and ~1/k of the nodes, by hash) walk their sublists
    (cw_dist_rs_walk), a walker crossing ranks travels as a 16-byte message in
    an all-to-all round; the links (one per ruler) are ranked on the root
    (cw_dist_rs_top), the rulers' positions broadcast, and every node's
    position = its ruler's + its offset (cw_dist_rs_pos).  The emit records
    {position, origin | render} go to the root (out="root") or to the owner of
    the position (out="sharded")."""
    W, r = dist.get_world_size(group), dist.get_rank(group)
    n, N = succ.numel(), sum(owns)
    starts = [sum(owns[:j]) for j in range(1, W)] + [N]
    split_t = torch.as_tensor(np.array(starts, np.int64), device=dev)
    word, rlist, nr = ops.rs_rulers(succ, thr, base, k, RULER_SEED)
    rc = [v[0] for v in _all_gather_ints([nr], group, dev)]
    rbase, M = sum(rc[:r]), sum(rc)
    own = ops.zeros32(2 * n)
    links = ops.zeros32(4 * M).view(M, 4)   # any walk may end on this rank
    nlinks, status = ops.zeros32(1), ops.zeros32(1)
    walkers, m, rounds, sent, syncs = None, nr, 0, 0, 0
    while True:
        msg, key = ops.rs_walk(walkers, m, rlist, rbase, word, thr, base, own, links, nlinks,
                               status)
        rounds += 1
        if W == 1:
            break
        # W + 1 buckets (the last: walks that stopped here); the sizes stay on
        # the device until the all_gather, whose one readback is both the
        # exchange's split sizes and the termination test
        perm, counts = ops.partition_dev(key, split_t)
        mat = _gather_count_rows(counts, W, group)
        syncs += 1
        send = mat[r]
        if not any(any(row) for row in mat):
            break
        if rounds > 2 * N + 4:
            raise RuntimeError("ruling set: the walks did not end")
        recv = [mat[j][r] for j in range(W)]
        sent += sum(sum(row) for row in mat)
        idx = perm[:sum(send)]
        walkers = _a2a(ops.gather_rows(msg, idx).reshape(-1), [4 * x for x in send],
                       [4 * x for x in recv], group).view(-1, 4)
        m = walkers.shape[0]
    del word, rlist, walkers
    info = {"rulers": M, "ruler_k": k, "rounds": rounds, "messages": sent,
            "syncs_per_round": syncs / rounds if rounds else 0.0}
    nl = int(nlinks[0])
    agg = _all_gather_ints([nl, int(status[0])], group, dev)
    bad = sum(v[0] for v in agg) != M or any(v[1] for v in agg)
    gsend = [4 * nl if j == root else 0 for j in range(W)]
    grecv = [4 * agg[j][0] if r == root else 0 for j in range(W)]
    all_links = _a2a(links[:nl].reshape(-1), gsend, grecv, group)
    del links
    pos_base = ops.zeros32(M)
    tstat = ops.zeros32(1)
    if r == root and not bad:
        pos_base = ops.rs_top(all_links.view(-1, 4), N, tstat)
    del all_links
    _bcast(pos_base, root, group)
    rec, key = ops.rs_pos(own, pos_base, succ, org, keys=(out == "sharded"))
    del own, pos_base
    estat = ops.zeros32(1)
    if out == "root":
        gsend = [2 * n if j == root else 0 for j in range(W)]
        grecv = [2 * owns[j] if r == root else 0 for j in range(W)]
        allrec = _a2a(rec.reshape(-1), gsend, grecv, group).view(-1, 2)
        if r != root:
            return GiantResult(None, None, None, None, N, n_own, max_ts, ranking=info)
        wp, bits, cnt = ops.rs_emit(allrec, 0, N, estat)
        st = int(tstat[0]) | int(estat[0]) | (STATUS_INTERNAL if bad else 0)
        return GiantResult(wp, bits, int(cnt[0]), st, N, n_own, max_ts, ranking=info)
    # sharded: rank j owns positions [j * chunk, (j + 1) * chunk)
    chunk = ((N + W - 1) // W + 31) // 32 * 32
    ps = torch.as_tensor(np.array([min(j * chunk, N) for j in range(1, W)] + [N], np.int64),
                         device=dev)
    perm, counts = ops.partition(key, ps)
    send = counts[:W]
    recv = _exchange_counts(send, group, dev)
    rows = ops.gather(rec.reshape(-1).view(torch.int64), perm[:sum(send)])
    mine = _a2a(rows, send, recv, group).view(torch.int32).view(-1, 2)
    p0 = min(r * chunk, N)
    wp, bits, cnt = ops.rs_emit(mine, p0, min(p0 + chunk, N) - p0, estat)
    tot = _all_gather_ints([int(cnt[0]), int(tstat[0]) | int(estat[0])], group, dev)
    st = (STATUS_INTERNAL if bad else 0)
    for v in tot:
        st |= v[1]
    return GiantResult(wp, bits, sum(v[0] for v in tot), st, N, n_own, max_ts, pos_base=p0,
                       ranking=info)


def _weave_distributed(ops, id_key, cause_key, kind, key_bits, ts_shift, group, root, samples,
                       tree="auto", ranking="auto", out="root", ruler_k=RULER_K):
    W, r = dist.get_world_size(group), dist.get_rank(group)
    dev = id_key.device
    n = id_key.numel()
    ns = [v[0] for v in _all_gather_ints([n], group, dev)]
    N, in_base = sum(ns), sum(ns[:r])
    if N >= 0x7FFFFFFE:
        raise ValueError(f"list of {N} nodes: limit 2^31-2")

    # 1. local id sort
    sk, si = ops.sort_keys(id_key, key_bits)

    # 2. sample sort: regular samples weighted by the share they stand for
    s = min(samples, n)
    if s:
        pos = ((np.arange(s) + 0.5) * n / s).astype(np.int64)
        smp = sk[torch.as_tensor(pos, device=dev)].cpu().numpy()
    else:
        smp = np.zeros(0, np.int64)
    counts = _all_gather_ints([s], group, dev)
    pad = np.zeros(samples, np.int64)
    pad[:s] = smp
    gath = _all_gather_ints(list(pad), group, dev)
    all_s = np.concatenate([np.array(g[:c[0]], np.int64) for g, c in zip(gath, counts)])
    all_w = np.concatenate([np.full(c[0], ns[j] / max(c[0], 1)) for j, c in enumerate(counts)])
    split = choose_splitters(all_s, all_w, W)
    split_t = torch.as_tensor(split, device=dev)
    # sk is sorted: the ids bound for rank j are one contiguous run
    bounds = torch.searchsorted(sk, split_t).cpu().tolist() if W > 1 else []
    edges = [0] + bounds + [n]
    send = [edges[j + 1] - edges[j] for j in range(W)]
    recv = _exchange_counts(send, group, dev)
    org = (si.to(torch.int64) + in_base).to(torch.int32)
    r_id = _a2a(sk, send, recv, group)
    r_ca = _a2a(ops.gather(cause_key, si), send, recv, group)
    r_kd = _a2a(ops.gather(kind, si), send, recv, group)
    r_org = _a2a(org, send, recv, group)
    del sk, si, org

    # 3. the owner's run of the global id order (one rank: already sorted)
    if W == 1:
        ok, oca, okd, oorg = r_id, r_ca, r_kd, r_org
    else:
        ok, oi = ops.sort_keys(r_id, key_bits)
        oca, okd, oorg = ops.gather(r_ca, oi), ops.gather(r_kd, oi), ops.gather(r_org, oi)
        del oi
    del r_id, r_ca, r_kd, r_org
    n_own = ok.numel()
    owns = [v[0] for v in _all_gather_ints([n_own], group, dev)]
    own_base = sum(owns[:r])
    local_max = int(ok[-1]) >> ts_shift if n_own else 0

    # 4. cause join at the owner of each cause id
    perm, qsend = ops.partition(oca, split_t)
    qrecv = _exchange_counts(qsend, group, dev)
    rq = _a2a(ops.gather(oca, perm), qsend, qrecv, group)
    ans, dup = ops.lookup(ok, rq, own_base)
    back = _a2a(ans, qrecv, qsend, group)
    par = ops.scatter32(back, perm)
    del perm, rq, ans, back, oca

    mx = _all_gather_ints([local_max, dup], group, dev)
    max_ts = max(v[0] for v in mx)
    dups = 0
    for v in mx:  # an id held twice meets itself at its owner (shared.cljc:166-171)
        dups |= v[1]
    if tree == "dist" or (tree == "auto" and W > 1):
        # 5'. the tree rank by rank (dist.hip) when the list is in the fast
        # path's domain; the rank-ordered successors gather on the root
        st = 0
        for v in _all_gather_ints([ops.dist_check(par, okd, own_base)], group, dev):
            st |= v[0]
        if not st and not dups:
            succ, thr = _tree_distributed(ops, par, okd, own_base, owns, group, dev)
            if ranking == "ruling" or (ranking == "auto" and W > 1):
                return _rank_ruling(ops, succ, thr, oorg, own_base, owns, group, dev, root, out,
                                    ruler_k, n_own, max_ts)
            gsend = [n_own if j == root else 0 for j in range(W)]
            grecv = [owns[j] if r == root else 0 for j in range(W)]
            g_succ = _a2a(succ, gsend, grecv, group)
            g_thr = _a2a(thr, gsend, grecv, group)
            g_org = _a2a(oorg, gsend, grecv, group)
            if r != root:
                return GiantResult(None, None, None, None, N, n_own, max_ts)
            o = ops.weave_linked(g_succ, g_thr, g_org)
            return GiantResult(o["weave_perm"], o["visible_bits"], int(o["visible_count"][0]),
                               int(o["status"][0]), N, n_own, max_ts)

    # 5. gather the rank-ordered arrays on the root and weave there (the whole
    # tree on one GPU; also the exact path for lists outside the domain)
    gsend = [n_own if j == root else 0 for j in range(W)]
    grecv = [owns[j] if r == root else 0 for j in range(W)]
    g_par = _a2a(par, gsend, grecv, group)
    g_kd = _a2a(okd, gsend, grecv, group)
    g_org = _a2a(oorg, gsend, grecv, group)
    if r != root:
        return GiantResult(None, None, None, None, N, n_own, max_ts)
    o = ops.weave_ranked(g_par, g_kd, g_org)
    return GiantResult(o["weave_perm"], o["visible_bits"], int(o["visible_count"][0]),
                       int(o["status"][0]) | dups, N, n_own, max_ts)
