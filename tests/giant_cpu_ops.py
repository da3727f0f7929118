"""CPU double of cause_amd.giant.HipOps for the gloo tests of the distributed
giant-list weave (test infrastructure: numpy + the oracle, never shipped).

The exchange logic of giant.weave_distributed (splitters, all_to_all splits,
cause routing, the gather on the root) is what these tests check on CPU; the
HIP kernels behind HipOps are checked against the same doubles on the GPU
(tests/test_gpu_giant.py)."""
import numpy as np
import torch

import oracle

NOT_FOUND = 0xFFFFFFFF


def _u64(t):
    return t.numpy().view(np.uint64)


class CpuOps:
    def sort_keys(self, keys, key_bits):
        k = _u64(keys)
        o = np.argsort(k, kind="stable")
        return torch.from_numpy(k[o].view(np.int64).copy()), torch.from_numpy(o.astype(np.int32))

    def partition(self, keys, splitters):
        b = np.searchsorted(splitters.numpy().view(np.uint64), _u64(keys), side="right")
        perm = np.argsort(b, kind="stable").astype(np.int32)
        counts = np.bincount(b, minlength=splitters.numel() + 1)
        return torch.from_numpy(perm), [int(x) for x in counts]

    def partition_dev(self, keys, splitters):
        perm, counts = self.partition(keys, splitters)
        return perm, torch.tensor(counts, dtype=torch.int64)

    def lookup(self, sorted_keys, queries, base):
        s, q = _u64(sorted_keys), _u64(queries)
        i = np.searchsorted(s, q)
        ok = (i < len(s)) & (s[np.minimum(i, max(len(s) - 1, 0))] == q) if len(s) else \
            np.zeros(len(q), bool)
        out = np.where(ok, i + base, NOT_FOUND).astype(np.uint32)
        out[q == np.uint64(2**64 - 1)] = 0xFFFFFFFE  # CW_NIL_RANK: a nil cause
        dup = 2 if len(s) > 1 and bool((s[1:] == s[:-1]).any()) else 0  # CW_STATUS_DUP
        return torch.from_numpy(out.view(np.int32)), dup

    def sort_keys32(self, keys, key_bits):
        k = keys.numpy().view(np.uint32)
        o = np.argsort(k, kind="stable")
        return torch.from_numpy(k[o].view(np.int32).copy()), torch.from_numpy(o.astype(np.int32))

    def gather(self, src, idx):
        return src[idx.long()]

    def scatter32(self, src, idx):
        out = torch.empty_like(src)
        out[idx.long()] = src
        return out

    def weave_ranked(self, par, kind, val):
        n = par.numel()
        p = par.numpy().view(np.uint32).astype(np.uint64)
        p[0] = np.uint64(2**64 - 1)  # the root's cause is nil
        ranks = np.arange(n, dtype=np.uint64)
        perm, vis, st = oracle.batch_lists(np.array([0, n], np.uint64), ranks, p,
                                           kind.numpy(), method=oracle.METHOD_EFF)
        wp = val.numpy()[perm]
        bits = np.packbits(vis.astype(np.uint8), bitorder="little")
        bits = np.pad(bits, (0, (-len(bits)) % 4)).view(np.int32)
        return {"weave_perm": torch.from_numpy(wp.astype(np.int32)),
                "visible_bits": torch.from_numpy(bits.copy()),
                "visible_count": torch.tensor([int(vis.sum())], dtype=torch.int32),
                "status": torch.tensor([int(st[0])], dtype=torch.int32)}

    # --- the distributed tree (numpy restatement of dist.hip) -------------------
    PEND = RES = 0x80000000
    NONE = 0xFFFFFFFF
    NSC_UP = 0x80000000
    END = 0x7FFFFFFF
    ROOT_KEY = 0xFFFFFFFF

    @staticmethod
    def _special(k):
        return (np.asarray(k) & 3) != 0

    @staticmethod
    def _hide(k):
        k = int(k) & 3
        return k == 1 or k == 2   # hide, h.hide (pack.KIND_*)

    @staticmethod
    def _u32(t):
        return t.numpy().view(np.uint32)

    @staticmethod
    def _t32(a):
        return torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))

    def dist_check(self, par, kind, base):
        p, k = self._u32(par), kind.numpy()
        st = 0
        for i in range(len(p)):
            g = base + i
            if (g == 0) != bool(k[i] & 4):
                st |= 1
            if g > 0 and p[i] >= g:
                st |= 4 if p[i] >= 0xFFFFFFFE else 8
        return st

    def _climb(self, c, p, k, base):
        n = len(p)
        while True:
            if c < base or c - base >= n:
                return self.PEND | c
            if not self._special(k[c - base]):
                return c
            c = int(p[c - base])

    def dist_eff(self, par, kind, base):
        p, k = self._u32(par), kind.numpy()
        out = np.empty(len(p), np.uint32)
        for i in range(len(p)):
            if base + i == 0:
                out[i] = self.NONE
            elif self._special(k[i]):
                out[i] = p[i]
            else:
                out[i] = self._climb(int(p[i]), p, k, base)
        return self._t32(out)

    def dist_climb(self, par, kind, base, q):
        p, k = self._u32(par), kind.numpy()
        return self._t32([self._climb(int(x), p, k, base) for x in _u64(q)])

    def dist_pending(self, w):
        x = self._u32(w).astype(np.uint64)
        pend = ((x & self.PEND) != 0) & (x != self.NONE)
        keys = np.where(pend, x & ~np.uint64(self.PEND), np.uint64(2**64 - 1))
        return torch.from_numpy(keys.view(np.int64)), int(pend.sum())

    def dist_gkey(self, eff, kind):
        e = self._u32(eff).astype(np.uint64)
        cls = np.where(self._special(kind.numpy()), 0, 1).astype(np.uint64)
        key = np.where(e == self.NONE, np.uint64(self.ROOT_KEY), (e << np.uint64(1)) | cls)
        return self._t32(key.astype(np.uint32))

    def dist_runs(self, skey, sidx, base, kind):
        sk, si, k = skey.numpy().view(np.uint32), sidx.numpy().view(np.uint32), kind.numpy()
        n = len(sk)
        nsc = np.zeros(n, np.uint32)
        okey = np.full(n, 2**64 - 1, np.uint64)
        rec = np.zeros((n, 4), np.uint32)
        for i in range(n):
            kk = int(sk[i])
            if kk == self.ROOT_KEY:
                continue
            x = int(si[i])
            if i > 0 and sk[i - 1] == sk[i]:
                nsc[x] = base + int(si[i - 1])
                continue
            j = i
            while j + 1 < n and sk[j + 1] == sk[i]:
                j += 1
            newest = int(si[j])
            nsc[x] = self.NSC_UP | (kk >> 1)
            okey[i] = kk >> 1
            rec[i] = (kk & 0xFFFFFFFF, base + x, base + newest, k[newest])
        return (self._t32(nsc), torch.from_numpy(okey.view(np.int64)),
                torch.from_numpy(rec.view(np.int32)))

    def dist_rkey(self, rec):
        r = rec.numpy().view(np.uint32)
        return self._t32(np.ascontiguousarray(r[:, 0]))

    def dist_link(self, skey, sidx, rec, base, n, fcS, fcN):
        sk, si = skey.numpy().view(np.uint32), sidx.numpy().view(np.uint32)
        r = rec.numpy().view(np.uint32)
        fs, fn = fcS.numpy().view(np.uint32), fcN.numpy().view(np.uint32)
        m = len(sk)
        g = sk.astype(np.uint64)
        reply = np.zeros(m, np.uint32)
        for j in range(m):
            gj, e = int(g[j]), int(g[j]) >> 1
            first = j == 0 or g[j - 1] != g[j]
            last = j + 1 == m or g[j + 1] != g[j]
            ns = self.NSC_UP | e
            if not first:
                ns = int(r[si[j - 1], 2])
            elif not gj & 1:
                hit = np.flatnonzero(g == (gj | 1))
                if len(hit):
                    ns = int(r[si[hit[-1]], 2])
            reply[si[j]] = ns
            if last and base <= e < base + n:
                hi = int(r[si[j], 2])
                if gj & 1:
                    fn[e - base] = hi
                else:
                    fs[e - base] = hi | (0x80000000 if self._hide(r[si[j], 3]) else 0)
        return self._t32(reply)

    def dist_put(self, rec, reply, base, nsc):
        r, rp, ns = rec.numpy().view(np.uint32), self._u32(reply), nsc.numpy().view(np.uint32)
        for i in range(len(rp)):
            ns[int(r[i, 1]) - base] = rp[i]

    def dist_thr(self, nsc, base, tile=1024):
        """Thread words: chains followed inside each tile of the run; one that
        leaves the tile ends as PEND | the ancestor outside."""
        s = self._u32(nsc)
        n = len(s)
        out = np.zeros(n, np.uint32)
        for i in range(n):
            g0 = base + (i // tile) * tile
            j = i
            while True:
                g = base + j
                if g == 0:
                    out[i] = self.END
                    break
                x = int(s[j])
                if not x & self.NSC_UP:
                    out[i] = x
                    break
                e = x & ~self.NSC_UP
                if e < g0:
                    out[i] = self.PEND | e
                    break
                if e >= g:   # (out of domain)
                    out[i] = self.END
                    break
                j = e - base
        return self._t32(out)

    def dist_succ(self, kind, fcS, fcN, base):
        k = kind.numpy()
        fs, fn = self._u32(fcS), self._u32(fcN)
        out = np.zeros(len(k), np.uint32)
        for i in range(len(k)):
            f = int(fs[i]) & 0x7FFFFFFF
            succ = f if f else (int(fn[i]) if fn[i] else 0x7FFFFFFE)
            vis = not self._special(k[i]) and base + i != 0 and not (fs[i] and fs[i] & 0x80000000)
            out[i] = succ | (0x80000000 if vis else 0)
        return self._t32(out)

    # --- the ruling-set ranking (numpy restatement of dist.hip k_rs_*) ---------
    CHASE = 0x80000000
    RS_NONE = 0xFFFFFFFF

    @staticmethod
    def _mix32(a, b):
        m = np.uint64(0xFFFFFFFF)
        h = (np.uint64(a) * np.uint64(0x9E3779B1) + np.asarray(b, np.uint64)) & m
        h ^= h >> np.uint64(16)
        h = (h * np.uint64(0x85EBCA6B)) & m
        h ^= h >> np.uint64(13)
        h = (h * np.uint64(0xC2B2AE35)) & m
        h ^= h >> np.uint64(16)
        return h

    def _ruler(self, g, k, seed):
        g = np.asarray(g, np.uint64)
        return (g == 0) | (self._mix32(seed, g) * np.uint64(k) < np.uint64(1 << 32))

    def rs_rulers(self, succ, thr, base, k, seed):
        s, t = self._u32(succ), self._u32(thr)
        n = len(s)
        nx = s & np.uint32(0x7FFFFFFF)
        ft = nx == 0x7FFFFFFE
        tv = np.where(t & self.PEND, self.CHASE | (t & np.uint32(0x7FFFFFFF)), t)
        nx = np.where(ft, tv, nx).astype(np.uint32)
        f = self._ruler(base + np.arange(n, dtype=np.uint64), k, seed)
        ridx = np.full(n, self.RS_NONE, np.uint32)
        ridx[f] = np.arange(int(f.sum()), dtype=np.uint32)
        word = np.stack([nx, ridx], 1)
        rlist = np.zeros(n, np.uint32)
        rlist[:int(f.sum())] = np.flatnonzero(f)
        return self._t32(word), self._t32(rlist), int(f.sum())

    def rs_walk(self, walkers, m, rlist, rbase, word, thr, base, own, links, nlinks, status):
        wd = word.numpy().view(np.uint32)
        th, rl = self._u32(thr), self._u32(rlist)
        ow, lk = own.numpy().view(np.uint32), links.numpy().view(np.uint32)
        nl = nlinks.numpy().view(np.uint32)
        n = wd.shape[0]
        out = np.zeros((m, 4), np.uint32)
        key = np.full(m, 2**64 - 1, np.uint64)
        wk = walkers.numpy().view(np.uint32) if walkers is not None else None
        for i in range(m):
            if wk is not None:
                R, cnt, tgt = int(wk[i, 0]), int(wk[i, 1]), int(wk[i, 2])
            else:
                R, cnt, tgt = rbase + i, 0, base + int(rl[i])
            link, lnext = False, self.RS_NONE
            while True:
                a = tgt & 0x7FFFFFFF
                if not base <= a < base + n:
                    key[i] = a
                    break
                if tgt & self.CHASE:
                    t = int(th[a - base])
                    nx = self.CHASE | (t & 0x7FFFFFFF) if t & self.PEND else t
                else:
                    x, r = int(wd[a - base, 0]), int(wd[a - base, 1])
                    if r != self.RS_NONE and cnt > 0:
                        link, lnext = True, rbase + r
                        break
                    ow[2 * (a - base)], ow[2 * (a - base) + 1] = R, cnt
                    cnt += 1
                    nx = x
                if nx == self.END:
                    link = True
                    break
                tgt = nx
            out[i] = (R, cnt, tgt, 0)
            if link:
                lk[int(nl[0])] = (R, lnext, cnt, 0)
                nl[0] += 1
        return self._t32(out), torch.from_numpy(key.view(np.int64))

    def rs_top(self, links, total, status):
        lk = links.numpy().view(np.uint32)
        m = lk.shape[0]
        nxt = np.full(m, self.RS_NONE, np.int64)
        ln = np.zeros(m, np.int64)
        nxt[lk[:, 0]] = lk[:, 1]
        ln[lk[:, 0]] = lk[:, 2]
        pos = np.zeros(m, np.uint32)
        r, p, seen = 0, 0, 0
        while r != self.RS_NONE and seen <= m:
            pos[r] = p
            p += int(ln[r])
            r = int(nxt[r])
            seen += 1
        if p != total or seen != m:
            status.numpy()[0] |= 32
        return self._t32(pos)

    def rs_pos(self, own, pos_base, succ, val, keys=False):
        ow = own.numpy().view(np.uint32).reshape(-1, 2)
        pb, s, v = self._u32(pos_base), self._u32(succ), self._u32(val)
        p = pb[ow[:, 0]].astype(np.uint64) + ow[:, 1] if len(ow) else np.zeros(0, np.uint64)
        rec = np.stack([p.astype(np.uint32), (v & np.uint32(0x7FFFFFFF)) | (s & np.uint32(0x80000000))], 1)
        return self._t32(rec.reshape(-1, 2)), (torch.from_numpy(p.astype(np.int64)) if keys else None)

    def rs_emit(self, rec, p0, length, status):
        r = rec.numpy().view(np.uint32).reshape(-1, 2)
        perm = np.zeros(length, np.uint32)
        vis = np.zeros(length, np.uint8)
        p = r[:, 0].astype(np.int64) - p0
        if ((p < 0) | (p >= length)).any():
            status.numpy()[0] |= 32
        ok = (p >= 0) & (p < length)
        perm[p[ok]] = r[ok, 1] & 0x7FFFFFFF
        vis[p[ok]] = r[ok, 1] >> 31
        bits = np.packbits(vis, bitorder="little")
        bits = np.pad(bits, (0, (-len(bits)) % 4)).view(np.int32)
        return (self._t32(perm), torch.from_numpy(bits.copy()),
                torch.tensor([int(vis.sum())], dtype=torch.int32))

    def gather_rows(self, rec, idx):
        return rec[idx.long()]

    def scatter_into(self, dst, src, idx):
        dst[idx.long()] = src

    def zeros32(self, n):
        return torch.zeros(n, dtype=torch.int32)

    def weave_linked(self, succ, thr, val):
        """The list ranking by walking the successors from the root (rank 0);
        a thread successor is chased through the thread words."""
        s, th = self._u32(succ), self._u32(thr)
        n = len(s)
        order, vis = np.empty(n, np.int64), np.zeros(n, np.uint8)
        x, g = 0, 0
        while x < n and g < n:
            order[g] = x
            vis[g] = 1 if s[x] & 0x80000000 else 0
            nx = int(s[x]) & 0x7FFFFFFF
            if nx == 0x7FFFFFFE:
                t = int(th[x])
                while t & self.PEND:
                    t = int(th[t & 0x7FFFFFFF])
                nx = t
            x = nx
            g += 1
        st = 0 if g == n else 32   # CW_STATUS_INTERNAL
        wp = val.numpy()[order[:g]] if g == n else np.zeros(n, np.int32)
        bits = np.packbits(vis, bitorder="little")
        bits = np.pad(bits, (0, (-len(bits)) % 4)).view(np.int32)
        return {"weave_perm": torch.from_numpy(np.ascontiguousarray(wp).astype(np.int32)),
                "visible_bits": torch.from_numpy(bits.copy()),
                "visible_count": torch.tensor([int(vis.sum())], dtype=torch.int32),
                "status": torch.tensor([st], dtype=torch.int32)}
