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

    def lookup(self, sorted_keys, queries, base):
        s, q = _u64(sorted_keys), _u64(queries)
        i = np.searchsorted(s, q)
        ok = (i < len(s)) & (s[np.minimum(i, max(len(s) - 1, 0))] == q) if len(s) else \
            np.zeros(len(q), bool)
        out = np.where(ok, i + base, NOT_FOUND).astype(np.uint32)
        out[q == np.uint64(2**64 - 1)] = 0xFFFFFFFE  # CW_NIL_RANK: a nil cause
        dup = 2 if len(s) > 1 and bool((s[1:] == s[:-1]).any()) else 0  # CW_STATUS_DUP
        return torch.from_numpy(out.view(np.int32)), dup

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
