"""CPU study: rounds and messages of a distributed ruling-set list
ranking for config 5, on the oracle's weave of a config-5-shaped list laid over W
ranks as the sample sort lays it.  python scripts/ruling_study.py [nodes]"""
import sys, dataclasses, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import oracle
from cause_amd import gen
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=N)
off, idk, ck, kd = gen.generate(spec, 0, 1, nthreads=8)
perm, st = oracle.list_weave(idk, ck, kd, oracle.METHOD_EFF)
assert st == 0
n = len(idk)
rank = np.empty(n, np.int64); rank[np.argsort(idk, kind='stable')] = np.arange(n)
seq = rank[perm]  # global id rank of the node at each weave position
rng = np.random.default_rng(1)
for W in (2, 4, 8):
    owner = seq * W // n
    cross = owner[1:] != owner[:-1]
    print(f"W={W}: successors crossing ranks {cross.mean():.3f}")
    for K in (8, 16, 32, 64, 256, 1024):
        ruler = rng.random(n) < 1.0 / K
        ruler[0] = True
        rpos = np.flatnonzero(ruler)
        # crossings inside each sublist [rpos[i], rpos[i+1])
        cc = np.concatenate([[0], np.cumsum(cross)])
        ends = np.concatenate([rpos[1:], [n]])
        c = cc[ends - 1] - cc[rpos]  # crossings between consecutive positions inside the sublist
        rounds = int(c.max()) + 1
        msgs = int(c.sum())
        print(f"  K={K:5d}: rulers {len(rpos):9,d}  rounds {rounds:4d}  messages {msgs:,} ({msgs / n:.3f}/node)"
              f"  top level {len(rpos):,}")
