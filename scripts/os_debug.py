import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cause_amd import abi
os.environ["CW_ONESWEEP"] = "1"
w = abi.Weaver(0)
for n, bits in ((65536, 9), (65536, 8), (4096 * 8, 9), (4096 * 16, 17), (65536, 17), (4096 * 24, 9)):
    rng = np.random.default_rng(1)
    k = rng.integers(0, 1 << bits, n, dtype=np.uint64)
    ko, io = w.sort_keys(k, bits)
    order = np.argsort(k, kind="stable")
    bad = np.nonzero(ko != k[order])[0]
    badi = np.nonzero(io != order)[0]
    print(n, bits, "bad keys", len(bad), bad[:10], "bad idx", len(badi), badi[:10], flush=True)
    if len(bad):
        i = bad[0]
        print("  got", ko[max(0, i - 3):i + 5], "want", k[order][max(0, i - 3):i + 5])
        # which tiles/chunks do the misplaced values come from
        src = io[bad[:20]]
        print("  src of bad", src, "tile", src // 4096, "chunk", (src // 4096) // ((n + 4095) // 4096 // 8 or 1))
        cnt = np.bincount((k & np.uint64((1 << bits) - 1)).astype(np.int64), minlength=1 << bits)
        print("  keys sorted multiset equal:", np.array_equal(np.sort(ko), np.sort(k)))
