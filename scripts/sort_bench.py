"""A/B of the one-array sort behind cw_sort_keys (config 5's id sort) on the
GPU: N random keys of B bits, each CW_ONESWEEP geometry in its own context,
per-kernel HIP-event times over R repetitions, outputs compared across
geometries.  python scripts/sort_bench.py [N] [B] [R]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cause_amd import abi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000_001
B = int(sys.argv[2]) if len(sys.argv) > 2 else 35
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
GEOMS = os.environ.get("GEOMS", "0,1,2,3").split(",")
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
keys = torch.randint(0, 1 << B, (N,), dtype=torch.int64, device=dev, generator=g)
kout = torch.empty_like(keys)
iout = torch.empty(N, dtype=torch.int32, device=dev)
ref = None
for geom in GEOMS:
    os.environ["CW_ONESWEEP"] = geom
    w = abi.Weaver(0)
    w.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    w.sort_keys_device(keys.data_ptr(), N, B, kout.data_ptr(), iout.data_ptr())  # warm
    torch.cuda.synchronize()
    w.reset_kernel_stats()
    w.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(R):
        w.sort_keys_device(keys.data_ptr(), N, B, kout.data_ptr(), iout.data_ptr())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / R
    w.set_profiling(False)
    st = w.kernel_stats()
    h = iout[:: max(1, N // 4_000_000)].cpu().numpy()
    same = None if ref is None else bool(np.array_equal(h, ref))
    if ref is None:
        ref = h
    ok = bool((kout[1:] >= kout[:-1]).all().item())
    line = {"geom": geom, "n": N, "bits": B, "ms_per_sort": round(dt * 1e3, 3), "sorted": ok,
            "same_as_first": same,
            "kernels_ms": {k: round(v[1] / R, 3) for k, v in st.items()},
            "kernel_gbs": {k: round(v[2] / (v[1] / 1e3) / 1e9, 1) for k, v in st.items() if v[1] > 0}}
    print(json.dumps(line), flush=True)
    w.close()
