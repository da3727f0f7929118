"""Worker of tests/test_gpu_giant.py::test_distributed_two_ranks_share_the_gpu:
one rank of the distributed giant-list weave with the HIP kernels (HipOps) on
cuda:0 and a gloo group (RANK / WORLD_SIZE / MASTER_* from the environment).
Rank 0 checks the gathered weave against the oracle and writes rank0.json."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(outdir):
    import torch
    import torch.distributed as dist

    import oracle
    from cause_amd import abi, giant
    from tests.test_giant_dist import make_list, shares

    torch.cuda.init()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec, idk, ck, kd = make_list(200_000, 31)
        sh = shares(len(idk), world, 31)[rank]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
        lay = spec.layout()
        with abi.Weaver(0) as w:
            ops = giant.HipOps(w, "cuda:0")
            res = giant.weave_distributed(ops, t(idk[sh].view(np.int64)), t(ck[sh].view(np.int64)),
                                          t(kd[sh]), lay.key_bits, ts_shift=lay.ts_shift)
            torch.cuda.synchronize()
        if rank == 0:
            perm, vis, st = oracle.batch_lists(np.array([0, len(idk)], np.uint64), idk, ck, kd,
                                               method=oracle.METHOD_EFF)
            allsh = np.concatenate(shares(len(idk), world, 31))
            wp = res.weave_perm.cpu().numpy().view(np.uint32)
            ok = (res.status == 0 and bool(np.array_equal(allsh[wp], perm))
                  and res.visible_count == int(vis.sum()))
            json.dump({"ok": ok, "status": res.status, "n": res.n_total},
                      open(os.path.join(outdir, "rank0.json"), "w"))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
