"""Worker of tests/test_gpu_giant.py::test_distributed_two_ranks_share_the_gpu:
one rank of the distributed giant-list weave with the HIP kernels (HipOps) on
cuda:0 and a gloo group (RANK / WORLD_SIZE / MASTER_* from the environment).
Rank 0 checks the gathered weave against the oracle and writes rank0.json."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(outdir, ranking="auto", out="root"):
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
                                          t(kd[sh]), lay.key_bits, ts_shift=lay.ts_shift,
                                          ranking=ranking, out=out)
            torch.cuda.synchronize()
        if out == "sharded":
            # the slices meet on rank 0 (gloo: host tensors)
            parts = [None] * world
            dist.all_gather_object(parts, (res.pos_base, res.weave_perm.cpu().numpy(),
                                           res.visible_bits.cpu().numpy(), res.status))
            if rank == 0:
                perm, vis, st = oracle.batch_lists(np.array([0, len(idk)], np.uint64), idk, ck, kd,
                                                   method=oracle.METHOD_EFF)
                allsh = np.concatenate(shares(len(idk), world, 31))
                parts.sort(key=lambda p: p[0])
                wp = np.concatenate([p[1] for p in parts]).view(np.uint32)
                bits = np.concatenate([np.unpackbits(p[2].view(np.uint8), bitorder="little")[:len(p[1])]
                                       for p in parts])
                ok = (all(p[3] == 0 for p in parts) and bool(np.array_equal(allsh[wp], perm))
                      and bool(np.array_equal(bits, vis)) and res.visible_count == int(vis.sum()))
                json.dump({"ok": ok, "status": [p[3] for p in parts], "n": res.n_total},
                          open(os.path.join(outdir, "rank0.json"), "w"))
            return
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
    main(*sys.argv[1:])
