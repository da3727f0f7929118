"""Document sharding across ranks (one process per GPU, torch.distributed).

Independent documents need no exchange: rank r of W
owns a contiguous document range and weaves it alone.  The only collectives are
bookkeeping: a barrier around the timed region and a MAX of the per-rank time
(bench.py) or a SUM of per-rank counters (tests).
"""
from __future__ import annotations


def doc_range(rank: int, world: int, docs_per_rank: int | None = None,
              total_docs: int | None = None):
    """[begin, end) documents of ``rank``.

    Weak scaling (``docs_per_rank``): every rank owns the same number of
    documents, rank r owns [r*D, (r+1)*D).  Strong scaling (``total_docs``):
    a fixed batch is split as evenly as possible, earlier ranks taking the
    remainder."""
    if (docs_per_rank is None) == (total_docs is None):
        raise ValueError("give exactly one of docs_per_rank / total_docs")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if docs_per_rank is not None:
        return rank * docs_per_rank, (rank + 1) * docs_per_rank
    q, r = divmod(total_docs, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def _dev(dist, device):
    """gloo reduces host tensors (it also carries ranks that share one GPU)."""
    return device if dist.get_backend() == "nccl" else None


def reduce_max_time(seconds: float, dist, device=None) -> float:
    """MAX over ranks of a per-rank wall time (the bench's whole-job time)."""
    import torch

    t = torch.tensor([seconds], dtype=torch.float64, device=_dev(dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(values, dist, device=None):
    """SUM over ranks of a list of integers (e.g. nodes woven, checksums)."""
    import torch

    t = torch.tensor(list(values), dtype=torch.int64, device=_dev(dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]
