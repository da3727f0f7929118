"""The document-sharded product path with two ranks on one GPU.

`python bench.py --gpus 2` (no launcher in the environment) starts its own two
ranks through torch.distributed.run (bench.launch_ranks); they share cuda:0
here, so their bookkeeping collectives go over gloo.  Each rank weaves its own
contiguous document range through the C ABI and, with --check, compares every
one of its documents / collections with the CPU oracle; the mismatch counts are
summed over the ranks into the JSON line (configs 2-4 shard with
no data-path collective).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]  # rank 0 only
    return json.loads(lines[0])


def test_config2_two_ranks_every_document_checked():
    line = _bench("--gpus", "2", "--config", "2", "--docs", "40", "--nodes", "3000",
                  "--steps", "2", "--warmup", "1", "--no-cpu", "--no-h2d", "--check")
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "docs sharded x2"
    assert line["check"]["documents_checked"] == 80
    assert line["check"]["mismatches"] == 0
    assert line["value"] > 0


def test_config4_two_ranks_every_collection_checked():
    line = _bench("--gpus", "2", "--config", "4", "--colls", "3000", "--steps", "2",
                  "--warmup", "1", "--no-cpu", "--check")
    assert line["n_gpus"] == 2
    assert line["check"]["collections_checked"] == 6000
    assert line["check"]["mismatches"] == 0
