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


def _measured(line):
    """An N > 1 line carries the CPU baseline (rank 0, after the GPU region) and a
    traffic field: the PMC bytes, or null with the reason."""
    cpu = line["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port"
    assert "traffic" in line["roofline"] and line["roofline"]["traffic_note"]


def test_config2_two_ranks_every_document_checked():
    line = _bench("--gpus", "2", "--config", "2", "--docs", "40", "--nodes", "3000",
                  "--steps", "2", "--warmup", "1", "--cpu-seconds", "1", "--no-h2d", "--check")
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "docs sharded x2"
    assert line["check"]["documents_checked"] == 80
    assert line["check"]["mismatches"] == 0
    assert line["value"] > 0
    _measured(line)


def test_config2_two_ranks_full_size_line_is_measured():
    # the driver's SCALE line at N = 2: the default per-GPU batch, so the PMC
    # traffic of this build applies (null only when profiles/ are stale)
    line = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu-seconds", "2",
                  timeout=600)
    assert line["n_gpus"] == 2 and line["config"]["nodes_per_gpu"] == 500_010_000
    _measured(line)
    r = line["roofline"]
    assert r["traffic"] is not None, r["traffic_note"]
    assert line["cpu_baseline_parallel"]["value"] > 0


def test_config3_two_ranks_every_streamed_document_checked():
    line = _bench("--gpus", "2", "--config", "3", "--stream-docs", "120", "--docs", "20",
                  "--nodes", "3000", "--warmup", "1", "--cpu-seconds", "1", "--check")
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "docs sharded x2"
    assert line["check"]["documents_checked"] == 120
    assert line["check"]["mismatches"] == 0
    _measured(line)


def test_config4_two_ranks_every_collection_checked():
    line = _bench("--gpus", "2", "--config", "4", "--colls", "3000", "--steps", "2",
                  "--warmup", "1", "--cpu-seconds", "1", "--check")
    assert line["n_gpus"] == 2
    assert line["check"]["collections_checked"] == 6000
    assert line["check"]["mismatches"] == 0
    _measured(line)
