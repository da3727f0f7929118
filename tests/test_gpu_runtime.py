"""One HIP runtime per process: a Weaver created before `import torch` must
leave torch's GPU usable (abi._share_torch_hip_runtime), and both see one
libamdhip64 mapping."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
import re
from cause_amd import abi
w = abi.Weaver(0)
import torch
assert torch.cuda.is_available(), "torch lost the GPU"
maps = set(re.findall(r"\S*libamdhip64\S*", open("/proc/self/maps").read()))
assert len(maps) == 1, maps
x = torch.arange(10, device="cuda")
w.set_stream(torch.cuda.current_stream().cuda_stream)
w.set_stream(None)
w.close()
print("ok", int(x.sum()))
"""


def test_weaver_first_then_torch_share_one_runtime():
    p = subprocess.run([sys.executable, "-c", PROG], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "ok 45" in p.stdout
