"""Code-object checks on the built library (CPU only): no kernel of
libcauseweave.so uses scratch memory or spills vector registers.  (A few SGPR
spills with no private segment go to VGPR lanes -- v_writelane/v_readlane, no
memory traffic -- and are allowed.)

A run-time index into a small register array (a uint4 picked by word number,
a lambda capturing arrays by reference) silently becomes a private-memory
array; k_front's rank pass ran 3x slower that way.  The metadata notes of the
gfx950 code object say so per kernel (.private_segment_fixed_size)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cause_amd", "libcauseweave.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernel_meta(tmp_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("llvm tools not present")
    if not os.path.exists(LIB):
        pytest.skip("libcauseweave.so not built")
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([objdump, "--offloading", str(lib)], cwd=tmp_path, check=True,
                   capture_output=True)
    cos = [f for f in os.listdir(tmp_path) if "gfx950" in f]
    assert cos, "no gfx950 code object in libcauseweave.so"
    notes = subprocess.run([readelf, "--notes", str(tmp_path / cos[0])], check=True,
                           capture_output=True, text=True).stdout
    kernels, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m and m.group(1).startswith("_Z"):
            cur = kernels.setdefault(m.group(1), {})
            continue
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\d+)",
                     line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return kernels


def test_no_kernel_uses_scratch(tmp_path):
    kernels = _kernel_meta(tmp_path)
    assert any("k_tree" in k for k in kernels) and any("k_front" in k for k in kernels)
    # the phase-stamp builds of k_tree_l and k_weave_doc (template flag PROF = true, CW_TREE_PROF
    # only) keep 16 timers in SGPRs and may spill a few more of them to lanes
    diag = lambda k: re.search(r"k_tree_lILi\d+ELi\d+ELb1E|k_weave_docILi\d+ELi\d+E.Lb1E", k) is not None
    # (an SGPR spill goes to a VGPR lane -- v_writelane, no memory -- as long as
    # there is no private segment; k_map_pack's look-back epoch and layout
    # arguments spill 10 of them)
    # the fused weave with in-kernel yarns (template flag YF = true, the last
    # one) holds the staged yarns' wave-uniform bounds on top of the tree's and
    # the tour's 30-odd pointer arguments: a few dozen SGPRs go to lanes there
    yarn = lambda k: re.search(r"k_weave_docILi\d+ELi\d+E.Lb0ELi\d+ELi\d+ELb1E", k) is not None
    lim = lambda k: 64 if diag(k) else 48 if yarn(k) else 16
    bad = {k: v for k, v in kernels.items() if v.get("private_segment_fixed_size", 0)
           or v.get("vgpr_spill_count", 0) or v.get("sgpr_spill_count", 0) > lim(k)}
    assert not bad, f"kernels using scratch: {bad}"
