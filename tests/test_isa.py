"""The gfx950 build of the kernels (tools/isa_check.py): no production kernel
touches scratch or issues flat memory operations.  Both appear when a kernel
indexes an array of its arguments at run time (the array is copied to
scratch, and the pointers the kernel loads from it lose their address space):
round 4 found the fan-out scan at 2x its time that way.  The bounds-checked
debug instantiations (CK = true) are exempt."""

import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="needs hipcc")
def test_no_scratch_or_flat_in_production_kernels():
    import isa_check
    res = isa_check.census()
    assert any("tm_match_tiles" in k for k in res)
    bad = {k: v for k, v in res.items() if (v[1] or v[2]) and "ILb1E" not in k}
    assert not bad, bad
