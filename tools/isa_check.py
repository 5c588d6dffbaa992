"""Per-kernel ISA census of tm_kernels.hip (dev tool): instruction count,
scratch and flat memory ops -- a kernel-argument array indexed at run time is
copied to scratch and every pointer it reaches becomes flat (slow).

    python tools/isa_check.py [kernel-substring]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def hipcc() -> str:
    """The compiler the test's skip check found: /opt/rocm/bin/hipcc, else hipcc on PATH."""
    import shutil
    if os.path.exists("/opt/rocm/bin/hipcc"):
        return "/opt/rocm/bin/hipcc"
    return shutil.which("hipcc") or "hipcc"


def census():
    """{kernel symbol: (instructions, scratch ops, flat ops)} of the gfx950 build."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                        os.path.join(ROOT, "emqx_amd", "csrc", "tm_kernels.hip"), "-o", out], check=True,
                       stderr=subprocess.DEVNULL)
        s = open(out).read()
    res = {}
    for m in re.finditer(r"^(_ZN3etm\w+):", s, re.M):
        name = m.group(1)
        j = s.find(".Lfunc_end", m.end())
        body = s[m.end():j]
        ops = [ln.split()[0] for ln in body.split("\n") if ln.startswith("\t") and ln.split() and not ln.startswith("\t.")]
        c = collections.Counter(ops)
        scratch = sum(v for k, v in c.items() if k.startswith("scratch_"))
        flat = sum(v for k, v in c.items() if k.startswith("flat_"))
        res[name] = (len(ops), scratch, flat)
    return res


def main():
    want = sys.argv[1] if len(sys.argv) > 1 else ""
    bad = 0
    for name, (n, scratch, flat) in census().items():
        if want in name:
            print(f"{name[:70]:70s} instrs {n:6d} scratch {scratch:4d} flat {flat:4d}")
        bad += scratch + flat
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
