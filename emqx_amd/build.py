"""In-tree build of the native libraries (no cmake/ninja, no JIT cache).

    python -m emqx_amd.build          # libemqx_tm.so (gfx950) + libemqx_gen.so
"""

from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

TM_SOURCES = ["tm_engine.cpp", "tm_churn.cpp", "tm_upload.cpp", "tm_batch.cpp", "tm_async.cpp", "tm_pipeline.cpp",
              "tm_fanout.cpp", "tm_group.cpp", "tm_shard.cpp", "tm_kernels.hip"]
TM_HEADERS = ["tm_internal.hpp", "tm_engine_impl.hpp", os.path.join("..", "..", "include", "emqx_tm.h")]


def _digest(deps, extra=""):
    h = hashlib.sha256(extra.encode())
    for d in deps:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _stale(out, deps, extra=""):
    """A built library is reused only if its stamp names the digest of exactly
    these sources (and flags): a snapshot copied to another machine keeps no
    trustworthy mtimes, and a stale .so must never pass for the current code."""
    stamp = out + ".srchash"
    if not os.path.exists(out) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(deps, extra)


def _stamp(out, deps, extra=""):
    with open(out + ".srchash", "w") as f:
        f.write(_digest(deps, extra) + "\n")


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_tm(force=False):
    out = os.path.join(HERE, "libemqx_tm.so")
    deps = [os.path.join(CSRC, f) for f in TM_SOURCES + TM_HEADERS]
    if force or _stale(out, deps, ARCH):
        tmp = out + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-fvisibility=hidden", "-Wall", "-Wl,-soname,libemqx_tm.so",
              f'-DTM_SRC_HASH="{_digest(deps, ARCH)}"', "-o", tmp]
             + [os.path.join(CSRC, f) for f in TM_SOURCES] + ["-lpthread"])
        os.replace(tmp, out)
        _stamp(out, deps, ARCH)
    return out


def source_hash():
    """Digest of the engine's sources: tm_build_info() of a library built from
    them ends with it (tests check the loaded .so is the current code)."""
    return _digest([os.path.join(CSRC, f) for f in TM_SOURCES + TM_HEADERS], ARCH)


def build_gen(force=False):
    out = os.path.join(HERE, "libemqx_gen.so")
    src = os.path.join(CSRC, "tm_gen.c")
    if force or _stale(out, [src]):
        _run(["gcc", "-O2", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall", "-o", out, src, "-lm"])
        _stamp(out, [src])
    return out


def build_load(force=False):
    """libemqx_load.so: the per-publish load generator (bench / tests only)."""
    out = os.path.join(HERE, "libemqx_load.so")
    src = os.path.join(CSRC, "tm_load.cpp")
    deps = [src, os.path.join(HERE, "libemqx_tm.so"), os.path.join(ROOT, "include", "emqx_tm.h")]
    if force or _stale(out, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall", "-o", out, src,
              "-L" + HERE, "-lemqx_tm", "-Wl,-rpath,$ORIGIN", "-lpthread"])
        _stamp(out, deps)
    return out


def build_nif_mock(force=False):
    """libemqx_nif_mock.so: the erl_nif shim linked against the test stand-in
    for the Erlang runtime (tests/nif_mock), so tests can drive the NIF."""
    out = os.path.join(HERE, "libemqx_nif_mock.so")
    mock = os.path.join(ROOT, "tests", "nif_mock")
    srcs = [os.path.join(CSRC, "nif", "emqx_tm_nif.c"), os.path.join(mock, "mock_erts.c")]
    deps = srcs + [os.path.join(mock, "erl_nif.h"), os.path.join(HERE, "libemqx_tm.so"),
                   os.path.join(ROOT, "include", "emqx_tm.h")]
    if force or _stale(out, deps):
        _run(["gcc", "-O1", "-g", "-std=gnu11", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror",
              "-I" + mock, "-I" + os.path.join(ROOT, "include"), "-o", out] + srcs +
             ["-L" + HERE, "-lemqx_tm", "-Wl,-rpath,$ORIGIN", "-lpthread"])
        _stamp(out, deps)
    return out


def build_all(force=False):
    return [build_tm(force), build_gen(force), build_load(force), build_nif_mock(force)]


SAN_FLAGS = {
    # host code only: every -fsanitize= right after -Xarch_host (no GPU sanitizer on this pool)
    "asan": ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-sanitize-recover=undefined"],
    "tsan": ["-Xarch_host", "-fsanitize=thread"],
}
SAN_LINK = {"asan": ["-fsanitize=address,undefined"], "tsan": ["-fsanitize=thread"]}
LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def san_runtime(kind):
    """The clang sanitizer runtime a process must preload to load a sanitized
    library from an uninstrumented interpreter (LD_PRELOAD)."""
    import glob
    name = {"asan": "libclang_rt.asan-x86_64.so", "tsan": "libclang_rt.tsan-x86_64.so"}[kind]
    hits = sorted(glob.glob(f"/opt/rocm/lib/llvm/lib/clang/*/lib/linux/{name}"))
    return hits[-1] if hits else None


def build_sanitized(kind, force=False, jobs=8):
    """Host-sanitized builds for the CPU sanitizer tests:
    emqx_amd/variants/<kind>/libemqx_tm.so (the engine's host C++ under
    ASan + UBSan, or TSan) and libemqx_nif_mock.so (the erl_nif shim + the
    runtime stand-in, same sanitizer, linked to it).  The kernels' object is
    built once, unsanitized (device code is not instrumented either way).
    -> the directory."""
    from concurrent.futures import ThreadPoolExecutor
    out_dir = os.path.join(HERE, "variants", kind)
    obj_dir = os.path.join(HERE, "variants", "obj")
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(obj_dir, exist_ok=True)
    hdrs = [os.path.join(CSRC, f) for f in TM_HEADERS]
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-g",
             "-fno-omit-frame-pointer"]
    lib = os.path.join(out_dir, "libemqx_tm.so")
    deps = [os.path.join(CSRC, f) for f in TM_SOURCES] + hdrs
    if force or _stale(lib, deps, kind + ARCH):
        def obj(src, san):
            base = os.path.splitext(os.path.basename(src))[0]
            o = os.path.join(obj_dir if not san else out_dir, base + ".o")
            key = (kind if san else "") + ARCH
            if force or _stale(o, [src] + hdrs, key):
                _run([HIPCC, *flags, "-O1" if san else "-O3", *(SAN_FLAGS[kind] if san else []),
                      f'-DTM_SRC_HASH="{_digest(deps, ARCH)}"', "-c", "-o", o, src])
                _stamp(o, [src] + hdrs, key)
            return o
        srcs = [os.path.join(CSRC, f) for f in TM_SOURCES]
        with ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(lambda s: obj(s, not s.endswith(".hip")), srcs))
        tmp = lib + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-fno-gpu-sanitize", "-shared-libsan",
              *SAN_LINK[kind], "-Wl,-soname,libemqx_tm.so", "-o", tmp, *objs, "-lpthread"])
        os.replace(tmp, lib)
        _stamp(lib, deps, kind + ARCH)
    mock = os.path.join(ROOT, "tests", "nif_mock")
    nsrcs = [os.path.join(CSRC, "nif", "emqx_tm_nif.c"), os.path.join(mock, "mock_erts.c")]
    nif = os.path.join(out_dir, "libemqx_nif_mock.so")
    ndeps = nsrcs + [os.path.join(mock, "erl_nif.h"), lib, os.path.join(ROOT, "include", "emqx_tm.h")]
    if force or _stale(nif, ndeps, kind):
        _run([os.path.join(LLVM_BIN, "clang"), "-O1", "-g", "-fno-omit-frame-pointer", "-std=gnu11", "-fPIC",
              "-shared", "-Wall", "-Wextra", "-Werror", *SAN_LINK[kind], "-shared-libsan",
              "-I" + mock, "-I" + os.path.join(ROOT, "include"), "-o", nif, *nsrcs,
              "-L" + out_dir, "-lemqx_tm", "-Wl,-rpath,$ORIGIN", "-lpthread"])
        _stamp(nif, ndeps, kind)
    return out_dir


def build_variant(name, defines):
    """A/B builds (dev): libemqx_tm with extra -D defines into
    emqx_amd/variants/libemqx_tm_<name>.so, loaded with EMQX_TM_LIB=<path>."""
    out_dir = os.path.join(HERE, "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"libemqx_tm_{name}.so")
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
          "-Wl,-soname,libemqx_tm.so", *defines, "-o", out]
         + [os.path.join(CSRC, f) for f in TM_SOURCES] + ["-lpthread"])
    return out


if __name__ == "__main__":
    if "--variant" in sys.argv:   # python -m emqx_amd.build --variant NAME -DFOO=1 ...
        i = sys.argv.index("--variant")
        build_variant(sys.argv[i + 1], [a for a in sys.argv[i + 2:] if a.startswith("-D")])
    else:
        build_all(force="--force" in sys.argv)
