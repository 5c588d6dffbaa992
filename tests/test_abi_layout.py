"""The ctypes mirrors in emqx_amd/_native.py against include/emqx_tm.h: a C
program built with gcc from the header prints every struct's size and each
mirrored field's offset, and they must equal ctypes' (a field added to the
header but not to the mirror, or in another place, shifts what Python reads)."""

import ctypes as C
import os
import shutil
import subprocess

import pytest

from emqx_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PAIRS = [("tm_config", N.Config), ("tm_trie_node", N.TrieNode), ("tm_result", N.Result),
         ("tm_result_packed", N.ResultPacked),
         ("tm_routes", N.Routes), ("tm_deliveries", N.Deliveries), ("tm_batch_stats", N.BatchStats),
         ("tm_engine_stats", N.EngineStats), ("tm_async_stats", N.AsyncStats),
         ("tm_sharded_stats", N.ShardedStats)]


@pytest.mark.skipif(not shutil.which("gcc"), reason="needs gcc")
def test_ctypes_mirrors_match_the_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "emqx_tm.h"', "int main(void) {"]
    for cname, py in PAIRS:
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        k1, k2, v = ln.split()
        got[(k1, k2)] = int(v)
    for cname, py in PAIRS:
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])
