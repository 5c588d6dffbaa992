"""Sanitizer builds of the host code (ASan/UBSan for the host
C++, TSan for the concurrent NIF / submit queue).  The engine library and
the NIF shim are rebuilt with clang's -fsanitize (host code only,
emqx_amd/build.py build_sanitized) and tests/sanitize_worker.py drives the
concurrent paths -- the parallel churn at 8 workers, the lingering workers,
concurrent per-publish callers, the NIF with concurrent writers and engines
dropped under load -- in a child process with the sanitizer runtime
preloaded.  Any report fails the test (halt_on_error)."""

import os
import subprocess
import sys

import pytest

from emqx_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: ThreadSanitizer",
           "ERROR: LeakSanitizer", "SUMMARY: UndefinedBehaviorSanitizer")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_sanitize_host_concurrency(kind):
    rt = B.san_runtime(kind)
    if rt is None or not os.path.exists(B.HIPCC):
        pytest.skip("clang sanitizer runtime or hipcc not available")
    out_dir = B.build_sanitized(kind)
    env = dict(os.environ)
    env.update({
        "EMQX_SANITIZER": kind,
        "LD_PRELOAD": rt,
        "EMQX_TM_LIB": os.path.join(out_dir, "libemqx_tm.so"),
        "EMQX_NIF_MOCK_LIB": os.path.join(out_dir, "libemqx_nif_mock.so"),
        # the interpreter is not instrumented: its allocations at exit are not ours
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1",
    })
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_worker.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=800)
    reports = [line for line in p.stderr.splitlines() if any(r in line for r in REPORTS)]
    assert p.returncode == 0 and not reports and "SANITIZE OK" in p.stdout, (
        p.returncode, reports[:5], p.stdout[-2000:], p.stderr[-4000:])
    assert f"instrumented: {kind}" in p.stdout
