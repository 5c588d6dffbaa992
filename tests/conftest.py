import json
import os
import subprocess
import sys

import pytest

# One HIP runtime per process: torch bundles its own libamdhip64 /
# libhsa-runtime64 (ROCm 7.0), the engine links /opt/rocm's (7.2).  Loading
# torch after the engine maps a second HSA runtime and torch's GPU init fails
# ("No HIP GPUs are available"); importing torch first makes the
# engine bind to torch's already-loaded runtime.  GPU tests that exchange
# tensors with the engine rely on this, whatever subset of tests runs.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def native_built():
    """Build (or refresh) the in-tree native artefacts once per session."""
    from emqx_amd import build as B
    B.build_all()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    yield


def gpu_count() -> int:
    """HIP devices visible to this process (0 without a GPU)."""
    try:
        from emqx_amd import _native as N
        return int(N.lib().tm_device_count())
    except Exception:   # noqa: BLE001
        return 0


@pytest.fixture(params=["dev00", "dev01"])
def device_pair(request):
    """Two devices for the multi-device paths: [0, 0] (two replicas / shards on
    one GPU: always) and [0, 1] (two physical GPUs: skipped on a 1-GPU box)."""
    if request.param == "dev01":
        if gpu_count() < 2:
            pytest.skip("needs two HIP devices")
        return [0, 1]
    return [0, 0]


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def lb(s: str) -> bytes:
    """fixture strings are latin-1 views of raw bytes"""
    return s.encode("latin-1")


@pytest.fixture
def golden():
    return load_golden
