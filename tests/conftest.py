"""Test configuration.

Markers:
  gpu  — needs an MI355X (runs the HIP engine).  `pytest -m "not gpu"` runs the CPU suite
         (oracle vs golden vectors, host logic, ABI surface); `pytest -m gpu` runs parity tests.

GPU tests that launch child processes (the C++ API harness, multi-rank runs) are ordered first:
a process that has initialised the GPU must not fork+exec afterwards (pool rule).
"""
import os
import resource
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-quantum-simulator_amd")
ORACLE = os.path.join(ROOT, "oracle")
# No core files: a process that aborts should fail fast, not spend minutes dumping GPU mappings.
resource.setrlimit(resource.RLIMIT_CORE, (0, 0))
for p in (ROOT, PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)
# Hermetic runs: no on-disk cache of kernels / layout decisions from earlier processes
# (csrc/hip/cache.hip); tests/test_cache_gpu.py turns it on for its own child processes.
os.environ.setdefault("QSIM_CACHE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (HIP engine)")
    config.addinivalue_line("markers", "subprocess: launches child processes (ordered first)")


def pytest_collection_modifyitems(config, items):
    first = [i for i in items if i.get_closest_marker("subprocess")]
    rest = [i for i in items if not i.get_closest_marker("subprocess")]
    items[:] = first + rest


@pytest.fixture(autouse=True)
def _shipped_policy():
    """Every test starts from, and leaves, the engine's shipped planning defaults (a test that
    lowers a threshold must not make later tests run non-default paths)."""
    yield
    if "qsim_amd" in sys.modules:
        from qsim_amd.plan import restore_defaults
        restore_defaults()


@pytest.fixture(scope="session")
def qsim():
    import qsim_amd
    return qsim_amd


@pytest.fixture(scope="session")
def oracle():
    import numpy_oracle
    return numpy_oracle


@pytest.fixture(scope="session")
def gpu_ready(qsim):
    n = qsim.device_count()
    assert n >= 1, "gpu-marked test needs a visible AMD GPU (no CPU fallback exists)"
    return n
