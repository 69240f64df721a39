"""GPU: the on-disk cache across processes (csrc/hip/cache.hip).  Two processes in turn run the same
circuit from |0..0> in bench.py's mode (inline compilation, calibrated first run at 26 qubits) with
one cache directory: the first writes the pass kernels' code objects and the layout decision, the
second loads them (no compile, no candidate timing) — and both end in the same state (probBitZero of
every qubit to 1e-12; the plans are the same, so the kernels and results are)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(env):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "first_run.py"), "26", "42"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.subprocess  # started before this process initialises the GPU (pool rule)
def test_second_process_loads_kernels_and_layout(tmp_path):
    env = dict(os.environ, QSIM_CACHE="1", QSIM_CACHE_DIR=str(tmp_path / "cache"))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    a = _run(env)
    b = _run(env)
    assert a["jit_stores"] >= 1 and a["layout_stores"] >= 1 and a["jit_hits"] == 0 and a["layout_hits"] == 0
    assert b["jit_hits"] >= 1 and b["layout_hits"] >= 1 and b["jit_stores"] == 0
    assert a["passes"] == b["passes"]
    assert max(abs(x - y) for x, y in zip(a["p0"], b["p0"])) < 1e-12
    off = _run(dict(env, QSIM_CACHE="0"))
    assert off["jit_hits"] == off["jit_stores"] == off["layout_hits"] == off["layout_stores"] == 0
