"""13-qubit tiles (qsim_set_tile_height(7): 128 KiB of LDS, one 512-thread workgroup per CU,
persistent software-pipelined hipRTC pass kernels) pinned to the oracle.

The same bench-path workloads as tests/test_bench_path_gpu.py — W-HC (seeds 42, 5) and W-REF at
20 and 22 qubits — run through `Simulator` in Fused mode with the specialised kernels (jit = 2)
and through the pass interpreter (jit = 0), and every amplitude is compared with the C++
CPUSimulator restatement at 1e-12 per component.  Batched noisy trajectories at h = 7 (Pauli
frames conjugating non-Clifford ops inside the 13-qubit passes) equal the per-gate execution.
"""
import numpy as np
import pytest

from test_batched_gpu import _mixed, _noise

pytestmark = pytest.mark.gpu


@pytest.fixture
def tile7(qsim):
    from qsim_amd.plan import set_jit, set_tile_height
    set_tile_height(7)
    yield set_jit
    set_tile_height(-1)
    set_jit(1, -1)


@pytest.mark.parametrize("rb7", [4, 3])
@pytest.mark.parametrize("n", [20, 22])
@pytest.mark.parametrize("jit", [2, 0])
def test_tile13_matches_oracle(qsim, oracle, gpu_ready, tile7, n, jit, rb7):
    """rb7 = 3: 13-qubit tiles with 8 amplitudes per thread (1024-thread workgroups) — the
    interpreter's k_fused_staged<7, ., ., 3> and generated kernels at that stage width."""
    from qsim_amd.plan import set_tile_rb7
    tile7(jit, -1)
    set_tile_rb7(rb7)
    try:
        _run_tile13(qsim, oracle, n, jit)
    finally:
        set_tile_rb7(-1)


def _run_tile13(qsim, oracle, n, jit):
    work = [(f"W-HC seed {s}", qsim.createRandomHCCircuit(n, 100, s)) for s in (42, 5)]
    work.append(("W-REF", qsim.createScalingBenchmarkCircuit(n)))
    for name, c in work:
        ref = oracle.run_cpu(n, oracle.gates_of(c))
        sim = qsim.Simulator(n, mode=qsim.RunMode.Fused)
        for rep in range(2):
            sim.reset()
            sim.run(c)
            got = sim.getStateVector()
            err = float(np.max(np.abs(np.concatenate([(got - ref).real, (got - ref).imag]))))
            assert err < 1e-12, f"{name} n={n} jit={jit} run {rep}: max component error {err}"
        passes, jit_passes = sim.state.lastRunInfo()
        assert passes >= 1 and (jit_passes >= 1) == (jit == 2)


def test_tile13_batched_frames_equal_per_gate(qsim, gpu_ready, tile7):
    tile7(2, -1)
    n, B, seed = 14, 8, 7
    c = _mixed(qsim, n, 60, seed)
    nm = _noise(qsim, n)
    fused, ref = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical), qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    fused.setSeed(seed)
    ref.setSeed(seed)
    for _ in range(2):
        fused.run(c)
        ref.run(c, per_gate=True)
    for t in range(B):
        np.testing.assert_allclose(fused.getStateVector(t), ref.getStateVector(t), atol=1e-12, rtol=0)
