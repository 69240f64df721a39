"""GPU: the large-n paths pinned against the ORACLE itself, not only HIP vs HIP.

Every check above 24 qubits used to compare the fused engine with RunMode::PerGate, and PerGate
was oracle-pinned only up to 16 qubits; the far-partner slice modes (targets 20-25 from 24 qubits)
and 16-byte offsets past 2^32 (28 qubits and up) run only at these sizes.  Here the oracle
(oracle/cpu_simulator.hpp, the reference CPUSimulator restatement) runs the same circuit on the
host, its gate loops split over threads (qsim_oracle_run_mt: bit-identical to the one-thread
oracle, tests/test_oracle.py), and the result is uploaded into a second device state and compared
on the device per real/imag component at 1e-12 (reference tests/test_gpu_cpu_equivalence.cu:26;
north_star's |amp|^2 < 1e-10 follows).

  * 28 qubits, BASELINE config 3 itself: createRandomHCCircuit(28, 100, 42) through the bench's
    path (inline compilation, calibrated first run, relabeled / relayout plan, specialised kernels).
  * 26 qubits, RunMode::PerGate: Ry(random) on every qubit, then H(t) and CNOT(t, t+1 mod 26) on
    every target t — k_m1_lane (t < 6), k_m1_slice, and the far-target mode-2 slice kernel
    (targets 20-25) each against the oracle.
  * 30 qubits, the headline W-HC seed 42 (16 GiB): the bench's exact line against the oracle.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get("QSIM_TEST_ORACLE_THREADS", "16"))  # (the GPU box's CPU share)


@pytest.fixture
def jit2(qsim):
    from qsim_amd.plan import set_jit
    set_jit(2, -1)
    yield


def _device_diff(qsim, sim_state, n, want):
    """max per-component |got - want| on the device: `want` uploaded into a second state."""
    ref = qsim.StateVector(n)
    try:
        ref.fromHost(want)
        return sim_state.maxAbsDiff(ref)
    finally:
        ref.close()


@pytest.mark.timeout(400)
def test_config3_28q_fused_bench_path_equals_oracle(qsim, oracle, gpu_ready, jit2):
    n = 28
    c = qsim.createRandomHCCircuit(n, 100, 42)
    sim = qsim.Simulator(n)
    sim.run(c)  # first run: layout + height calibration, then the chosen plan
    info = sim.state.layoutInfo()
    assert info["calibrated"], info
    want = oracle.run_cpu_mt(n, oracle.gates_of(c), threads=THREADS)
    err = _device_diff(qsim, sim.state, n, want)
    assert err < 1e-12, err
    # the second run starts from the layout the first one ends in (the bench's timed steady state)
    sim.run(c)
    want = oracle.run_cpu_mt(n, oracle.gates_of(c), state=want, threads=THREADS)
    err = _device_diff(qsim, sim.state, n, want)
    assert err < 1e-12, err
    sim.state.close()


@pytest.mark.timeout(400)
def test_per_gate_26q_every_target_equals_oracle(qsim, oracle, gpu_ready):
    n = 26
    rng = np.random.default_rng(26)
    c = qsim.Circuit(n)
    for q in range(n):
        c.ry(q, float(rng.uniform(0.2, 2.9)))
    for t in range(n):
        c.h(t)
        c.cnot(t, (t + 1) % n)
    for t in (0, 5, 6, 13, 19, 20, 22, 25):  # Rz / X on lane, slice and far-partner targets
        c.rz(t, float(rng.uniform(0, 6.2)))
        c.x(t)
    sim = qsim.Simulator(n, mode=qsim.RunMode.PerGate)
    sim.run(c)
    want = oracle.run_cpu_mt(n, oracle.gates_of(c), threads=THREADS)
    err = _device_diff(qsim, sim.state, n, want)
    assert err < 1e-12, err
    sim.state.close()


@pytest.mark.timeout(600)
def test_headline_30q_equals_oracle(qsim, oracle, gpu_ready, jit2):
    n = 30
    c = qsim.createRandomHCCircuit(n, 100, 42)
    sim = qsim.Simulator(n)
    sim.run(c)
    sim.run(c)  # the bench's steady state: the second run of the circuit
    info = sim.state.layoutInfo()
    assert info["calibrated"] and info["relabeled"], info
    g = oracle.gates_of(c)
    want = oracle.run_cpu_mt(n, g + g, threads=THREADS)
    err = _device_diff(qsim, sim.state, n, want)
    del want
    assert err < 1e-12, err
    sim.state.close()
