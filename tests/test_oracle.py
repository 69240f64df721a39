"""CPU: pin the parity oracle.

* Both oracle implementations (C++ CPUSimulator restatement, numpy tensordot) reproduce every
  known-answer vector transcribed from the reference's tests (tests/golden/kat_reference.json).
* They agree with each other on the reference's random-circuit suites (test_gpu_cpu_equivalence
  seeds) and with the frozen fixtures (tests/golden/random_circuits.json).
* Mode::StrictCpu reproduces the reference CPUSimulator's CRY/CRZ/Toffoli no-ops.
"""
import json
import math
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def check_case(case, state, tol_default):
    tol = case.get("tol", tol_default)
    probs = np.abs(state) ** 2
    if "state" in case:
        exp = np.array([complex(r, i) for r, i in case["state"]])
        assert np.max(np.abs(state.real - exp.real)) <= tol
        assert np.max(np.abs(state.imag - exp.imag)) <= tol
    if "probs" in case:
        for k, v in case["probs"].items():
            assert abs(probs[int(k)] - v) <= tol, (case["name"], k)
    if "abs" in case:
        for k, v in case["abs"].items():
            assert abs(abs(state[int(k)]) - v) <= tol, (case["name"], k)
    if "probs_sum" in case:
        idx = case["probs_sum"]["indices"]
        s = probs.sum() if idx == "all" else sum(probs[i] for i in idx)
        assert abs(s - case["probs_sum"]["value"]) <= tol
    if "probs_gt" in case:
        for k, v in case["probs_gt"].items():
            assert probs[int(k)] > v


KATS = load("kat_reference.json")


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_cpp_oracle_matches_reference_kats(case, oracle):
    st = oracle.run_cpu(case["n"], [tuple(g) for g in case["gates"]])
    check_case(case, st, KATS["tolerance_default"])


@pytest.mark.parametrize("case", KATS["cases"], ids=[c["name"] for c in KATS["cases"]])
def test_numpy_oracle_matches_reference_kats(case, oracle):
    if case["n"] > 16:
        pytest.skip("numpy tensordot oracle kept to n <= 16 for runtime")
    st = oracle.run_numpy(case["n"], [tuple(g) for g in case["gates"]])
    check_case(case, st, KATS["tolerance_default"])


def test_random_circuit_fixtures(oracle, qsim):
    data = load("random_circuits.json")
    for case in data["cases"]:
        c = qsim.createRandomCircuit(case["n"], case["depth"], case["seed"])
        gates = oracle.gates_of(c)
        # factory stream is frozen: same gate list as when the fixture was made
        assert [[t, q, p] for t, q, p in gates] == case["gates"]
        st = oracle.run_cpu(case["n"], gates)
        np.testing.assert_allclose(st, oracle.run_numpy(case["n"], gates), atol=1e-12, rtol=0)
        if case["state"] is not None:
            exp = np.array([complex(r, i) for r, i in case["state"]])
            assert np.max(np.abs(st - exp)) <= 1e-12
        np.testing.assert_allclose(np.abs(st[:16]) ** 2, case["state_sha_probs"], atol=1e-12)


def test_strict_cpu_mode_reproduces_reference_noops(oracle):
    # reference CPUSimulator ignores CRY/CRZ (default: break) and never dispatches Toffoli (F4)
    for g in [(13, [0, 1], 0.7), (14, [0, 1], 0.7), (16, [0, 1, 2], 0.0)]:
        gates = [(0, [0], 0.0), (0, [1], 0.0), (9, [2], 0.3), g]
        strict = oracle.run_cpu(3, gates, strict_cpu=True)
        base = oracle.run_cpu(3, gates[:-1])
        np.testing.assert_array_equal(strict, base)
        full = oracle.run_cpu(3, gates)
        assert np.max(np.abs(full - base)) > 1e-3


def test_all_gate_types_all_targets_against_numpy(oracle):
    rng = np.random.default_rng(7)
    n = 5
    psi = rng.normal(size=32) + 1j * rng.normal(size=32)
    psi /= np.linalg.norm(psi)
    for t in range(17):
        arity = 1 if t <= 10 else (2 if t <= 15 else 3)
        for _ in range(6):
            qs = list(rng.choice(n, size=arity, replace=False))
            g = (t, [int(q) for q in qs], float(rng.uniform(0, 2 * math.pi)))
            a = oracle.run_cpu(n, [g], state=psi)
            b = oracle.run_numpy(n, [g], state=psi)
            np.testing.assert_allclose(a, b, atol=1e-13, rtol=0)


def test_oracle_sampling_lower_bound(oracle):
    st = np.array([0.5 ** 0.5, 0, 0, 0.5 ** 0.5], complex)
    u = np.array([0.0, 0.25, 0.4999999, 0.5, 0.5000001, 0.99])
    out = oracle.sample_cpu(2, st, u)
    assert list(out) == [0, 0, 0, 0, 3, 3]


@pytest.mark.parametrize("threads", [2, 7, 16])
def test_threaded_oracle_is_bit_identical(oracle, threads):
    """qsim_oracle_run_mt (each gate's loop split over threads, used by the 26-30 qubit GPU parity
    tests) equals the single-threaded oracle bit for bit on every gate type, targets low and high."""
    n = 17
    rng = np.random.default_rng(threads)
    gates = []
    for _ in range(60):
        t = int(rng.integers(0, 17))
        ar = 1 if t <= 10 else (2 if t <= 15 else 3)
        qs = [int(x) for x in rng.choice(n, size=ar, replace=False)]
        gates.append((t, qs, float(rng.uniform(0, 2 * math.pi))))
    start = oracle.run_cpu(n, [(3, [q], 0.0) for q in range(n)])
    want = oracle.run_cpu(n, gates, state=start)
    got = oracle.run_cpu_mt(n, gates, state=start, threads=threads)
    assert np.array_equal(got, want)
