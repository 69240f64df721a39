"""Sampling index parity with the reference's sequential CDF ("make sampling index
parity exact or provably tie-only").

The reference builds `partial_sum` of the probabilities sequentially and takes `lower_bound` of
each uniform (src/StateVector.cu:316-342, src/Simulator.cu:164-185, src/NoiseModel.cu:938-957).
The device computes the CDF with compensated chunk prefixes (reduce.hip: sample_indices), i.e.
the exactly rounded CDF up to a few ulps.  The two can only disagree where the uniform u lies
between the sequentially rounded CDF and the exact CDF at a step.  Every test below proves that
for EACH mismatching shot: with k the step between the two indices, u lies within
[min(C_seq[k], C_exact[k]) - 4 ulp, max(C_seq[k], C_exact[k]) + 4 ulp], C_exact computed with
math.fsum (exactly rounded).  Any other mismatch (an off-by-one in the search) fails.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _assert_tie_only(probs, u, got, exp):
    seq = np.add.accumulate(probs)  # sequential left-to-right, == std::partial_sum
    bad = np.nonzero(got != exp)[0]
    for i in bad:
        a, b = int(min(got[i], exp[i])), int(max(got[i], exp[i]))
        # lower_bound semantics: every index in [a, b) has its CDF step straddling u
        assert b - a == 1 or np.all(probs[a + 1:b] == 0.0), \
            f"shot {i}: indices {got[i]} vs {exp[i]} are not adjacent steps"
        k = a
        exact = math.fsum(probs[:k + 1])
        lo, hi = min(seq[k], exact), max(seq[k], exact)
        tol = 4 * np.spacing(u[i])
        assert lo - tol <= u[i] <= hi + tol, \
            f"shot {i}: u={u[i]!r} is not between C_seq={seq[k]!r} and C_exact={exact!r} at {k}"
    return len(bad)


@pytest.mark.parametrize("n", [5, 12, 16, 20])
def test_state_sampling_matches_sequential_cdf(qsim, oracle, gpu_ready, n):
    c = qsim.createRandomCircuit(n, 80, n)
    sim = qsim.Simulator(n)
    sim.run(c)
    st = oracle.run_cpu(n, oracle.gates_of(c))
    probs = np.abs(st) ** 2
    rng = np.random.default_rng(1000 + n)
    u = rng.random(20000)
    seq = np.add.accumulate(probs)
    # shots aimed at CDF steps (within an ulp or two of a step), where rounding matters most
    steps = rng.integers(0, probs.size - 1, 2000)
    u = np.concatenate([u, np.nextafter(seq[steps], 0.0), seq[steps], np.nextafter(seq[steps], 2.0)])
    u = u[(u > 0) & (u < 1)]
    got = sim.state.sampleWith(u)
    exp = oracle.sample_cpu(n, st, u)
    _assert_tie_only(probs, u, got, exp)
    # uniform shots (not aimed at steps) essentially never land in such a gap
    assert np.count_nonzero(got[:20000] != exp[:20000]) <= 2


def test_sampling_past_the_end(qsim, gpu_ready):
    """u above the rounded total -> index 2^n, as lower_bound returns end() in the reference."""
    sim = qsim.Simulator(3)
    sim.run(qsim.createGHZCircuit(3))
    got = sim.state.sampleWith(np.array([0.25, 0.75, 1.0 - 1e-17, 1.5]))
    assert list(got[:2]) == [0, 7] and got[3] == 8


@pytest.mark.parametrize("n,B", [(6, 64), (12, 32)])
def test_batched_sampling_matches_sequential_cdf(qsim, gpu_ready, n, B):
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.05)
    b = qsim.BatchedSimulator(n, B, nm)
    b.setSeed(3)
    b.run(qsim.createRandomCircuit(n, 60, 11))
    u = np.random.default_rng(5).random((B, 500))
    got = b.sampleWith(u)
    assert got.shape == (B, 500)
    for t in range(B):
        probs = b.getProbabilities(t)
        exp = np.searchsorted(np.add.accumulate(probs), u[t], side="left")
        _assert_tie_only(probs, u[t], got[t], exp)


def test_batched_sample_and_histogram_agree(qsim, gpu_ready):
    n, B, shots = 4, 16, 300
    c = qsim.Circuit(n)
    c.h(0).h(1).cnot(1, 2).ry(3, 0.7)
    out = []
    for _ in range(2):
        b = qsim.BatchedSimulator(n, B)
        b.setSeed(9)
        b.run(c)
        out.append(b)
    s = out[0].sample(shots)
    assert s.shape == (shots, B)
    h = out[1].getHistogram(shots)  # same seed -> same uniforms, same draw order
    np.testing.assert_array_equal(h, np.bincount(s.ravel(), minlength=1 << n))
    assert h.sum() == shots * B
    assert out[0].sample(0).shape == (0, B)
