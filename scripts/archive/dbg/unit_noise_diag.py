"""Diagnose k_noise_units vs per-channel flips: same circuit/seed under both paths."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q


def run(n, B, qubits, p, unit, gates):
    os.environ["QSIM_NOISE_UNIT_MIN"] = "1" if unit else str(1 << 40)
    nm = q.NoiseModel()
    nm.addDepolarizing(qubits, p)
    c = q.Circuit(n)
    for k in range(gates):
        c.h(k % n)
    s = q.BatchedSimulator(n, B, nm, noise=q.BatchedNoise.Reference)
    s.setSeed(4)
    s.run(c)
    return np.stack([s.getStateVector(t) for t in range(B)])


for (n, B, qubits, p, gates) in [(6, 8, [0], 0.2, 1), (6, 8, [0, 1], 0.2, 1), (6, 8, list(range(6)), 0.2, 1),
                                 (6, 8, list(range(6)), 0.2, 3), (12, 4, list(range(12)), 0.2, 2),
                                 (6, 8, [3], 0.9, 1), (6, 8, [3, 3], 0.9, 1)]:
    a = run(n, B, qubits, p, True, gates)
    b = run(n, B, qubits, p, False, gates)
    d = np.abs(a - b) > 1e-12
    print(n, B, qubits, p, gates, "mismatch", int(d.sum()), "traj", sorted(set(np.nonzero(d)[0].tolist())),
          "idx", np.nonzero(d)[1][:12].tolist(), flush=True)
