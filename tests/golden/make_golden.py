"""Generate tests/golden/*.json.

kat_reference.json — known-answer vectors TRANSCRIBED from the reference's own test files (the
inputs are the circuits those tests build, the expectations are the values those tests assert;
each entry cites file:line in rylanmalarchick/cuda-quantum-simulator).  These pin the oracle and
the HIP path without executing the reference (execution was denied).

random_circuits.json — gate lists of the reference factory createRandomCircuit(n, depth, seed)
for the seeds used by tests/test_gpu_cpu_equivalence.cu:227-275, produced by this repo's C++
factory (libqsim.so, libstdc++ mt19937 draw order of src/Circuit.cpp:252-282), together with the
final state computed by the oracle restatement; they freeze the factory stream and the oracle
output so a drift in either shows up as a fixture failure.

Run:  python tests/golden/make_golden.py   (needs the built libqsim.so and oracle library)
"""
from __future__ import annotations

import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

R = 0.7071067811865476
PI = math.pi
X, Y, Z, H, S, T, SDG, TDG, RX, RY, RZ, CNOT, CZ, CRY, CRZ, SWAP, CCX = range(17)


def g(t, *qs, p=0.0):
    return [t, list(qs), p]


def basis(n, idx):
    v = [[0.0, 0.0] for _ in range(1 << n)]
    v[idx] = [1.0, 0.0]
    return v


KATS = [
    # tests/test_gates.cu
    dict(name="XGate", src="tests/test_gates.cu:39-48", n=1, gates=[g(X, 0)], state=[[0, 0], [1, 0]]),
    dict(name="HGate", src="tests/test_gates.cu:50-59", n=1, gates=[g(H, 0)], state=[[R, 0], [R, 0]]),
    dict(name="HH_Identity", src="tests/test_gates.cu:61-70", n=1, gates=[g(H, 0), g(H, 0)], state=[[1, 0], [0, 0]]),
    dict(name="ZGate", src="tests/test_gates.cu:72-84", n=1, gates=[g(H, 0), g(Z, 0)], state=[[R, 0], [-R, 0]]),
    dict(name="YGate", src="tests/test_gates.cu:86-95", n=1, gates=[g(Y, 0)], state=[[0, 0], [0, 1]]),
    dict(name="SGate", src="tests/test_gates.cu:97-106", n=1, gates=[g(X, 0), g(S, 0)], state=[[0, 0], [0, 1]]),
    dict(name="TGate", src="tests/test_gates.cu:108-116", n=1, gates=[g(X, 0), g(T, 0)], state=[[0, 0], [R, R]]),
    dict(name="RzGate", src="tests/test_gates.cu:118-128", n=1, gates=[g(H, 0), g(RZ, 0, p=PI)], probs={"0": 0.5, "1": 0.5}),
    dict(name="RxGate", src="tests/test_gates.cu:130-140", n=1, gates=[g(RX, 0, p=PI)], abs={"0": 0.0, "1": 1.0}),
    dict(name="RyGate", src="tests/test_gates.cu:142-152", n=1, gates=[g(RY, 0, p=PI)], abs={"0": 0.0, "1": 1.0}),
    dict(name="CNOT_Control0", src="tests/test_gates.cu:158-168", n=2, gates=[g(CNOT, 0, 1)], state=basis(2, 0)),
    dict(name="CNOT_Control1", src="tests/test_gates.cu:170-181", n=2, gates=[g(X, 0), g(CNOT, 0, 1)], state=basis(2, 3)),
    dict(name="BellState", src="tests/test_gates.cu:183-195", n=2, gates=[g(H, 0), g(CNOT, 0, 1)],
         state=[[R, 0], [0, 0], [0, 0], [R, 0]]),
    dict(name="CZGate", src="tests/test_gates.cu:197-206", n=2, gates=[g(X, 0), g(X, 1), g(CZ, 0, 1)],
         state=[[0, 0], [0, 0], [0, 0], [-1, 0]]),
    dict(name="SWAPGate", src="tests/test_gates.cu:208-219", n=2, gates=[g(X, 0), g(SWAP, 0, 1)], state=basis(2, 2)),
    dict(name="GHZState", src="tests/test_gates.cu:225-238", n=4,
         gates=[g(H, 0), g(CNOT, 0, 1), g(CNOT, 1, 2), g(CNOT, 2, 3)],
         probs={str(i): (0.5 if i in (0, 15) else 0.0) for i in range(16)}),
    dict(name="HadamardAllQubits", src="tests/test_gates.cu:240-252", n=4, gates=[g(H, q) for q in range(4)],
         probs={str(i): 1.0 / 16.0 for i in range(16)}),
    dict(name="Toffoli_BothControlsOn", src="tests/test_gates.cu:258-273", n=3,
         gates=[g(X, 0), g(X, 1), g(CCX, 0, 1, 2)], state=basis(3, 7)),
    dict(name="Toffoli_OneControlOff", src="tests/test_gates.cu:275-287", n=3, gates=[g(X, 0), g(CCX, 0, 1, 2)],
         state=basis(3, 1)),
    dict(name="Toffoli_NoControlsOn", src="tests/test_gates.cu:289-299", n=3, gates=[g(CCX, 0, 1, 2)], state=basis(3, 0)),
    dict(name="Toffoli_SelfInverse", src="tests/test_gates.cu:301-316", n=3,
         gates=[g(X, 0), g(X, 1), g(CCX, 0, 1, 2), g(CCX, 0, 1, 2)], state=basis(3, 3)),
    dict(name="CRY_ControlOff", src="tests/test_gates.cu:318-327", n=2, gates=[g(CRY, 0, 1, p=PI)], state=basis(2, 0)),
    dict(name="CRY_ControlOn", src="tests/test_gates.cu:329-341", n=2, gates=[g(X, 0), g(CRY, 0, 1, p=PI)],
         abs={"3": 1.0}),
    dict(name="CRY_Superposition", src="tests/test_gates.cu:343-358", n=2, gates=[g(X, 0), g(CRY, 0, 1, p=PI / 2)],
         probs_sum={"indices": [1, 3], "value": 1.0}, probs_gt={"1": 0.1, "3": 0.1}),
    dict(name="CRZ_ControlOff", src="tests/test_gates.cu:360-371", n=2, gates=[g(H, 1), g(CRZ, 0, 1, p=PI)],
         state=[[R, 0], [0, 0], [R, 0], [0, 0]]),
    dict(name="CRZ_ControlOn", src="tests/test_gates.cu:373-386", n=2, gates=[g(X, 0), g(H, 1), g(CRZ, 0, 1, p=PI)],
         probs={"1": 0.5, "3": 0.5}),
    # tests/test_boundary.cu
    dict(name="SingleQubit_HTH", src="tests/test_boundary.cu:30-47", n=1, gates=[g(H, 0), g(T, 0), g(H, 0)],
         probs_sum={"indices": [0, 1], "value": 1.0}, tol=1e-12),
    dict(name="MediumQubitCount_16", src="tests/test_boundary.cu:63-82", n=16, gates=[g(H, q) for q in range(16)],
         probs={str(i): 1.0 / 65536.0 for i in range(16)}, tol=1e-12),
    dict(name="LargerQubitCount_20_GHZ", src="tests/test_boundary.cu:84-104", n=20,
         gates=[g(H, 0)] + [g(CNOT, q, q + 1) for q in range(19)],
         probs={"0": 0.5, str((1 << 20) - 1): 0.5, "1": 0.0, "1000": 0.0, "500000": 0.0}, tol=1e-12),
    dict(name="Normalization_AfterGates", src="tests/test_boundary.cu:176-195", n=6,
         gates=[g(H, q) for q in range(6)] + [g(CNOT, 0, 1), g(CNOT, 2, 3), g(CNOT, 4, 5), g(CZ, 0, 2),
                                              g(CZ, 1, 3), g(RX, 0, p=1.23), g(RY, 2, p=0.45), g(RZ, 4, p=2.34)],
         probs_sum={"indices": "all", "value": 1.0}, tol=1e-12),
]


def main():
    out = {"description": __doc__.split("\n\n")[1], "tolerance_default": 1e-10, "cases": KATS}
    with open(os.path.join(HERE, "kat_reference.json"), "w") as f:
        json.dump(out, f, indent=1)

    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import qsim_amd
    import numpy_oracle as orc

    cases = []
    specs = [(3 + s % 3, 10 + s % 20, s) for s in range(20)]      # RandomCircuits_Small
    specs += [(8 + s % 4, 50 + s % 50, s) for s in range(10)]     # RandomCircuits_Medium
    specs += [(4, 500, s) for s in range(5)]                      # RandomCircuits_Deep
    for n, d, s in specs:
        c = qsim_amd.createRandomCircuit(n, d, s)
        gates = orc.gates_of(c)
        st = orc.run_cpu(n, gates)
        assert np.allclose(st, orc.run_numpy(n, gates), atol=1e-12)
        cases.append({"n": n, "depth": d, "seed": s, "gates": [[t, q, p] for t, q, p in gates],
                      "state": [[float(z.real), float(z.imag)] for z in st] if n <= 8 else None,
                      "state_sha_probs": [float(x) for x in np.abs(st[:16]) ** 2]})
    with open(os.path.join(HERE, "random_circuits.json"), "w") as f:
        json.dump({"source": "tests/test_gpu_cpu_equivalence.cu:227-275 seeds; "
                             "createRandomCircuit src/Circuit.cpp:252-282", "cases": cases}, f)
    print("wrote", len(KATS), "KATs and", len(cases), "random-circuit fixtures")


if __name__ == "__main__":
    main()
