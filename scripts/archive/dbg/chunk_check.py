"""Checksum of the W-HC state (for comparing execution strategies across processes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
import numpy as np
import qsim_amd as q
from qsim_amd.plan import set_jit
n = int(sys.argv[1])
set_jit(2, -1)
c = q.createRandomHCCircuit(n, 100, 42)
sim = q.Simulator(n)
sim.run(c)
sim.run(c)
psi = sim.getStateVector()
w = np.cos(np.arange(psi.size) * 0.001)
print("checksum", n, os.environ.get("QSIM_CHUNK_QUBITS"), repr(complex(np.dot(w, psi))), repr(float(np.vdot(psi, psi).real)))
