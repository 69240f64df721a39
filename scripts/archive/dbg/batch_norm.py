import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
import numpy as np
import qsim_amd as qsim
for n, B, pg in ((12, 32, False), (12, 32, True), (10, 8, False), (13, 4, False)):
    nm = qsim.NoiseModel(); nm.addDepolarizingAll(n, 0.05)
    b = qsim.BatchedSimulator(n, B, nm); b.setSeed(3)
    b.run(qsim.createRandomCircuit(n, 60, 11), per_gate=pg)
    norms = [float(np.sum(b.getProbabilities(t))) for t in range(B)]
    print(n, B, pg, "norms before", min(norms), max(norms), flush=True)
    u = np.random.default_rng(5).random((B, 500))
    got = b.sampleWith(u)
    norms = [float(np.sum(b.getProbabilities(t))) for t in range(B)]
    print(n, B, pg, "norms after", min(norms), max(norms), got.min(), got.max(), flush=True)
