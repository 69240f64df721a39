import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
import qsim_amd as q
import numpy_oracle as orc
from qsim_amd.dist import DistributedSimulator, plan
n, world = int(sys.argv[1]), int(sys.argv[2])
for name, c in (("hc", q.createRandomHCCircuit(n, 100, 42)), ("rand", q.createRandomCircuit(n, 100, 5))):
    steps, _ = plan(c, world, 0)
    print(name, "plan", [(s["kind"][0], s.get("role"), s.get("pivot"), len(s.get("ops", [])), s.get("lpos")) for s in steps])
    ref = orc.run_cpu(n, orc.gates_of(c))
    for fused in (True, False):
        d = DistributedSimulator.virtual(n, world)
        d.run(c, fused=fused)
        got = d.getStateVector()
        print(" ", "fused" if fused else "pergate", "overlapped", d.overlappedRemaps(), "maxerr", float(np.max(np.abs(got - ref))))
