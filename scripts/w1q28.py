"""W-1Q at 28 qubits alone (bench.py's roofline_1q28: 100 unfused H gates on targets i % 28,
one kernel per gate) — the command the PMC summary profiles/pmc_1q_28q.json is collected on."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import bench  # noqa: E402
import qsim_amd as q  # noqa: E402

print(json.dumps(bench.roofline_1q28(q, steps=int(os.environ.get("STEPS", 2)))))
