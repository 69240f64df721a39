"""CPU: the host side of the layout-aware relabeling (qsim_plan_relabel, no GPU).

The permutation keeps the contiguous run qubits (0..3, in every tile) in place, is a bijection,
and never predicts a slower layout; the layout model (csrc/hip/layout_cost.hpp, fitted by
scripts/fit_layout_cost.py to the probes in profiles/r02/layout/) ranks the measured tiles the
way the probes did."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _relabeled(qsim, c, perm):
    n = c.getNumQubits()
    c1 = qsim.Circuit(n)
    for g in c.getGates():
        c1.append(qsim.GateOp(g.type, [perm[x] for x in g.qubits], g.parameter))
    return c1


@pytest.mark.parametrize("n,seed", [(26, 42), (28, 42), (30, 42), (30, 7)])
def test_plan_relabel_is_a_valid_improving_permutation(qsim, n, seed):
    from qsim_amd.plan import plan_fused, plan_relabel
    c = qsim.createRandomHCCircuit(n, 100, seed)
    perm, before, after = plan_relabel(c)
    assert sorted(perm) == list(range(n))
    passes0, passes1 = plan_fused(c)[2], plan_fused(_relabeled(qsim, c, perm))[2]
    # never more passes; as many passes only with a cheaper predicted layout
    assert passes1 < passes0 or (passes1 == passes0 and (after < before or perm == list(range(n))))
    again = plan_relabel(c)
    assert again[0] == perm  # deterministic (fixed seeds)


def test_relabel_finds_fewer_passes_at_28_qubits(qsim):
    """W-HC 28q plans into 6 passes as labelled and into 5 under the chosen labels (every control
    a tile qubit); with tile-constant controls (the default) into 5 as labelled, and relabeling
    keeps that."""
    from qsim_amd.plan import plan_fused, plan_relabel, set_tile_ctrl_out
    c = qsim.createRandomHCCircuit(28, 100, 42)
    set_tile_ctrl_out(0)
    try:
        perm, _, _ = plan_relabel(c)
        assert plan_fused(c)[2] == 6 and plan_fused(_relabeled(qsim, c, perm))[2] == 5
    finally:
        set_tile_ctrl_out(1)
    perm, _, _ = plan_relabel(c)
    assert plan_fused(c)[2] == 5 and plan_fused(_relabeled(qsim, c, perm))[2] <= 5


def test_small_circuit_keeps_identity(qsim):
    from qsim_amd.plan import plan_relabel
    c = qsim.Circuit(12)
    for q in range(12):
        c.h(q)
    perm, before, after = plan_relabel(c)  # one pass over every qubit: nothing to gain
    assert perm == list(range(12)) and after == before


def test_layout_model_orders_the_w_hc_tiles_like_the_probes():
    """The five W-HC 30q pass tiles: the model's order of predicted cost agrees with the measured
    pass times at least on the extremes (fastest and slowest)."""
    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    rows = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "r02", "layout", "probe_families.jsonl"))]
    whc = [r for r in rows if r["kind"] == "whc"]
    assert len(whc) == 5
    import numpy as np
    text = open(os.path.join(ROOT, "cuda-quantum-simulator_amd", "csrc", "hip", "layout_cost.hpp")).read()
    import re
    base = float(re.search(r"kBase = ([-\d.]+)f", text).group(1))
    w1 = [float(x) for x in re.search(r"kW1\[kN\] = \{([^}]*)\}", text).group(1).replace("f", "").split(",")]
    block = text.split("kW2[kN][kN] = {")[1].split("};")[0]
    w2 = np.array([float(x) for x in re.findall(r"-?\d+\.\d+", block)]).reshape(30, 30)

    def cost(t):
        t = [q for q in t if q >= 4]
        return base + sum(w1[q] for q in t) + sum(w2[a][b] for i, a in enumerate(t) for b in t[i + 1:])

    pred = np.array([cost(r["tile"]) for r in whc])
    meas = np.array([r["ms_per_pass"] for r in whc])
    assert int(np.argmax(pred)) == int(np.argmax(meas))
    assert int(np.argmin(pred)) == int(np.argmin(meas))
