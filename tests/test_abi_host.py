"""CPU: the C-ABI boundary and host logic (no GPU compute calls).

* libqsim_hip.so / libqsim.so load and export every function include/*.h declares.
* Argument validation / error mapping of the ABI matches the reference's exception classes.
* The fused-pass planner only reorders gates on disjoint qubits: replaying the circuit in the
  planner's execution order on the oracle reproduces the original state.
* Circuit API semantics (src/Circuit.cpp): validation, depth, factories, toString.
"""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?\w+\s*\*?\s*(qsim_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_functions():
    names = declared_functions()
    assert "qsim_run" in names and "qsim_state_create" in names and "qsim_circuit_make" in names
    assert len(names) > 40


def test_every_declared_symbol_is_exported(qsim):
    from qsim_amd import _lib
    missing = [n for n in declared_functions()
               if not hasattr(_lib.hip, n) and not hasattr(_lib.api, n)]
    assert not missing, missing


def test_abi_version(qsim):
    from qsim_amd import _lib
    assert _lib.hip.qsim_abi_version() == 2


def test_state_create_validation_without_gpu(qsim):
    # qubit-count validation happens before any device call (StateVector.cu:135-141)
    for bad in (0, -1, 31, 40):
        with pytest.raises(ValueError):
            qsim.StateVector(bad)
        with pytest.raises(ValueError):
            qsim.Circuit(bad)


def test_circuit_validation_matches_reference(qsim):
    c = qsim.Circuit(4)
    for f in (lambda: c.h(-1), lambda: c.h(4), lambda: c.h(100), lambda: c.cnot(0, 4),
              lambda: c.cnot(-1, 0)):
        with pytest.raises(IndexError):
            f()
    for f in (lambda: c.cnot(0, 0), lambda: c.cz(2, 2), lambda: c.swap(1, 1),
              lambda: c.toffoli(1, 1, 2), lambda: c.rx(0, float("nan")),
              lambda: c.ry(0, float("inf"))):
        with pytest.raises(ValueError):
            f()
    assert c.getGateCount() == 0


def test_circuit_depth_and_string(qsim):
    c = qsim.Circuit(3)
    c.h(0).h(1).cnot(0, 1).h(2).toffoli(0, 1, 2).rz(2, 0.5)
    assert c.getDepth() == 4
    s = c.toString()
    assert s.startswith("Circuit(3 qubits, 6 gates):") and "Toffoli(0, 1, 2)" in s
    assert "Rz(2, 0.5)" in s
    assert qsim.Circuit(2).getDepth() == 0


def test_factories(qsim):
    b = qsim.createBellCircuit()
    assert [(g.type.name, g.qubits) for g in b.getGates()] == [("H", [0]), ("CNOT", [0, 1])]
    ghz = qsim.createGHZCircuit(5)
    assert ghz.getGateCount() == 5 and ghz.getGates()[-1].qubits == [3, 4]
    with pytest.raises(ValueError):
        qsim.createGHZCircuit(1)
    w = qsim.createScalingBenchmarkCircuit(10)
    assert w.getGateCount() == 120
    hc = qsim.createRandomHCCircuit(30, 100, 42)
    assert hc.getGateCount() == 100
    assert {g.type.name for g in hc.getGates()} == {"H", "CNOT"}
    r1 = qsim.createRandomCircuit(6, 40, 9)
    r2 = qsim.createRandomCircuit(6, 40, 9)
    assert r1.getGates() == r2.getGates()
    assert {g.type.name for g in r1.getGates()} <= {"H", "X", "CNOT", "Rz"}


def test_random_factory_on_one_qubit_uses_h_for_cnot(qsim):
    c = qsim.createRandomCircuit(1, 50, 3)
    assert all(g.type.name in ("H", "X", "Rz") for g in c.getGates())


@pytest.mark.parametrize("n,depth,seed,hmax", [(8, 60, 1, 6), (12, 200, 2, 6), (20, 100, 42, 6),
                                               (20, 100, 7, 3), (30, 100, 42, 6), (9, 80, 5, 0),
                                               (5, 40, 3, 6), (14, 150, 11, 4),
                                               (14, 150, 11, 7), (20, 100, 1, 7), (30, 100, 42, 7)])
def test_planner_reordering_preserves_circuit(qsim, oracle, n, depth, seed, hmax):
    from qsim_amd.plan import plan_fused
    c = qsim.createRandomCircuit(n, depth, seed) if n <= 14 else qsim.createRandomHCCircuit(n, depth, seed)
    order, pass_of, npass = plan_fused(c, hmax)
    assert sorted(order.tolist()) == list(range(c.getGateCount()))
    gates = c.getGates()
    # commutation check: any two gates whose relative order changed act on disjoint qubits, or
    # share only qubits that are controls of both (a tile-constant control is read, never written,
    # so stages may order such gates either way)
    pos = {int(g): i for i, g in enumerate(order)}
    swap = int(qsim.GateType.SWAP)

    def targets(g):
        return set(g.qubits) if int(g.type) == swap else {g.qubits[-1]}
    for i in range(len(gates)):
        for j in range(i + 1, len(gates)):
            if pos[i] > pos[j]:
                shared = set(gates[i].qubits) & set(gates[j].qubits)
                assert not shared & (targets(gates[i]) | targets(gates[j])), (i, j)
    # every pass fits one tile: qubits 0..r0-1 (the contiguous run) plus at most 6 + h - r0
    # others; r0 = 6 for small tiles, 4..6 (planner's choice) for staged ones (h >= 4).  Staged
    # tiles hold the gates' TARGETS (a control outside the tile is a tile constant,
    # qsim_set_tile_ctrl_out); small tiles every qubit.
    h = min(hmax, n - 6)
    runs = (4, 5, 6) if h >= 4 else (6,)
    swap = int(qsim.GateType.SWAP)
    for p in range(npass):
        qs = set()
        for k in np.nonzero(pass_of == p)[0]:
            g = gates[order[k]]
            if h >= 4:
                qs |= set(g.qubits) if int(g.type) == swap else {g.qubits[-1]}
            else:
                qs |= set(g.qubits)
        assert any(len({q for q in qs if q >= r0}) <= 6 + h - r0 for r0 in runs), (p, sorted(qs))
    if n <= 14:
        g = oracle.gates_of(c)
        np.testing.assert_allclose(oracle.run_cpu(n, [g[i] for i in order]), oracle.run_cpu(n, g),
                                   atol=1e-12, rtol=0)


def test_plan_pass_counts_for_bench_workload(qsim):
    from qsim_amd.plan import plan_fused
    # beam-searched pass sequences (QSIM_PLAN_BEAM): W-HC 100 gates in 5-6 HBM passes
    for n, most in ((20, 8), (28, 6), (30, 5)):
        _, _, npass = plan_fused(qsim.createRandomHCCircuit(n, 100, 42))
        assert npass <= most, (n, npass)


def test_noise_model_host_semantics(qsim):
    nm = qsim.NoiseModel()
    nm.addDepolarizing(0.01)              # global form: empty qubit list (F6)
    nm.addDepolarizing([0, 2], 0.1)
    nm.addDepolarizingAll(3, 0.2)
    ch = nm.getChannels()
    assert len(ch) == 1 + 2 + 3 and ch[0].qubits == [] and ch[1].qubits == [0]
    arr, cnt = nm.to_abi()
    assert cnt == 5  # the global channel contributes no per-qubit entry
