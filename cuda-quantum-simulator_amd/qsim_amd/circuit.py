"""Circuit IR mirroring the reference C++ API (include/Circuit.hpp:42-144, src/Circuit.cpp).

Exceptions follow the reference's classes through their Python analogues:
std::invalid_argument -> ValueError, std::out_of_range -> IndexError.
The random factories call the C++ implementation in libqsim.so so that gate lists are exactly
the libstdc++ std::mt19937 / uniform_*_distribution streams of src/Circuit.cpp:252-282.
"""
from __future__ import annotations

import ctypes
import enum
import math
from typing import Iterable, List, Sequence

from . import _lib

MIN_QUBITS = 1
MAX_QUBITS = 30  # reference include/Constants.hpp:68


class GateType(enum.IntEnum):
    X = 0
    Y = 1
    Z = 2
    H = 3
    S = 4
    T = 5
    Sdag = 6
    Tdag = 7
    Rx = 8
    Ry = 9
    Rz = 10
    CNOT = 11
    CZ = 12
    CRY = 13
    CRZ = 14
    SWAP = 15
    Toffoli = 16


PARAMETRIC = {GateType.Rx, GateType.Ry, GateType.Rz, GateType.CRY, GateType.CRZ}
ARITY = {t: (1 if t <= GateType.Rz else 2 if t <= GateType.SWAP else 3) for t in GateType}


class GateOp:
    __slots__ = ("type", "qubits", "parameter")

    def __init__(self, type: GateType, qubits: Sequence[int], parameter: float = 0.0):
        self.type = GateType(type)
        self.qubits = list(qubits)
        self.parameter = float(parameter)

    def __repr__(self) -> str:
        return f"GateOp({self.type.name}, {self.qubits}, {self.parameter})"

    def __eq__(self, other) -> bool:
        return (isinstance(other, GateOp) and self.type == other.type
                and self.qubits == other.qubits and self.parameter == other.parameter)


def is_valid_qubit_count(n: int) -> bool:
    return MIN_QUBITS <= n <= MAX_QUBITS


class Circuit:
    def __init__(self, num_qubits: int):
        if not is_valid_qubit_count(num_qubits):
            raise ValueError(f"Number of qubits must be between {MIN_QUBITS} and {MAX_QUBITS}")
        self._n = int(num_qubits)
        self._gates: List[GateOp] = []
        self._abi = None  # cached to_abi() result, dropped by every mutation

    # -- construction (src/Circuit.cpp:26-55 validation)
    def _add(self, t: GateType, qubits: Sequence[int], param: float = 0.0) -> "Circuit":
        for q in qubits:
            if not (0 <= q < self._n):
                raise IndexError(f"Qubit index {q} out of range [0, {self._n - 1}]")
        if len(set(qubits)) != len(qubits):
            raise ValueError("Two-qubit gate requires distinct qubits" if len(qubits) == 2
                             else "Three-qubit gate requires three distinct qubits")
        if t in PARAMETRIC and not math.isfinite(param):
            raise ValueError("Rotation angle must be a finite number")
        self._gates.append(GateOp(t, qubits, param))
        self._abi = None
        return self

    def x(self, q): return self._add(GateType.X, [q])
    def y(self, q): return self._add(GateType.Y, [q])
    def z(self, q): return self._add(GateType.Z, [q])
    def h(self, q): return self._add(GateType.H, [q])
    def s(self, q): return self._add(GateType.S, [q])
    def t(self, q): return self._add(GateType.T, [q])
    def sdag(self, q): return self._add(GateType.Sdag, [q])
    def tdag(self, q): return self._add(GateType.Tdag, [q])
    def rx(self, q, th): return self._add(GateType.Rx, [q], th)
    def ry(self, q, th): return self._add(GateType.Ry, [q], th)
    def rz(self, q, th): return self._add(GateType.Rz, [q], th)
    def cnot(self, c, t): return self._add(GateType.CNOT, [c, t])
    cx = cnot
    def cz(self, c, t): return self._add(GateType.CZ, [c, t])
    def cry(self, c, t, th): return self._add(GateType.CRY, [c, t], th)
    def crz(self, c, t, th): return self._add(GateType.CRZ, [c, t], th)
    def swap(self, a, b): return self._add(GateType.SWAP, [a, b])
    def toffoli(self, c1, c2, t): return self._add(GateType.Toffoli, [c1, c2, t])
    ccx = toffoli

    def append(self, op: GateOp) -> "Circuit":
        return self._add(op.type, op.qubits, op.parameter)

    def extend(self, other: "Circuit") -> "Circuit":
        """Append every gate of `other` (same qubit count) in order."""
        if other.getNumQubits() != self._n:
            raise ValueError("Circuit qubit count doesn't match")
        self._gates.extend(GateOp(g.type, g.qubits, g.parameter) for g in other._gates)
        self._abi = None
        return self

    # -- access
    def getNumQubits(self) -> int: return self._n
    num_qubits = property(getNumQubits)
    def getGates(self) -> List[GateOp]:
        """Copies of the gate list's entries (mutating them does not change the circuit)."""
        return [GateOp(g.type, g.qubits, g.parameter) for g in self._gates]
    gates = property(getGates)
    def getGateCount(self) -> int: return len(self._gates)
    def clear(self) -> None:
        self._gates.clear()
        self._abi = None

    def getDepth(self) -> int:
        level = [0] * self._n
        depth = 0
        for g in self._gates:
            lv = max(level[q] for q in g.qubits)
            for q in g.qubits:
                level[q] = lv + 1
            depth = max(depth, lv + 1)
        return depth

    def toString(self) -> str:
        lines = [f"Circuit({self._n} qubits, {len(self._gates)} gates):"]
        for i, g in enumerate(self._gates):
            args = ", ".join(str(q) for q in g.qubits)
            if g.type in PARAMETRIC:
                args += f", {g.parameter:g}"
            lines.append(f"  {i}: {g.type.name}({args})")
        return "\n".join(lines) + "\n"

    __str__ = toString

    # -- C ABI
    def to_abi(self):
        """(qsim_gate array, count).  Cached until the circuit changes: re-running one circuit
        (a benchmark loop, trajectories) does not rebuild it (~65 us for 100 gates)."""
        if self._abi is not None and self._abi[1] == len(self._gates):
            return self._abi
        arr = (_lib.qsim_gate * max(1, len(self._gates)))()
        for i, g in enumerate(self._gates):
            arr[i].type = int(g.type)
            arr[i].nqubits = len(g.qubits)
            for j, q in enumerate(g.qubits):
                arr[i].qubits[j] = q
            arr[i].parameter = g.parameter
        self._abi = (arr, len(self._gates))
        return self._abi

    @classmethod
    def from_abi(cls, n: int, arr, count: int) -> "Circuit":
        c = cls(n)
        for i in range(count):
            g = arr[i]
            c._gates.append(GateOp(GateType(g.type), [g.qubits[j] for j in range(g.nqubits)],
                                   g.parameter))
        c._abi = None
        return c


def _factory(kind: int, n: int, depth: int = 0, seed: int = 42) -> Circuit:
    count = ctypes.c_size_t(0)
    _lib.check_circ(_lib.api.qsim_circuit_make(kind, n, depth, seed, None, 0, ctypes.byref(count)))
    arr = (_lib.qsim_gate * max(1, count.value))()
    _lib.check_circ(_lib.api.qsim_circuit_make(kind, n, depth, seed, arr, count.value,
                                               ctypes.byref(count)))
    return Circuit.from_abi(2 if kind == _lib.QSIM_CIRCUIT_BELL else n, arr, count.value)


def createBellCircuit() -> Circuit:
    return _factory(_lib.QSIM_CIRCUIT_BELL, 2)


def createGHZCircuit(n: int) -> Circuit:
    return _factory(_lib.QSIM_CIRCUIT_GHZ, n)


def createRandomCircuit(n: int, depth: int, seed: int = 42) -> Circuit:
    return _factory(_lib.QSIM_CIRCUIT_RANDOM, n, depth, seed)


def createRandomHCCircuit(n: int, depth: int, seed: int = 42) -> Circuit:
    return _factory(_lib.QSIM_CIRCUIT_RANDOM_HC, n, depth, seed)


def createScalingBenchmarkCircuit(n: int) -> Circuit:
    return _factory(_lib.QSIM_CIRCUIT_SCALING, n)
