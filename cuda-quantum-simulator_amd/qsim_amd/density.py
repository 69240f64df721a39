"""DensityMatrix / DensityMatrixSimulator (reference include/DensityMatrix.cuh:63-224,
src/DensityMatrix.cu) over the C ABI (qsim_dm_*, include/qsim_hip.h).

rho of n qubits is a 2n-index-bit state of the HIP engine (rho[i][j] at i * 2^n + j, the
reference's row-major layout): gates run as U on the row bits and conj(U) on the column bits, noise
channels as short op sequences on (row bit, column bit) — all through the fused tile passes.
Exceptions follow the reference: ValueError ~ std::invalid_argument (bad qubit count, state size
mismatch), RuntimeError ~ std::runtime_error (CRY/CRZ/Toffoli, src/DensityMatrix.cu:264-266).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import _lib
from .circuit import Circuit, GateOp
from .simulator import NoiseModel, RunMode, StateVector

MAX_QUBITS = 15
_c = ctypes


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_c.c_void_p)


class DensityMatrix:
    def __init__(self, n_qubits: int, pure_state=None):
        if n_qubits < 1 or n_qubits > MAX_QUBITS:
            raise ValueError(f"Density matrix supports 1-{MAX_QUBITS} qubits")
        self._n = n_qubits
        self._sv = StateVector(2 * n_qubits)  # |0..0> = |0><0| (src/DensityMatrix.cu:72-79)
        if pure_state is not None:
            self.initFromPureState(pure_state)

    @property
    def state(self) -> StateVector:
        return self._sv

    def reset(self) -> None: self._sv.initializeZero()

    def initFromPureState(self, psi) -> None:
        a = np.ascontiguousarray(psi, dtype=np.complex128)
        if a.shape != (1 << self._n,):
            raise ValueError("State vector size mismatch")
        _lib.check(_lib.hip.qsim_dm_init_pure(self._sv.handle, self._n, _ptr(a)))

    def initMaximallyMixed(self) -> None:
        _lib.check(_lib.hip.qsim_dm_init_maximally_mixed(self._sv.handle, self._n))

    def getNumQubits(self) -> int: return self._n
    def getDimension(self) -> int: return 1 << self._n
    def getNumElements(self) -> int: return 1 << (2 * self._n)
    def getMemoryBytes(self) -> int: return 16 << (2 * self._n)

    def getProbabilities(self) -> np.ndarray:
        out = np.empty(1 << self._n, dtype=np.float64)
        _lib.check(_lib.hip.qsim_dm_diagonal(self._sv.handle, self._n, _ptr(out)))
        return out

    def getMatrix(self) -> np.ndarray:
        return self._sv.toHost().reshape(1 << self._n, 1 << self._n)

    def trace(self) -> float: return float(np.sum(self.getProbabilities()))
    def purity(self) -> float: return self._sv.getTotalProbability()  # sum |rho_ij|^2 (:147-167)

    def isValid(self, tolerance: float = 1e-10) -> bool:
        if abs(self.trace() - 1.0) > tolerance:
            return False
        p = self.purity()
        return 1.0 / (1 << self._n) - tolerance <= p <= 1.0 + tolerance


class DensityMatrixSimulator:
    def __init__(self, n_qubits: int, noise: Optional[NoiseModel] = None,
                 mode: RunMode = RunMode.Fused, reference_y: bool = False):
        self._rho = DensityMatrix(n_qubits)
        self._noise = noise or NoiseModel()
        self._mode = RunMode(mode)
        self._ref_y = bool(reference_y)
        self._rng = np.random.default_rng(int.from_bytes(os.urandom(4), "little"))

    @property
    def density(self) -> DensityMatrix:
        return self._rho

    def setSeed(self, seed: int) -> None: self._rng = np.random.default_rng(seed)

    def setReferenceCompatible(self, on: bool = True) -> None:
        """Y as the reference's dmApplyY (-Y rho Y^dag, src/DensityMatrix.cu:507-546)."""
        self._ref_y = bool(on)

    def _flags(self) -> int:
        return int(self._mode) | (_lib.QSIM_DM_REFERENCE_Y if self._ref_y else 0)
    def reset(self) -> None: self._rho.reset()

    def _channels(self):
        """(type, qubit, p) entries; a global channel (empty qubit list) applies to every gate
        qubit (channelAppliesToQubit, include/NoiseModel.cuh:119-122) -> qubit -1."""
        flat = []
        for ch in self._noise.getChannels():
            for q in (ch.qubits or [-1]):
                flat.append((int(ch.type), q, ch.probability))
        arr = (_lib.qsim_noise_channel * max(1, len(flat)))()
        for i, (t, q, p) in enumerate(flat):
            arr[i].type, arr[i].qubit, arr[i].probability = t, q, p
        return arr, len(flat)

    def run(self, circuit: Circuit) -> None:
        g, ng = circuit.to_abi()
        ch, nch = self._channels()
        _lib.check(_lib.hip.qsim_dm_run(self._rho.state.handle, self._rho.getNumQubits(), g, ng,
                                        ch, nch, self._flags()))

    def applyGate(self, op: GateOp) -> None:
        c = Circuit(self._rho.getNumQubits())
        c.append(op)
        g, ng = c.to_abi()
        _lib.check(_lib.hip.qsim_dm_run(self._rho.state.handle, self._rho.getNumQubits(), g, ng,
                                        None, 0, self._flags()))

    def applyChannel(self, type, qubit: int, p: float) -> None:
        _lib.check(_lib.hip.qsim_dm_apply_channel(self._rho.state.handle, self._rho.getNumQubits(),
                                                  int(type), qubit, p))

    def getProbabilities(self) -> np.ndarray: return self._rho.getProbabilities()
    def getDensityMatrix(self) -> np.ndarray: return self._rho.getMatrix()
    def getPurity(self) -> float: return self._rho.purity()
    def getTrace(self) -> float: return self._rho.trace()
    def getNumQubits(self) -> int: return self._rho.getNumQubits()

    def measureQubit(self, qubit: int) -> int:
        """Reference semantics (src/DensityMatrix.cu:374-406): LSB bit `qubit`, result 1 with
        probability p1, rho <- P rho P / p."""
        n = self._rho.getNumQubits()
        if qubit < 0 or qubit >= n:
            raise ValueError(f"Qubit index {qubit} out of range [0, {n - 1}]")
        probs = self.getProbabilities()
        p1 = float(np.sum(probs[(np.arange(probs.size) >> qubit) & 1 == 1]))
        result = 1 if float(self._rng.random()) < p1 else 0
        pr = p1 if result == 1 else 1.0 - p1
        sv = self._rho.state
        sv.collapse(qubit + n, result, 1.0 / pr)
        sv.collapse(qubit, result, 1.0)
        return result
