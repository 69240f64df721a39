"""StateVector / Simulator / NoiseModel / BatchedSimulator over the C ABI.

Mirrors the reference C++ classes (include/StateVector.cuh:66-124, include/Simulator.hpp:53-85,
include/NoiseModel.cuh:46-297) with the same method names, argument meanings and exception
classes (ValueError ~ std::invalid_argument, IndexError ~ std::out_of_range,
RuntimeError ~ std::runtime_error).  All compute runs in the HIP engine; nothing here falls back
to the CPU.
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .circuit import Circuit, GateOp, is_valid_qubit_count, MAX_QUBITS, MIN_QUBITS

_c = ctypes


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_c.c_void_p)


class RunMode(enum.IntEnum):
    PerGate = _lib.QSIM_RUN_PER_GATE
    Fused = _lib.QSIM_RUN_FUSED


def device_count() -> int:
    c = _c.c_int(0)
    _lib.check(_lib.hip.qsim_device_count(_c.byref(c)))
    return c.value


def set_device(device: int) -> None:
    """Device the calling thread's next objects are created on (one process per GPU)."""
    _lib.check(_lib.hip.qsim_set_device(int(device)))


def device_info(device: int = 0):
    name = _c.create_string_buffer(256)
    cus = _c.c_int(0)
    mem = _c.c_size_t(0)
    _lib.check(_lib.hip.qsim_device_info(device, name, 256, _c.byref(cus), _c.byref(mem)))
    return {"name": name.value.decode(), "cu_count": cus.value, "total_mem": mem.value}


def sequence_circuit(circuits, n: int) -> Circuit:
    """The gates of `circuits` (each of n qubits) in order, as one circuit."""
    seq = Circuit(n)
    for c in circuits:
        if c.getNumQubits() != n:
            raise ValueError("Circuit qubit count doesn't match simulator")
        seq.extend(c)
    return seq


class StateVector:
    def __init__(self, num_qubits: int, device: Optional[int] = None):
        if not is_valid_qubit_count(num_qubits):
            raise ValueError(f"Number of qubits must be between {MIN_QUBITS} and {MAX_QUBITS}")
        self._h = _c.c_void_p()
        if device is None:
            _lib.check(_lib.hip.qsim_state_create(num_qubits, _c.byref(self._h)))
        else:
            _lib.check(_lib.hip.qsim_state_create_on(device, num_qubits, _c.byref(self._h)))
        self._n = num_qubits
        self._rng: Optional[np.random.Generator] = None

    def __del__(self):
        self.close()

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.hip.qsim_state_destroy(h)
            self._h = _c.c_void_p()

    @property
    def handle(self):
        return self._h

    def getNumQubits(self) -> int: return self._n
    def getSize(self) -> int: return 1 << self._n

    def initializeZero(self) -> None:
        _lib.check(_lib.hip.qsim_state_init_zero(self._h))

    def initializeBasis(self, idx: int) -> None:
        if idx < 0 or idx >= (1 << self._n):
            raise ValueError("Basis index out of range")
        _lib.check(_lib.hip.qsim_state_init_basis(self._h, idx))

    def devicePtr(self) -> int:
        p = _c.c_void_p()
        _lib.check(_lib.hip.qsim_state_device_ptr(self._h, _c.byref(p)))
        return p.value

    def stream(self) -> int:
        p = _c.c_void_p()
        _lib.check(_lib.hip.qsim_state_stream(self._h, _c.byref(p)))
        return p.value

    def synchronize(self) -> None:
        _lib.check(_lib.hip.qsim_state_sync(self._h))

    def toHost(self) -> np.ndarray:
        out = np.empty(1 << self._n, dtype=np.complex128)
        _lib.check(_lib.hip.qsim_state_to_host(self._h, _ptr(out)))
        return out

    def fromHost(self, amps) -> None:
        a = np.ascontiguousarray(amps, dtype=np.complex128)
        if a.shape != (1 << self._n,):
            raise ValueError("amplitude count does not match 2^n")
        _lib.check(_lib.hip.qsim_state_from_host(self._h, _ptr(a)))

    def getProbabilities(self) -> np.ndarray:
        out = np.empty(1 << self._n, dtype=np.float64)
        _lib.check(_lib.hip.qsim_state_probabilities(self._h, _ptr(out)))
        return out

    def getTotalProbability(self) -> float:
        t = _c.c_double()
        _lib.check(_lib.hip.qsim_state_total_probability(self._h, _c.byref(t)))
        return t.value

    def isNormalized(self, tolerance: float = 1e-10) -> bool:
        return abs(self.getTotalProbability() - 1.0) <= tolerance

    def assertNormalized(self, tolerance: float = 1e-10) -> None:
        t = self.getTotalProbability()
        if abs(t - 1.0) > tolerance:
            raise RuntimeError(f"State vector not normalized: total probability = {t}")

    def maxAbsDiff(self, other: "StateVector") -> float:
        """Larger per-component |a - b| against another state of the same size, computed on the
        device in the identity layout (qsim_state_max_abs_diff; the reference's 1e-12 per-component
        bar, tests/test_gpu_cpu_equivalence.cu:26, without a host copy)."""
        d = _c.c_double()
        _lib.check(_lib.hip.qsim_state_max_abs_diff(self._h, other._h, _c.byref(d)))
        return d.value

    def getDeviceMemoryBytes(self) -> int:
        """Device bytes this state owns now, the relayout plans' second buffer included."""
        b = _c.c_uint64()
        _lib.check(_lib.hip.qsim_state_memory_bytes(self._h, _c.byref(b)))
        return b.value

    def probBitZero(self, bit: int) -> float:
        p = _c.c_double()
        _lib.check(_lib.hip.qsim_state_prob_bit_zero(self._h, bit, _c.byref(p)))
        return p.value

    def collapse(self, bit: int, result: int, scale: float) -> None:
        _lib.check(_lib.hip.qsim_state_collapse(self._h, bit, result, scale))

    def setSeed(self, seed: int) -> None:
        self._rng = np.random.default_rng(seed)

    def _uniforms(self, k: int) -> np.ndarray:
        rng = self._rng if self._rng is not None else np.random.default_rng()
        return rng.random(k)

    def measureBit(self, bit: int) -> int:
        if bit < 0 or bit >= self._n:
            raise ValueError(f"Qubit index {bit} out of range [0, {self._n - 1}]")
        p0 = self.probBitZero(bit)
        r = float(self._uniforms(1)[0])
        result = 0 if r < p0 else 1
        pr = p0 if result == 0 else 1.0 - p0
        if pr < 1e-15:
            raise RuntimeError(f"Measurement result {result} has zero probability")
        self.collapse(bit, result, 1.0 / np.sqrt(pr))
        return result

    def measure(self, qubit: int) -> int:
        """Reference semantics: big-endian index bit n-1-qubit (src/StateVector.cu:87-89, F2)."""
        if qubit < 0 or qubit >= self._n:
            raise ValueError(f"Qubit index {qubit} out of range [0, {self._n - 1}]")
        return self.measureBit(self._n - 1 - qubit)

    def sampleWith(self, uniforms) -> np.ndarray:
        u = np.ascontiguousarray(uniforms, dtype=np.float64)
        if u.size <= 0:
            raise ValueError("n_shots must be positive")
        out = np.empty(u.size, dtype=np.int64)
        _lib.check(_lib.hip.qsim_state_sample(self._h, _ptr(u), int(u.size), _ptr(out)))
        return out

    def sample(self, n_shots: int) -> np.ndarray:
        if n_shots <= 0:
            raise ValueError("n_shots must be positive")
        return self.sampleWith(self._uniforms(n_shots))

    # -- direct gate application (kernel-level entry, Gates.cuh analogue)
    def applyGate(self, op: GateOp) -> None:
        g = _lib.qsim_gate()
        g.type = int(op.type)
        g.nqubits = len(op.qubits)
        for j, q in enumerate(op.qubits):
            g.qubits[j] = q
        g.parameter = op.parameter
        _lib.check(_lib.hip.qsim_apply_gate(self._h, _c.byref(g)))

    def applyMatrix1Q(self, target: int, m, controls: Sequence[int] = ()) -> None:
        mm = np.asarray(m, dtype=np.complex128).reshape(4)
        buf = (_c.c_double * 8)(*[v for z in mm for v in (z.real, z.imag)])
        ctl = (_c.c_int * max(1, len(controls)))(*controls)
        _lib.check(_lib.hip.qsim_apply_matrix1q(self._h, target, buf, ctl, len(controls)))

    def applyMatrix2Q(self, q0: int, q1: int, m, controls: Sequence[int] = ()) -> None:
        """General 4x4 on (q0, q1), row-major over (bit q1 << 1) | bit q0 (qsim_apply_matrix2q)."""
        mm = np.asarray(m, dtype=np.complex128).reshape(16)
        buf = (_c.c_double * 32)(*[v for z in mm for v in (z.real, z.imag)])
        ctl = (_c.c_int * max(1, len(controls)))(*controls)
        _lib.check(_lib.hip.qsim_apply_matrix2q(self._h, q0, q1, buf, ctl, len(controls)))

    def applyMatrix(self, targets: Sequence[int], m, controls: Sequence[int] = ()) -> None:
        """General 2^k x 2^k matrix, k = len(targets) <= 8, row-major; matrix-index bit j is
        qubit targets[j]; applied on the control == 1 subspace (qsim_apply_matrix)."""
        k = len(targets)
        mm = np.asarray(m, dtype=np.complex128)
        if k < 1 or k > 8 or mm.size != (1 << k) ** 2:
            raise ValueError("matrix must be 2^k x 2^k for 1 <= k <= 8 targets")
        buf = np.ascontiguousarray(mm.reshape(-1)).view(np.float64)
        tg = (_c.c_int * k)(*targets)
        ctl = (_c.c_int * max(1, len(controls)))(*controls)
        _lib.check(_lib.hip.qsim_apply_matrix(self._h, tg, k,
                                              buf.ctypes.data_as(_c.POINTER(_c.c_double)),
                                              ctl, len(controls)))

    def applyDiagonalLayer(self, gate_params, active_qubits: int) -> None:
        """applyFusedSingleQubitLayer (src/OptimizedGates.cu:344-382): gate_params[q][0] / [q][3]
        scale the bit-q = 0 / 1 amplitudes of every active qubit."""
        gp = np.ascontiguousarray(np.asarray(gate_params, dtype=np.complex128).reshape(-1, 4))
        if gp.shape[0] < self._n:
            raise ValueError("gate_params needs 4 entries per qubit")
        flat = gp.view(np.float64).reshape(-1)
        _lib.check(_lib.hip.qsim_apply_diagonal_layer(
            self._h, flat.ctypes.data_as(_c.POINTER(_c.c_double)), active_qubits))

    def run(self, circuit: Circuit, mode: RunMode = RunMode.Fused) -> None:
        arr, n = circuit.to_abi()
        _lib.check(_lib.hip.qsim_run(self._h, arr, n, int(mode)))

    def runSequence(self, circuits, mode: RunMode = RunMode.Fused) -> None:
        """Apply `circuits` one after the other as ONE engine run (no reference counterpart): the
        planner sees their gates together, so a pass may hold the end of one circuit and the
        start of the next — consecutive 100-gate W-HC circuits at 30 qubits plan into 2.5-2.75
        passes each instead of 4.  The same state as run() on each in turn."""
        seq = sequence_circuit(circuits, self._n)
        self.run(seq, mode)

    def perm(self):
        """Current logical -> physical qubit map (identity unless a fused run relabeled)."""
        p = (_c.c_int32 * self._n)()
        _lib.check(_lib.hip.qsim_state_perm(self._h, p))
        return list(p)

    def layoutInfo(self) -> dict:
        """The first-run layout decision: tile height of the fused runs, whether it was chosen by
        timing candidates on the device, whether the qubits are relabeled now."""
        h, c, r = _c.c_int(0), _c.c_int(0), _c.c_int(0)
        _lib.check(_lib.hip.qsim_state_layout_info(self._h, _c.byref(h), _c.byref(c), _c.byref(r)))
        rl = _c.c_int(0)
        _lib.check(_lib.hip.qsim_state_relayout(self._h, _c.byref(rl)))
        return {"tile_qubits": 6 + h.value, "calibrated": bool(c.value), "relabeled": bool(r.value),
                "relayout": bool(rl.value)}

    def restoreLayout(self) -> None:
        """Undo a relabeling now (the SWAP network every index-based reader runs first)."""
        _lib.check(_lib.hip.qsim_state_restore_layout(self._h))

    # -- profiling
    def profile(self, enable: bool = True) -> None:
        _lib.check(_lib.hip.qsim_state_profile(self._h, 1 if enable else 0))

    def profileReset(self) -> None:
        _lib.check(_lib.hip.qsim_state_profile_reset(self._h))

    def lastRunInfo(self):
        """(tile passes, passes run by circuit-specialised kernels) of the last fused run."""
        p, j = _c.c_int(0), _c.c_int(0)
        _lib.check(_lib.hip.qsim_state_last_run(self._h, _c.byref(p), _c.byref(j)))
        return p.value, j.value

    def profileStats(self):
        n = _c.c_int(0)
        _lib.check(_lib.hip.qsim_state_profile_count(self._h, _c.byref(n)))
        out = []
        for i in range(n.value):
            name = _c.create_string_buffer(64)
            ms, cnt, by = _c.c_double(), _c.c_int64(), _c.c_double()
            _lib.check(_lib.hip.qsim_state_profile_get(self._h, i, name, 64, _c.byref(ms),
                                                       _c.byref(cnt), _c.byref(by)))
            out.append({"name": name.value.decode(), "ms": ms.value, "launches": cnt.value,
                        "alg_bytes": by.value})
        return out


class Simulator:
    """Reference Simulator (src/Simulator.cu:22-189).  run() defaults to fused passes."""

    def __init__(self, num_qubits: int, mode: RunMode = RunMode.Fused, device: Optional[int] = None):
        self._state = StateVector(num_qubits, device)
        self._mode = RunMode(mode)

    @property
    def state(self) -> StateVector:
        return self._state

    def setRunMode(self, mode: RunMode) -> None: self._mode = RunMode(mode)
    def getRunMode(self) -> RunMode: return self._mode
    def setSeed(self, seed: int) -> None: self._state.setSeed(seed)
    def reset(self) -> None: self._state.initializeZero()

    def run(self, circuit: Circuit) -> None:
        if circuit.getNumQubits() != self._state.getNumQubits():
            raise ValueError("Circuit qubit count doesn't match simulator")
        self._state.run(circuit, self._mode)

    def runSequence(self, circuits) -> None:
        """run() of each circuit in turn, planned as one (StateVector.runSequence)."""
        self._state.runSequence(circuits, self._mode)

    def applyGate(self, op: GateOp) -> None: self._state.applyGate(op)
    def getStateVector(self) -> np.ndarray: return self._state.toHost()
    def getProbabilities(self) -> np.ndarray: return self._state.getProbabilities()

    def sample(self, n_shots: int) -> np.ndarray:
        if n_shots == 0:
            return np.empty(0, dtype=np.int64)
        return self._state.sample(n_shots)

    def measureQubit(self, qubit: int) -> int: return self._state.measure(qubit)
    def getNumQubits(self) -> int: return self._state.getNumQubits()
    def getStateSize(self) -> int: return self._state.getSize()
    def synchronize(self) -> None: self._state.synchronize()


class NoiseType(enum.IntEnum):
    Depolarizing = 0
    AmplitudeDamping = 1
    PhaseDamping = 2
    BitFlip = 3
    PhaseFlip = 4
    BitPhaseFlip = 5


class NoiseChannel:
    def __init__(self, type: NoiseType, qubits: Sequence[int], probability: float):
        self.type = NoiseType(type)
        self.qubits = list(qubits)
        self.probability = float(probability)


class NoiseModel:
    """Reference NoiseModel (src/NoiseModel.cu:24-101), incl. the empty-qubit 'global' form (F6)."""

    def __init__(self):
        self._ch: List[NoiseChannel] = []

    def _per(self, t, qubits, p):
        for q in qubits:
            self._ch.append(NoiseChannel(t, [q], p))

    def addDepolarizing(self, qubits_or_p, p=None):
        if p is None:
            self._ch.append(NoiseChannel(NoiseType.Depolarizing, [], qubits_or_p))
        else:
            self._per(NoiseType.Depolarizing, qubits_or_p, p)

    def addBitFlip(self, qubits_or_p, p=None):
        if p is None:
            self._ch.append(NoiseChannel(NoiseType.BitFlip, [], qubits_or_p))
        else:
            self._per(NoiseType.BitFlip, qubits_or_p, p)

    def addPhaseFlip(self, qubits_or_p, p=None):
        if p is None:
            self._ch.append(NoiseChannel(NoiseType.PhaseFlip, [], qubits_or_p))
        else:
            self._per(NoiseType.PhaseFlip, qubits_or_p, p)

    def addBitPhaseFlip(self, qubits_or_p, p=None):
        if p is None:
            self._ch.append(NoiseChannel(NoiseType.BitPhaseFlip, [], qubits_or_p))
        else:
            self._per(NoiseType.BitPhaseFlip, qubits_or_p, p)

    def addAmplitudeDamping(self, qubits_or_g, g=None):
        if g is None:
            self._ch.append(NoiseChannel(NoiseType.AmplitudeDamping, [], qubits_or_g))
        else:
            self._per(NoiseType.AmplitudeDamping, qubits_or_g, g)

    def addPhaseDamping(self, qubits_or_g, g=None):
        if g is None:
            self._ch.append(NoiseChannel(NoiseType.PhaseDamping, [], qubits_or_g))
        else:
            self._per(NoiseType.PhaseDamping, qubits_or_g, g)

    def addDepolarizingAll(self, n, p): self._per(NoiseType.Depolarizing, range(n), p)
    def addAmplitudeDampingAll(self, n, g): self._per(NoiseType.AmplitudeDamping, range(n), g)
    def addPhaseDampingAll(self, n, g): self._per(NoiseType.PhaseDamping, range(n), g)
    def getChannels(self) -> List[NoiseChannel]: return list(self._ch)
    def hasNoise(self) -> bool: return bool(self._ch)
    def clear(self) -> None: self._ch.clear()

    def to_abi(self):
        flat = [(c.type, q, c.probability) for c in self._ch for q in c.qubits]
        arr = (_lib.qsim_noise_channel * max(1, len(flat)))()
        for i, (t, q, p) in enumerate(flat):
            arr[i].type, arr[i].qubit, arr[i].probability = int(t), q, p
        return arr, len(flat)


class NoisySimulator:
    """Reference NoisySimulator (include/NoiseModel.cuh:139-214, src/NoiseModel.cu:320-651):
    Monte-Carlo noise on one state vector.  run() applies each gate and then every channel entry
    of the model (one per-pair noise pass each, noise.hip); global channels act on no qubit (F6).
    measureQubit measures index bit `qubit` (LSB-first, src/NoiseModel.cu:615-651) unlike
    StateVector.measure (F2).  Seeded from os.urandom like the reference's random_device."""

    def __init__(self, num_qubits: int, noise_model: Optional[NoiseModel] = None):
        self._state = StateVector(num_qubits)
        self._noise = noise_model or NoiseModel()
        self.setSeed(int.from_bytes(os.urandom(4), "little"))

    def setNoiseModel(self, nm: NoiseModel) -> None: self._noise = nm
    def getNoiseModel(self) -> NoiseModel: return self._noise

    def setSeed(self, seed: int) -> None:
        self._seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self._counter = 0
        self._rng = np.random.default_rng(seed)

    @property
    def state(self) -> StateVector:
        return self._state

    def reset(self) -> None: self._state.initializeZero()

    def run(self, circuit: Circuit, mode: RunMode = RunMode.Fused) -> None:
        if circuit.getNumQubits() != self._state.getNumQubits():
            raise ValueError("Circuit qubit count doesn't match simulator")
        g, ng = circuit.to_abi()
        ch, nch = self._noise.to_abi()
        ctr = _c.c_uint64(self._counter)
        _lib.check(_lib.hip.qsim_noisy_run(self._state.handle, g, ng, ch, nch, self._seed,
                                           _c.byref(ctr), int(mode)))
        self._counter = ctr.value

    def applyGate(self, op: GateOp) -> None: self._state.applyGate(op)

    def applyNoise(self, channel: NoiseChannel) -> None:
        for q in channel.qubits:
            self.applyNoiseToQubit(channel.type, q, channel.probability)

    def applyNoiseToQubit(self, type: NoiseType, qubit: int, probability: float) -> None:
        _lib.check(_lib.hip.qsim_noise_apply(self._state.handle, int(type), qubit, probability,
                                             self._seed, self._counter))
        self._counter += 1

    def getStateVector(self) -> np.ndarray: return self._state.toHost()
    def getProbabilities(self) -> np.ndarray: return self._state.getProbabilities()

    def sample(self, n_shots: int) -> np.ndarray:
        """CDF + lower_bound like the reference (src/NoiseModel.cu:599-613), on the device."""
        if n_shots <= 0:
            return np.empty(0, dtype=np.int64)
        return self._state.sampleWith(self._rng.random(n_shots))

    def measureQubit(self, qubit: int) -> int:
        p0 = self._state.probBitZero(qubit)
        result = 0 if float(self._rng.random()) < p0 else 1
        kept = p0 if result == 0 else self._state.getTotalProbability() - p0
        self._state.collapse(qubit, result, 1.0 / np.sqrt(kept))
        return result

    def getNumQubits(self) -> int: return self._state.getNumQubits()
    def getStateSize(self) -> int: return self._state.getSize()
    def synchronize(self) -> None: self._state.synchronize()


class BatchedGateSet(enum.IntEnum):
    Full = _lib.QSIM_BATCH_FULL_GATESET
    Reference = _lib.QSIM_BATCH_REFERENCE_GATESET


class BatchedNoise(enum.IntEnum):
    """Reference (the default, as the reference behaves): the per-amplitude-pair depolarizing
    process after every gate (src/NoiseModel.cu:834-892; Depolarizing entries only, SURVEY
    F5/F7).  Physical (opt-in): one draw per trajectory, channel and gate (the Kraus channel on a
    pure-state trajectory), run as Pauli frames inside fused passes."""
    Physical = 0
    Reference = _lib.QSIM_BATCH_REFERENCE_NOISE


class BatchedSimulator:
    """Reference BatchedSimulator (src/NoiseModel.cu:653-972)."""

    def __init__(self, num_qubits: int, batch_size: int, noise_model: Optional[NoiseModel] = None,
                 gate_set: BatchedGateSet = BatchedGateSet.Full,
                 noise: BatchedNoise = BatchedNoise.Reference):
        self._h = _c.c_void_p()
        _lib.check(_lib.hip.qsim_batch_create(num_qubits, batch_size, _c.byref(self._h)))
        self._n, self._b = num_qubits, batch_size
        self._noise = noise_model or NoiseModel()
        self._gate_set = BatchedGateSet(gate_set)
        self._noise_sem = BatchedNoise(noise)
        self._rng = np.random.default_rng()

    def __del__(self):
        self.close()

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.hip.qsim_batch_destroy(h)
            self._h = _c.c_void_p()

    def setNoiseModel(self, nm: NoiseModel) -> None: self._noise = nm
    def setGateSet(self, g: BatchedGateSet) -> None: self._gate_set = BatchedGateSet(g)
    def setNoiseSemantics(self, m: BatchedNoise) -> None: self._noise_sem = BatchedNoise(m)

    def setReferenceCompatible(self) -> None:
        """Both reference behaviours: gate set X/Y/Z/H/CNOT and per-pair depolarizing noise."""
        self._gate_set = BatchedGateSet.Reference
        self._noise_sem = BatchedNoise.Reference

    def setSeed(self, seed: int) -> None:
        self._rng = np.random.default_rng(seed)
        _lib.check(_lib.hip.qsim_batch_set_seed(self._h, seed))

    def setTrajectoryOffset(self, first: int) -> None:
        """This object's trajectories are [first, first + batch_size) of a larger ensemble: noise
        draws are keyed by the global trajectory index, so shards of an ensemble (one per GPU)
        reproduce the single-object run exactly (qsim_batch_set_trajectory_offset)."""
        _lib.check(_lib.hip.qsim_batch_set_trajectory_offset(self._h, int(first)))

    def reset(self) -> None: _lib.check(_lib.hip.qsim_batch_reset(self._h))

    def run(self, circuit: Circuit, per_gate: bool = False) -> None:
        """per_gate: one kernel per gate and one Pauli pass per noisy step (the reference's
        structure) instead of fused passes under Pauli frames; identical trajectories."""
        if circuit.getNumQubits() != self._n:
            raise ValueError("Circuit qubit count doesn't match simulator")
        g, ng = circuit.to_abi()
        ch, nch = self._noise.to_abi()
        flags = int(self._gate_set) | int(self._noise_sem) | \
            (_lib.QSIM_BATCH_PER_GATE if per_gate else 0)
        _lib.check(_lib.hip.qsim_batch_run(self._h, g, ng, ch, nch, flags))

    def synchronize(self) -> None: _lib.check(_lib.hip.qsim_batch_sync(self._h))

    def getAverageProbabilities(self) -> np.ndarray:
        out = np.empty(1 << self._n, dtype=np.float64)
        _lib.check(_lib.hip.qsim_batch_avg_probabilities(self._h, _ptr(out)))
        return out

    def getProbabilities(self, t: int) -> np.ndarray:
        if t < 0 or t >= self._b:
            raise IndexError("Invalid trajectory index")
        out = np.empty(1 << self._n, dtype=np.float64)
        _lib.check(_lib.hip.qsim_batch_traj_probabilities(self._h, t, _ptr(out)))
        return out

    def getStateVector(self, t: int) -> np.ndarray:
        if t < 0 or t >= self._b:
            raise IndexError("Invalid trajectory index")
        out = np.empty(1 << self._n, dtype=np.complex128)
        _lib.check(_lib.hip.qsim_batch_traj_state(self._h, t, _ptr(out)))
        return out

    def sampleWith(self, uniforms: np.ndarray) -> np.ndarray:
        """Device sampling with given uniforms, shape (B, shots) trajectory-major; returns the
        (B, shots) outcomes (lower_bound over each trajectory's CDF, 2^n past its end)."""
        u = np.ascontiguousarray(uniforms, dtype=np.float64)
        if u.ndim != 2 or u.shape[0] != self._b:
            raise ValueError("uniforms must have shape (batch_size, shots)")
        out = np.empty(u.shape, dtype=np.int64)
        _lib.check(_lib.hip.qsim_batch_sample(self._h, _ptr(u), int(u.shape[1]), _ptr(out)))
        return out

    def _draw(self, n_shots: int) -> np.ndarray:
        if n_shots < 0:
            raise ValueError("n_shots must be non-negative")
        # the reference draws shot by shot inside the trajectory loop (NoiseModel.cu:944-954)
        return self._rng.random((self._b, n_shots))

    def sample(self, n_shots: int) -> np.ndarray:
        """[shot][trajectory] outcomes: per-trajectory CDF + lower_bound (NoiseModel.cu:938-957),
        on the device."""
        return np.ascontiguousarray(self.sampleWith(self._draw(n_shots)).T)

    def getHistogram(self, n_shots: int) -> np.ndarray:
        """Counts over every trajectory and shot, out-of-range outcomes skipped
        (NoiseModel.cu:959-972); sampling and counting on the device."""
        u = np.ascontiguousarray(self._draw(n_shots))
        hist = np.empty(1 << self._n, dtype=np.int64)
        _lib.check(_lib.hip.qsim_batch_histogram(self._h, _ptr(u), int(n_shots), _ptr(hist)))
        return hist

    def getNumQubits(self) -> int: return self._n
    def getBatchSize(self) -> int: return self._b
    def getTotalMemoryBytes(self) -> int: return self._b * (1 << self._n) * 16

    def lastRunInfo(self):
        """(tile passes, passes run by circuit-specialised kernels) of the last fused run."""
        p, j = _c.c_int(0), _c.c_int(0)
        _lib.check(_lib.hip.qsim_batch_last_run(self._h, _c.byref(p), _c.byref(j)))
        return p.value, j.value

    def profile(self, enable: bool = True) -> None:
        _lib.check(_lib.hip.qsim_batch_profile(self._h, 1 if enable else 0))

    def profileStats(self):
        n = _c.c_int(0)
        _lib.check(_lib.hip.qsim_batch_profile_count(self._h, _c.byref(n)))
        out = []
        for i in range(n.value):
            name = _c.create_string_buffer(64)
            ms, cnt, by = _c.c_double(), _c.c_int64(), _c.c_double()
            _lib.check(_lib.hip.qsim_batch_profile_get(self._h, i, name, 64, _c.byref(ms),
                                                       _c.byref(cnt), _c.byref(by)))
            out.append({"name": name.value.decode(), "ms": ms.value, "launches": cnt.value,
                        "alg_bytes": by.value})
        return out
