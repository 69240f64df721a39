"""qsim_amd — MI355X-native state-vector simulator (Python mirror of the reference C++ API).

Importing this package loads lib/libqsim_hip.so (hand-written HIP kernels for gfx950) and
lib/libqsim.so (C++17 API incl. circuit factories).  There is no CPU fallback.
"""
from . import _lib
from .circuit import (Circuit, GateOp, GateType, MAX_QUBITS, MIN_QUBITS, createBellCircuit,
                      createGHZCircuit, createRandomCircuit, createRandomHCCircuit,
                      createScalingBenchmarkCircuit, is_valid_qubit_count)
from .simulator import (BatchedGateSet, BatchedNoise, BatchedSimulator, NoiseChannel, NoiseModel, NoiseType,
                        NoisySimulator, RunMode, Simulator, StateVector, device_count, device_info,
                        set_device)
from .density import DensityMatrix, DensityMatrixSimulator

__all__ = [
    "DensityMatrix", "DensityMatrixSimulator",
    "Circuit", "GateOp", "GateType", "MAX_QUBITS", "MIN_QUBITS", "createBellCircuit",
    "createGHZCircuit", "createRandomCircuit", "createRandomHCCircuit",
    "createScalingBenchmarkCircuit", "is_valid_qubit_count", "BatchedGateSet", "BatchedNoise",
    "BatchedSimulator", "NoiseChannel", "NoiseModel", "NoiseType", "NoisySimulator", "RunMode", "Simulator",
    "StateVector", "device_count", "device_info", "set_device",
]
