// OptimizedGates.hpp — the reference's named gate dispatchers (include/OptimizedGates.cuh:152-166,
// src/OptimizedGates.cu:388-413) for code that drives raw device state pointers.
//
// `state` is a device pointer to 2^n_qubits {double re, im} amplitudes (StateVector::devicePtr())
// and `stream` an opaque hipStream_t (nullptr: the default stream).  The reference picked a
// shared-memory or coalesced CUDA kernel per call; here every call runs this build's wave64
// per-gate kernels (csrc/hip/gates.hip), which already stage by target height.  Errors throw
// like the rest of the API (std::invalid_argument / std::out_of_range / std::runtime_error).
#pragma once

#include <complex>

namespace qsim {

void applyHadamardOptimized(void* state, int n_qubits, int target, void* stream = nullptr);
void applyCNOTOptimized(void* state, int n_qubits, int control, int target, void* stream = nullptr);
// applyGate1Q_opt / applyGate1Q_coalesced: general [[m0, m1], [m2, m3]] on `target`.
void applyGate1QOptimized(void* state, int n_qubits, int target, const std::complex<double> (&m)[4],
                          void* stream = nullptr);

}  // namespace qsim
