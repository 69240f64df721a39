// OptimizedGates.cpp — named dispatchers over the C ABI (include/qsim/OptimizedGates.hpp).
#include "qsim/OptimizedGates.hpp"

#include "abi_util.hpp"

namespace qsim {

using detail::check;

void applyHadamardOptimized(void* state, int n_qubits, int target, void* stream) {
    check(qsim_apply_hadamard_optimized(state, n_qubits, target, stream));
}

void applyCNOTOptimized(void* state, int n_qubits, int control, int target, void* stream) {
    check(qsim_apply_cnot_optimized(state, n_qubits, control, target, stream));
}

void applyGate1QOptimized(void* state, int n_qubits, int target, const std::complex<double> (&m)[4],
                          void* stream) {
    double mm[8];
    for (int i = 0; i < 4; ++i) {
        mm[2 * i] = m[i].real();
        mm[2 * i + 1] = m[i].imag();
    }
    check(qsim_apply_matrix1q_raw(state, n_qubits, target, mm, stream));
}

}  // namespace qsim
