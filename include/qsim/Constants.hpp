// Constants.hpp — numeric constants, limits and qubit-count checks of the qsim C++ API.
//
// Mirrors the user-visible parts of the reference's include/Constants.hpp:34-50 (constants),
// :60-69 (block size and qubit limits) and :112-132 (helpers).  The CUDA error macros of the
// reference (:83-100) have no counterpart: device errors surface from the C ABI as status codes
// and are rethrown as std::runtime_error by the API classes.
#pragma once

#include <cstddef>

namespace qsim {

namespace constants {
constexpr double PI = 3.14159265358979323846;
constexpr double TWO_PI = 2.0 * PI;
constexpr double HALF_PI = PI / 2.0;
constexpr double QUARTER_PI = PI / 4.0;
constexpr double SQRT2 = 1.41421356237309504880;
constexpr double INV_SQRT2 = 0.70710678118654752440;
constexpr double EPSILON = 1e-10;
constexpr double PROBABILITY_EPSILON = 1e-12;
}  // namespace constants

namespace device_config {
// One 256-thread workgroup = 4 wave64s on gfx950.
constexpr int DEFAULT_BLOCK_SIZE = 256;
constexpr int WAVE_SIZE = 64;
// Single-GPU state limit kept at the reference's 30 (16 GiB of complex<double>); the sharded
// DistributedSimulator goes beyond it.
constexpr int MAX_QUBITS = 30;
constexpr int MIN_QUBITS = 1;
}  // namespace device_config

// Source compatibility with code written against the reference (include/Constants.hpp:56-75):
// `qsim::cuda_config::MAX_QUBITS`, `DEFAULT_BLOCK_SIZE`, ... keep compiling.  The values are the
// MI355X ones (a block of 256 threads is 4 wave64s); TARGET_CC_* name the gfx950 target.
namespace cuda_config {
constexpr int DEFAULT_BLOCK_SIZE = device_config::DEFAULT_BLOCK_SIZE;
constexpr int REDUCTION_BLOCK_SIZE = device_config::DEFAULT_BLOCK_SIZE;
constexpr int MAX_QUBITS = device_config::MAX_QUBITS;
constexpr int MIN_QUBITS = device_config::MIN_QUBITS;
constexpr int TARGET_CC_MAJOR = 9;  // gfx950: GFX9 family (CDNA4)
constexpr int TARGET_CC_MINOR = 50;
}  // namespace cuda_config

inline bool isValidQubit(int qubit, int num_qubits) { return qubit >= 0 && qubit < num_qubits; }
inline bool isValidQubitCount(int num_qubits) {
    return num_qubits >= device_config::MIN_QUBITS && num_qubits <= device_config::MAX_QUBITS;
}

}  // namespace qsim
