// StateVector.hpp — GPU-resident 2^n complex<double> state (reference include/StateVector.cuh:66-124).
//
// Host-only header: the device buffer and its HIP stream live behind the C ABI handle
// qsim_state (include/qsim_hip.h).  Move-only RAII owner like the reference (copy deleted,
// moved-from object holds nothing: src/StateVector.cu:150-171).
#pragma once

#include <complex>
#include <cstddef>
#include <cstdint>
#include <random>
#include <vector>

struct qsim_state;

namespace qsim {

// Layout of one device amplitude: interleaved {re, im} doubles (what devicePtr() points at).
struct Amplitude {
    double re;
    double im;
};

class StateVector {
public:
    explicit StateVector(int num_qubits);  // std::invalid_argument outside [1, 30]
    ~StateVector();
    StateVector(const StateVector&) = delete;
    StateVector& operator=(const StateVector&) = delete;
    StateVector(StateVector&& other) noexcept;
    StateVector& operator=(StateVector&& other) noexcept;

    void initializeZero();
    void initializeBasis(size_t basis_idx);  // std::invalid_argument if >= 2^n

    int getNumQubits() const { return num_qubits_; }
    size_t getSize() const { return size_; }

    // Device address of amplitude 0 (for the kernel-level entry qsim_apply_gate_raw).
    Amplitude* devicePtr();
    const Amplitude* devicePtr() const;

    // General controlled 2x2 unitary [[m0, m1], [m2, m3]] on `target` (src/OptimizedGates.cu:165-183
    // applyGate1Q_coalesced, plus controls); std::out_of_range / std::invalid_argument on bad qubits.
    void applyMatrix1Q(int target, const std::complex<double> (&m)[4],
                       const std::vector<int>& controls = {});
    // General 2^k x 2^k matrix (row-major, k = targets.size() <= 8; matrix-index bit j = qubit
    // targets[j]) on the control == 1 subspace (qsim_apply_matrix).
    void applyMatrix(const std::vector<int>& targets, const std::vector<std::complex<double>>& m,
                     const std::vector<int>& controls = {});

    std::vector<std::complex<double>> toHost() const;
    void fromHost(const std::vector<std::complex<double>>& amplitudes);
    std::vector<double> getProbabilities() const;
    double getTotalProbability() const;  // device wave64 reduction
    bool isNormalized(double tolerance = 1e-10) const;
    // Extensions (no reference counterpart): the larger per-component |a - b| against another
    // state of the same size, on the device; the device bytes this state owns now
    // (qsim_state_max_abs_diff / qsim_state_memory_bytes).
    double maxAbsDiff(const StateVector& other) const;
    size_t getDeviceMemoryBytes() const;
    void assertNormalized(double tolerance = 1e-10) const;  // std::runtime_error

    // Reference semantics (src/StateVector.cu:260-314): measures index bit n-1-qubit
    // (big-endian), collapses and renormalizes.  std::invalid_argument on a bad
    // qubit, std::runtime_error when the drawn outcome has probability < 1e-15.
    int measure(int qubit);
    // Consistent with the gate convention: measures index bit `bit` (== gate qubit `bit`).
    int measureBit(int bit);
    std::vector<int> sample(int n_shots);  // std::invalid_argument if n_shots <= 0

    // Reproducible measurement/sampling (the reference seeds from std::random_device).
    void setSeed(unsigned int seed);

    qsim_state* handle() const { return h_; }

private:
    int num_qubits_;
    size_t size_;
    qsim_state* h_;
    bool seeded_ = false;
    std::mt19937 rng_;

    // Uniforms on [0,1) from uniform_real_distribution<double> over mt19937, seeded by
    // std::random_device per call (reference) or from setSeed's persistent engine.
    std::vector<double> uniforms(int count);
    void release();
};

}  // namespace qsim
