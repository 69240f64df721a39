// DensityMatrix.hpp — mixed-state simulation (reference include/DensityMatrix.cuh:63-224).
//
// Host-only header over the qsim_dm_* C ABI (include/qsim_hip.h): rho of n qubits lives in a
// 2n-index-bit engine state (rho[i][j] at i * 2^n + j, the reference's row-major layout), so gates
// and channels run through the same fused HIP passes as a state vector.  n in [1, 15]
// (std::invalid_argument otherwise; the reference allows 1-14).
#pragma once

#include <complex>
#include <random>
#include <vector>

#include "Circuit.hpp"
#include "NoiseModel.hpp"
#include "StateVector.hpp"

namespace qsim {

class DensityMatrix {
public:
    explicit DensityMatrix(int n_qubits);
    DensityMatrix(int n_qubits, const std::vector<std::complex<double>>& pure_state);
    DensityMatrix(DensityMatrix&&) noexcept = default;
    DensityMatrix& operator=(DensityMatrix&&) noexcept = default;

    void reset();
    void initFromPureState(const std::vector<std::complex<double>>& state);
    void initMaximallyMixed();

    int getNumQubits() const { return n_qubits_; }
    size_t getDimension() const { return size_t(1) << n_qubits_; }
    size_t getNumElements() const { return getDimension() * getDimension(); }
    size_t getMemoryBytes() const { return getNumElements() * 16; }

    std::vector<double> getProbabilities() const;
    std::vector<std::complex<double>> getMatrix() const { return rho_.toHost(); }
    double trace() const;
    double purity() const { return rho_.getTotalProbability(); }  // sum |rho_ij|^2
    bool isValid(double tolerance = 1e-10) const;

    Amplitude* getDevicePtr() { return rho_.devicePtr(); }
    StateVector& state() { return rho_; }
    const StateVector& state() const { return rho_; }

private:
    int n_qubits_;
    StateVector rho_;
};

class DensityMatrixSimulator {
public:
    explicit DensityMatrixSimulator(int n_qubits, const NoiseModel& noise = NoiseModel());

    void reset() { rho_.reset(); }
    void run(const Circuit& circuit);    // std::runtime_error for CRY/CRZ/Toffoli
    void applyGate(const GateOp& gate);  // unitary only, no noise (src/DensityMatrix.cu:214-267)

    std::vector<double> getProbabilities() const { return rho_.getProbabilities(); }
    std::vector<std::complex<double>> getDensityMatrix() const { return rho_.getMatrix(); }
    double getPurity() const { return rho_.purity(); }
    double getTrace() const { return rho_.trace(); }
    int measureQubit(int qubit);  // index bit `qubit` (src/DensityMatrix.cu:374-406)
    int getNumQubits() const { return rho_.getNumQubits(); }

    void setSeed(unsigned int seed) { rng_.seed(seed); }
    DensityMatrix& density() { return rho_; }
    // Reference results: Y as src/DensityMatrix.cu:507-546 computes it (-Y rho Y^dag); the
    // default is the physical Y rho Y^dag.  (Amplitude damping has no switch: the reference's
    // kernel reads rho11 while another thread rescales it, :1023-1036, so its result is not
    // deterministic; this engine uses the pre-channel rho11, the race-free reading.)
    void setReferenceCompatible(bool on = true) { reference_y_ = on; }

private:
    DensityMatrix rho_;
    NoiseModel noise_model_;
    std::mt19937 rng_;
    bool reference_y_ = false;
};

}  // namespace qsim
