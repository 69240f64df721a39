// DensityMatrix.cpp — reference DensityMatrix / DensityMatrixSimulator (src/DensityMatrix.cu) over
// the qsim_dm_* C ABI.
#include "qsim/DensityMatrix.hpp"

#include <numeric>
#include <stdexcept>
#include <string>

#include "abi_util.hpp"

namespace qsim {

using detail::check;

static int checked_n(int n) {
    if (n < 1 || n > QSIM_DM_MAX_QUBITS)
        throw std::invalid_argument("Density matrix supports 1-" + std::to_string(QSIM_DM_MAX_QUBITS) + " qubits");
    return n;
}

DensityMatrix::DensityMatrix(int n_qubits) : n_qubits_(checked_n(n_qubits)), rho_(2 * n_qubits) {}

DensityMatrix::DensityMatrix(int n_qubits, const std::vector<std::complex<double>>& pure_state)
    : DensityMatrix(n_qubits) {
    initFromPureState(pure_state);
}

void DensityMatrix::reset() { rho_.initializeZero(); }

void DensityMatrix::initFromPureState(const std::vector<std::complex<double>>& state) {
    if (state.size() != getDimension()) throw std::invalid_argument("State vector size mismatch");
    check(qsim_dm_init_pure(rho_.handle(), n_qubits_, reinterpret_cast<const double*>(state.data())));
}

void DensityMatrix::initMaximallyMixed() { check(qsim_dm_init_maximally_mixed(rho_.handle(), n_qubits_)); }

std::vector<double> DensityMatrix::getProbabilities() const {
    std::vector<double> p(getDimension());
    check(qsim_dm_diagonal(rho_.handle(), n_qubits_, p.data()));
    return p;
}

double DensityMatrix::trace() const {
    const std::vector<double> p = getProbabilities();
    return std::accumulate(p.begin(), p.end(), 0.0);
}

bool DensityMatrix::isValid(double tolerance) const {
    if (std::abs(trace() - 1.0) > tolerance) return false;
    const double pur = purity();
    return pur >= 1.0 / (double)getDimension() - tolerance && pur <= 1.0 + tolerance;
}

DensityMatrixSimulator::DensityMatrixSimulator(int n_qubits, const NoiseModel& noise)
    : rho_(n_qubits), noise_model_(noise), rng_(std::random_device{}()) {}

void DensityMatrixSimulator::run(const Circuit& circuit) {
    const std::vector<qsim_gate> gates = detail::toAbi(circuit);
    std::vector<qsim_noise_channel> ch;  // a global channel (empty qubit list) -> qubit -1
    for (const NoiseChannel& c : noise_model_.getChannels()) {
        if (c.qubits.empty()) ch.push_back(qsim_noise_channel{static_cast<int>(c.type), -1, c.probability});
        for (int q : c.qubits) ch.push_back(qsim_noise_channel{static_cast<int>(c.type), q, c.probability});
    }
    check(qsim_dm_run(rho_.state().handle(), rho_.getNumQubits(), gates.data(), gates.size(),
                      ch.data(), ch.size(), QSIM_RUN_FUSED | (reference_y_ ? QSIM_DM_REFERENCE_Y : 0)));
}

void DensityMatrixSimulator::applyGate(const GateOp& gate) {
    const qsim_gate g = detail::toAbi(gate);
    check(qsim_dm_run(rho_.state().handle(), rho_.getNumQubits(), &g, 1, nullptr, 0,
                      QSIM_RUN_PER_GATE | (reference_y_ ? QSIM_DM_REFERENCE_Y : 0)));
}

int DensityMatrixSimulator::measureQubit(int qubit) {
    const int n = rho_.getNumQubits();
    if (qubit < 0 || qubit >= n) throw std::invalid_argument("Qubit index out of range");
    const std::vector<double> p = rho_.getProbabilities();
    double p1 = 0.0;
    for (size_t i = 0; i < p.size(); ++i)
        if ((i >> qubit) & 1) p1 += p[i];
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    const int result = dist(rng_) < p1 ? 1 : 0;
    const double pr = result ? p1 : 1.0 - p1;
    check(qsim_state_collapse(rho_.state().handle(), qubit + n, result, 1.0 / pr));
    check(qsim_state_collapse(rho_.state().handle(), qubit, result, 1.0));
    return result;
}

}  // namespace qsim
