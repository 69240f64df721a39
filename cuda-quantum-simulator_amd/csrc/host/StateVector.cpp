// StateVector.cpp — C++ owner of a qsim_state handle (reference src/StateVector.cu:130-342).
#include "qsim/StateVector.hpp"

#include <cmath>
#include <stdexcept>
#include <string>
#include <utility>

#include "abi_util.hpp"
#include "qsim/Constants.hpp"

namespace qsim {

using detail::check;

StateVector::StateVector(int num_qubits)
    : num_qubits_(num_qubits), size_(0), h_(nullptr) {
    if (!isValidQubitCount(num_qubits))
        throw std::invalid_argument("Number of qubits must be between " +
                                    std::to_string(device_config::MIN_QUBITS) + " and " +
                                    std::to_string(device_config::MAX_QUBITS));
    check(qsim_state_create(num_qubits, &h_));  // allocates and initializes |0...0>
    size_ = size_t(1) << num_qubits;
}

StateVector::~StateVector() { release(); }

void StateVector::release() {
    if (h_) qsim_state_destroy(h_);
    h_ = nullptr;
}

StateVector::StateVector(StateVector&& o) noexcept
    : num_qubits_(o.num_qubits_), size_(o.size_), h_(o.h_), seeded_(o.seeded_), rng_(o.rng_) {
    o.h_ = nullptr;
    o.size_ = 0;
    o.num_qubits_ = 0;
}

StateVector& StateVector::operator=(StateVector&& o) noexcept {
    if (this != &o) {
        release();
        num_qubits_ = o.num_qubits_;
        size_ = o.size_;
        h_ = o.h_;
        seeded_ = o.seeded_;
        rng_ = o.rng_;
        o.h_ = nullptr;
        o.size_ = 0;
        o.num_qubits_ = 0;
    }
    return *this;
}

void StateVector::applyMatrix1Q(int target, const std::complex<double> (&m)[4],
                                const std::vector<int>& controls) {
    double mm[8];
    for (int i = 0; i < 4; ++i) {
        mm[2 * i] = m[i].real();
        mm[2 * i + 1] = m[i].imag();
    }
    check(qsim_apply_matrix1q(h_, target, mm, controls.empty() ? nullptr : controls.data(),
                              (int)controls.size()));
}

void StateVector::applyMatrix(const std::vector<int>& targets, const std::vector<std::complex<double>>& m,
                              const std::vector<int>& controls) {
    const size_t dim = size_t(1) << targets.size();
    if (targets.empty() || targets.size() > 8 || m.size() != dim * dim)
        throw std::invalid_argument("matrix must be 2^k x 2^k for 1 <= k <= 8 targets");
    std::vector<double> mm(2 * m.size());
    for (size_t i = 0; i < m.size(); ++i) {
        mm[2 * i] = m[i].real();
        mm[2 * i + 1] = m[i].imag();
    }
    check(qsim_apply_matrix(h_, targets.data(), (int)targets.size(), mm.data(),
                            controls.empty() ? nullptr : controls.data(), (int)controls.size()));
}

void StateVector::initializeZero() { check(qsim_state_init_zero(h_)); }

void StateVector::initializeBasis(size_t basis_idx) {
    if (basis_idx >= size_) throw std::invalid_argument("Basis index out of range");
    check(qsim_state_init_basis(h_, basis_idx));
}

Amplitude* StateVector::devicePtr() {
    void* p = nullptr;
    if (h_) check(qsim_state_device_ptr(h_, &p));
    return static_cast<Amplitude*>(p);
}
const Amplitude* StateVector::devicePtr() const {
    return const_cast<StateVector*>(this)->devicePtr();
}

std::vector<std::complex<double>> StateVector::toHost() const {
    std::vector<std::complex<double>> out(size_);
    // std::complex<double> is layout-compatible with double[2] ([complex.numbers.general]).
    check(qsim_state_to_host(h_, reinterpret_cast<double*>(out.data())));
    return out;
}

void StateVector::fromHost(const std::vector<std::complex<double>>& a) {
    if (a.size() != size_) throw std::invalid_argument("amplitude count does not match 2^n");
    check(qsim_state_from_host(h_, reinterpret_cast<const double*>(a.data())));
}

std::vector<double> StateVector::getProbabilities() const {
    std::vector<double> p(size_);
    check(qsim_state_probabilities(h_, p.data()));
    return p;
}

double StateVector::getTotalProbability() const {
    double t = 0.0;
    check(qsim_state_total_probability(h_, &t));
    return t;
}

double StateVector::maxAbsDiff(const StateVector& other) const {
    double d = 0.0;
    check(qsim_state_max_abs_diff(h_, other.h_, &d));
    return d;
}

size_t StateVector::getDeviceMemoryBytes() const {
    uint64_t b = 0;
    check(qsim_state_memory_bytes(h_, &b));
    return (size_t)b;
}

bool StateVector::isNormalized(double tolerance) const {
    return std::abs(getTotalProbability() - 1.0) <= tolerance;
}

void StateVector::assertNormalized(double tolerance) const {
    const double t = getTotalProbability();
    if (std::abs(t - 1.0) > tolerance)
        throw std::runtime_error("State vector not normalized: total probability = " +
                                 std::to_string(t) + " (expected 1.0, tolerance = " +
                                 std::to_string(tolerance) + ")");
}

void StateVector::setSeed(unsigned int seed) {
    rng_.seed(seed);
    seeded_ = true;
}

std::vector<double> StateVector::uniforms(int count) {
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    std::vector<double> u(count);
    if (seeded_) {
        for (double& x : u) x = dist(rng_);
    } else {
        std::random_device rd;
        std::mt19937 rng(rd());
        for (double& x : u) x = dist(rng);
    }
    return u;
}

int StateVector::measureBit(int bit) {
    if (bit < 0 || bit >= num_qubits_)
        throw std::invalid_argument("Qubit index " + std::to_string(bit) + " out of range [0, " +
                                    std::to_string(num_qubits_ - 1) + "]");
    double p0 = 0.0;
    check(qsim_state_prob_bit_zero(h_, bit, &p0));
    const double r = uniforms(1)[0];
    const int result = r < p0 ? 0 : 1;
    const double pr = result == 0 ? p0 : 1.0 - p0;
    if (pr < 1e-15)
        throw std::runtime_error("Measurement result " + std::to_string(result) +
                                 " has zero probability - state may be corrupted");
    check(qsim_state_collapse(h_, bit, result, 1.0 / std::sqrt(pr)));
    return result;
}

int StateVector::measure(int qubit) {
    if (qubit < 0 || qubit >= num_qubits_)
        throw std::invalid_argument("Qubit index " + std::to_string(qubit) + " out of range [0, " +
                                    std::to_string(num_qubits_ - 1) + "]");
    return measureBit(num_qubits_ - 1 - qubit);  // big-endian, src/StateVector.cu:87-89 (F2)
}

std::vector<int> StateVector::sample(int n_shots) {
    if (n_shots <= 0) throw std::invalid_argument("n_shots must be positive");
    const std::vector<double> u = uniforms(n_shots);
    std::vector<int64_t> idx(n_shots);
    check(qsim_state_sample(h_, u.data(), n_shots, idx.data()));
    return std::vector<int>(idx.begin(), idx.end());
}

}  // namespace qsim
