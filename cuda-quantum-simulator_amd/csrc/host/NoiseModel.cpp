// NoiseModel.cpp — noise-channel container (reference src/NoiseModel.cu:24-101) and the
// BatchedSimulator front end (src/NoiseModel.cu:653-972) over the qsim_batch C ABI.
#include "qsim/NoiseModel.hpp"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <stdexcept>

#include "abi_util.hpp"

namespace qsim {

using detail::check;

// ---- NoiseModel: the per-qubit forms store one single-qubit channel per listed qubit; the
// "global" forms store an empty qubit list (which the Monte-Carlo simulators apply to no qubit).
void NoiseModel::addPerQubit(NoiseType t, const std::vector<int>& qubits, double p) {
    for (int q : qubits) channels_.emplace_back(t, std::vector<int>{q}, p);
}
void NoiseModel::addDepolarizing(const std::vector<int>& q, double p) { addPerQubit(NoiseType::Depolarizing, q, p); }
void NoiseModel::addAmplitudeDamping(const std::vector<int>& q, double g) { addPerQubit(NoiseType::AmplitudeDamping, q, g); }
void NoiseModel::addPhaseDamping(const std::vector<int>& q, double g) { addPerQubit(NoiseType::PhaseDamping, q, g); }
void NoiseModel::addBitFlip(const std::vector<int>& q, double p) { addPerQubit(NoiseType::BitFlip, q, p); }
void NoiseModel::addPhaseFlip(const std::vector<int>& q, double p) { addPerQubit(NoiseType::PhaseFlip, q, p); }
void NoiseModel::addBitPhaseFlip(const std::vector<int>& q, double p) { addPerQubit(NoiseType::BitPhaseFlip, q, p); }

void NoiseModel::addDepolarizing(double p) { channels_.emplace_back(NoiseType::Depolarizing, std::vector<int>{}, p); }
void NoiseModel::addAmplitudeDamping(double g) { channels_.emplace_back(NoiseType::AmplitudeDamping, std::vector<int>{}, g); }
void NoiseModel::addPhaseDamping(double g) { channels_.emplace_back(NoiseType::PhaseDamping, std::vector<int>{}, g); }
void NoiseModel::addBitFlip(double p) { channels_.emplace_back(NoiseType::BitFlip, std::vector<int>{}, p); }
void NoiseModel::addPhaseFlip(double p) { channels_.emplace_back(NoiseType::PhaseFlip, std::vector<int>{}, p); }
void NoiseModel::addBitPhaseFlip(double p) { channels_.emplace_back(NoiseType::BitPhaseFlip, std::vector<int>{}, p); }

static std::vector<int> allQubits(int n) {
    std::vector<int> v(n);
    std::iota(v.begin(), v.end(), 0);
    return v;
}
void NoiseModel::addDepolarizingAll(int n, double p) { addDepolarizing(allQubits(n), p); }
void NoiseModel::addAmplitudeDampingAll(int n, double g) { addAmplitudeDamping(allQubits(n), g); }
void NoiseModel::addPhaseDampingAll(int n, double g) { addPhaseDamping(allQubits(n), g); }

// ---- NoisySimulator (src/NoiseModel.cu:320-651)
NoisySimulator::NoisySimulator(int num_qubits, const NoiseModel& noise_model)
    : state_(num_qubits), noise_model_(noise_model) {
    setSeed(std::random_device{}());
}
NoisySimulator::NoisySimulator(int num_qubits) : NoisySimulator(num_qubits, NoiseModel{}) {}

void NoisySimulator::setSeed(unsigned int seed) {
    rng_.seed(seed);
    seed_ = seed;
    counter_ = 0;
}

void NoisySimulator::reset() { state_.initializeZero(); }

void NoisySimulator::run(const Circuit& circuit) {
    if (circuit.getNumQubits() != state_.getNumQubits())
        throw std::invalid_argument("Circuit qubit count doesn't match simulator");
    const std::vector<qsim_gate> gates = detail::toAbi(circuit);
    std::vector<qsim_noise_channel> ch;
    for (const NoiseChannel& c : noise_model_.getChannels())
        for (int q : c.qubits) ch.push_back(qsim_noise_channel{static_cast<int>(c.type), q, c.probability});
    check(qsim_noisy_run(state_.handle(), gates.data(), gates.size(), ch.data(), ch.size(), seed_,
                         &counter_, QSIM_RUN_FUSED));
}

void NoisySimulator::applyGate(const GateOp& gate) {
    const qsim_gate g = detail::toAbi(gate);
    check(qsim_apply_gate(state_.handle(), &g));
}

void NoisySimulator::applyNoise(const NoiseChannel& channel) {
    for (int q : channel.qubits) applyNoiseToQubit(channel.type, q, channel.probability);
}

void NoisySimulator::applyNoiseToQubit(NoiseType type, int qubit, double probability) {
    check(qsim_noise_apply(state_.handle(), static_cast<int>(type), qubit, probability, seed_, counter_));
    ++counter_;
}

std::vector<int> NoisySimulator::sample(int n_shots) {
    // src/NoiseModel.cu:599-613: uniforms drawn in shot order; CDF + lower_bound on the device
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    std::vector<int> out(n_shots > 0 ? n_shots : 0);
    if (out.empty()) return out;
    std::vector<double> u(out.size());
    for (double& r : u) r = dist(rng_);
    std::vector<int64_t> idx(out.size());
    check(qsim_state_sample(state_.handle(), u.data(), n_shots, idx.data()));
    for (size_t i = 0; i < out.size(); ++i) out[i] = static_cast<int>(idx[i]);
    return out;
}

int NoisySimulator::measureQubit(int qubit) {
    double p0 = 0.0, total = 0.0;
    check(qsim_state_prob_bit_zero(state_.handle(), qubit, &p0));
    check(qsim_state_total_probability(state_.handle(), &total));
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    const int result = dist(rng_) < p0 ? 0 : 1;
    const double kept = result == 0 ? p0 : total - p0;
    check(qsim_state_collapse(state_.handle(), qubit, result, 1.0 / std::sqrt(kept)));
    return result;
}

// ---- BatchedSimulator
BatchedSimulator::BatchedSimulator(int num_qubits, int batch_size)
    : num_qubits_(num_qubits), batch_size_(batch_size), rng_(std::random_device{}()) {
    check(qsim_batch_create(num_qubits, batch_size, &h_));
}

BatchedSimulator::BatchedSimulator(int num_qubits, int batch_size, const NoiseModel& noise_model)
    : BatchedSimulator(num_qubits, batch_size) {
    noise_model_ = noise_model;
}

BatchedSimulator::~BatchedSimulator() {
    if (h_) qsim_batch_destroy(h_);
}

BatchedSimulator::BatchedSimulator(BatchedSimulator&& o) noexcept
    : num_qubits_(o.num_qubits_), batch_size_(o.batch_size_), h_(o.h_),
      noise_model_(std::move(o.noise_model_)), gate_set_(o.gate_set_), rng_(o.rng_) {
    o.h_ = nullptr;
}

BatchedSimulator& BatchedSimulator::operator=(BatchedSimulator&& o) noexcept {
    if (this != &o) {
        if (h_) qsim_batch_destroy(h_);
        num_qubits_ = o.num_qubits_;
        batch_size_ = o.batch_size_;
        h_ = o.h_;
        noise_model_ = std::move(o.noise_model_);
        gate_set_ = o.gate_set_;
        rng_ = o.rng_;
        o.h_ = nullptr;
    }
    return *this;
}

void BatchedSimulator::setSeed(unsigned int seed) {
    rng_.seed(seed);
    check(qsim_batch_set_seed(h_, seed));
}

void BatchedSimulator::setTrajectoryOffset(unsigned long long first) {
    check(qsim_batch_set_trajectory_offset(h_, first));
}

void BatchedSimulator::reset() { check(qsim_batch_reset(h_)); }

void BatchedSimulator::run(const Circuit& circuit) {
    if (circuit.getNumQubits() != num_qubits_)
        throw std::invalid_argument("Circuit qubit count doesn't match simulator");
    const std::vector<qsim_gate> gates = detail::toAbi(circuit);
    std::vector<qsim_noise_channel> ch;
    for (const NoiseChannel& c : noise_model_.getChannels())
        for (int q : c.qubits) ch.push_back(qsim_noise_channel{static_cast<int>(c.type), q, c.probability});
    check(qsim_batch_run(h_, gates.data(), gates.size(), ch.data(), ch.size(),
                         (gate_set_ == BatchedGateSet::Reference ? QSIM_BATCH_REFERENCE_GATESET
                                                                 : QSIM_BATCH_FULL_GATESET) |
                             (noise_ == BatchedNoise::Reference ? QSIM_BATCH_REFERENCE_NOISE : 0)));
}

std::vector<double> BatchedSimulator::getAverageProbabilities() const {
    std::vector<double> p(size_t(1) << num_qubits_);
    check(qsim_batch_avg_probabilities(h_, p.data()));
    return p;
}

std::vector<double> BatchedSimulator::getProbabilities(int t) const {
    if (t < 0 || t >= batch_size_) throw std::out_of_range("Invalid trajectory index");
    std::vector<double> p(size_t(1) << num_qubits_);
    check(qsim_batch_traj_probabilities(h_, t, p.data()));
    return p;
}

// Uniforms of src/NoiseModel.cu:944-954, in its order: trajectory-major, shot by shot.
static std::vector<double> draw_uniforms(std::mt19937& rng, int batch, int n_shots) {
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    std::vector<double> u((size_t)batch * (size_t)n_shots);
    for (double& r : u) r = dist(rng);
    return u;
}

std::vector<std::vector<int>> BatchedSimulator::sample(int n_shots) {
    if (n_shots < 0) throw std::invalid_argument("n_shots must be non-negative");
    std::vector<std::vector<int>> out(n_shots, std::vector<int>(batch_size_));
    if (n_shots == 0) return out;
    const std::vector<double> u = draw_uniforms(rng_, batch_size_, n_shots);
    std::vector<int64_t> idx(u.size());
    check(qsim_batch_sample(h_, u.data(), n_shots, idx.data()));  // per-trajectory device CDF
    for (int t = 0; t < batch_size_; ++t)
        for (int s = 0; s < n_shots; ++s) out[s][t] = static_cast<int>(idx[(size_t)t * n_shots + s]);
    return out;
}

std::vector<int> BatchedSimulator::getHistogram(int n_shots) {
    if (n_shots < 0) throw std::invalid_argument("n_shots must be non-negative");
    const std::vector<double> u = draw_uniforms(rng_, batch_size_, n_shots);
    std::vector<int64_t> h(size_t(1) << num_qubits_, 0);
    check(qsim_batch_histogram(h_, u.data(), n_shots, h.data()));
    return std::vector<int>(h.begin(), h.end());
}

}  // namespace qsim
