// NoiseModel.hpp — noise channels and the batched-trajectory simulator.
//
// NoiseType / NoiseChannel / NoiseModel mirror the reference include/NoiseModel.cuh:46-126
// (including the "global" overloads that store an empty qubit list and therefore act on no qubit
// in the Monte-Carlo simulators).  BatchedSimulator mirrors :231-297.
#pragma once

#include <algorithm>
#include <complex>
#include <cstdint>
#include <cstddef>
#include <random>
#include <vector>

#include "Circuit.hpp"
#include "StateVector.hpp"

struct qsim_batch;

namespace qsim {

enum class NoiseType { Depolarizing, AmplitudeDamping, PhaseDamping, BitFlip, PhaseFlip, BitPhaseFlip };

struct NoiseChannel {
    NoiseType type;
    std::vector<int> qubits;
    double probability;
    NoiseChannel(NoiseType t, std::vector<int> q, double p) : type(t), qubits(std::move(q)), probability(p) {}
};

class NoiseModel {
public:
    NoiseModel() = default;

    void addDepolarizing(const std::vector<int>& qubits, double probability);
    void addAmplitudeDamping(const std::vector<int>& qubits, double gamma);
    void addPhaseDamping(const std::vector<int>& qubits, double gamma);
    void addBitFlip(const std::vector<int>& qubits, double probability);
    void addPhaseFlip(const std::vector<int>& qubits, double probability);
    void addBitPhaseFlip(const std::vector<int>& qubits, double probability);

    void addDepolarizing(double probability);
    void addAmplitudeDamping(double gamma);
    void addPhaseDamping(double gamma);
    void addBitFlip(double probability);
    void addPhaseFlip(double probability);
    void addBitPhaseFlip(double probability);

    void addDepolarizingAll(int num_qubits, double probability);
    void addAmplitudeDampingAll(int num_qubits, double gamma);
    void addPhaseDampingAll(int num_qubits, double gamma);

    const std::vector<NoiseChannel>& getChannels() const { return channels_; }
    bool hasNoise() const { return !channels_.empty(); }
    void clear() { channels_.clear(); }
    bool channelAppliesToQubit(const NoiseChannel& channel, int qubit) const {
        return channel.qubits.empty() ||
               std::find(channel.qubits.begin(), channel.qubits.end(), qubit) != channel.qubits.end();
    }

private:
    std::vector<NoiseChannel> channels_;
    void addPerQubit(NoiseType t, const std::vector<int>& qubits, double p);
};

// Reference NoisySimulator (include/NoiseModel.cuh:139-214): Monte-Carlo noise on one state.
// run() applies each gate and then every channel entry (one per-pair noise pass each, reference
// kernels src/NoiseModel.cu:115-314); global channels act on no qubit (F6).  measureQubit uses
// index bit `qubit` (LSB-first, :615-651).
class NoisySimulator {
public:
    NoisySimulator(int num_qubits, const NoiseModel& noise_model);
    explicit NoisySimulator(int num_qubits);
    NoisySimulator(const NoisySimulator&) = delete;
    NoisySimulator& operator=(const NoisySimulator&) = delete;
    NoisySimulator(NoisySimulator&&) noexcept = default;
    NoisySimulator& operator=(NoisySimulator&&) noexcept = default;

    void setNoiseModel(const NoiseModel& noise_model) { noise_model_ = noise_model; }
    const NoiseModel& getNoiseModel() const { return noise_model_; }
    void setSeed(unsigned int seed);
    void reset();
    void run(const Circuit& circuit);
    void applyGate(const GateOp& gate);
    void applyNoise(const NoiseChannel& channel);
    void applyNoiseToQubit(NoiseType type, int qubit, double probability);
    std::vector<std::complex<double>> getStateVector() const { return state_.toHost(); }
    std::vector<double> getProbabilities() const { return state_.getProbabilities(); }
    std::vector<int> sample(int n_shots);
    int measureQubit(int qubit);
    int getNumQubits() const { return state_.getNumQubits(); }
    size_t getStateSize() const { return state_.getSize(); }
    StateVector& state() { return state_; }

private:
    StateVector state_;
    NoiseModel noise_model_;
    uint64_t seed_ = 0, counter_ = 0;
    std::mt19937 rng_;
};

// Gate set applied per trajectory.  Reference: only X/Y/Z/H and CNOT act, everything else is
// silently skipped (src/NoiseModel.cu:742-763, 808-812).  Full: every GateType.
enum class BatchedGateSet { Full, Reference };

// Noise process of the batched trajectories.  Reference (default, the drop-in behaviour): the
// reference's per-amplitude-pair process — Depolarizing entries only, one draw per pair per pass
// after every gate (applyBatchedDepolarizingKernel, src/NoiseModel.cu:834-892).
// Physical (opt-in): one draw per trajectory, channel and gate — the Kraus channel on a
// pure-state trajectory, all four Pauli channel types, run as Pauli frames inside fused passes.
enum class BatchedNoise { Physical, Reference };

class BatchedSimulator {
public:
    BatchedSimulator(int num_qubits, int batch_size);
    BatchedSimulator(int num_qubits, int batch_size, const NoiseModel& noise_model);
    ~BatchedSimulator();
    BatchedSimulator(const BatchedSimulator&) = delete;
    BatchedSimulator& operator=(const BatchedSimulator&) = delete;
    BatchedSimulator(BatchedSimulator&& o) noexcept;
    BatchedSimulator& operator=(BatchedSimulator&& o) noexcept;

    void setNoiseModel(const NoiseModel& noise_model) { noise_model_ = noise_model; }
    void setSeed(unsigned int seed);
    // Trajectory sharding (one object per GPU): this object's trajectories are
    // [first, first + batch_size) of a larger ensemble; noise draws use the global index.
    void setTrajectoryOffset(unsigned long long first);
    void reset();
    void run(const Circuit& circuit);

    std::vector<double> getAverageProbabilities() const;
    std::vector<double> getProbabilities(int trajectory_idx) const;  // std::out_of_range
    std::vector<std::vector<int>> sample(int n_shots);                // [shot][trajectory]
    std::vector<int> getHistogram(int n_shots);

    int getNumQubits() const { return num_qubits_; }
    int getBatchSize() const { return batch_size_; }
    size_t getTotalMemoryBytes() const { return (size_t)batch_size_ * (1ULL << num_qubits_) * 16u; }

    void setGateSet(BatchedGateSet g) { gate_set_ = g; }
    void setNoiseSemantics(BatchedNoise m) { noise_ = m; }
    // Both reference behaviours at once (gate set X/Y/Z/H/CNOT, per-pair depolarizing noise).
    void setReferenceCompatible() {
        gate_set_ = BatchedGateSet::Reference;
        noise_ = BatchedNoise::Reference;
    }
    qsim_batch* handle() const { return h_; }

private:
    int num_qubits_;
    int batch_size_;
    qsim_batch* h_ = nullptr;
    NoiseModel noise_model_;
    BatchedGateSet gate_set_ = BatchedGateSet::Full;
    BatchedNoise noise_ = BatchedNoise::Reference;
    std::mt19937 rng_;  // host sampling stream (reference rng_, src/NoiseModel.cu:661)
};

}  // namespace qsim
