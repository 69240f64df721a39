// Simulator.hpp — circuit execution on one MI355X (reference include/Simulator.hpp:53-85).
//
// Drop-in for the reference `Simulator`: same constructor, run/applyGate, readout, sampling and
// measurement signatures and exception types.  run() is asynchronous like the reference
// (src/Simulator.cu:95-97); every readout synchronizes.  By default run() hands the whole circuit
// to the engine's fused-pass planner (RunMode::Fused); RunMode::PerGate reproduces the
// reference's one-launch-per-gate execution.
//
// CPUSimulator (reference include/Simulator.hpp:91-112, src/Simulator.cu:195-345) is this
// library's own host implementation (csrc/host/CPUSimulator.cpp: gate table + thread pool over
// the amplitude pairs), kept for code that compares against the CPU (benchmark_scaling.cu:85).
// It is not the parity oracle (oracle/ is test infrastructure and is never linked here).
#pragma once

#include <complex>
#include <cstdint>
#include <memory>
#include <random>
#include <vector>

#include "Circuit.hpp"
#include "StateVector.hpp"

namespace qsim {

enum class RunMode { PerGate, Fused };

class Simulator {
public:
    explicit Simulator(int num_qubits);

    void reset();
    void run(const Circuit& circuit);  // std::invalid_argument on qubit-count mismatch
    // run() of each circuit in turn as ONE engine run (no reference counterpart): the planner
    // sees their gates together, so a fused pass may hold the end of one and the start of the
    // next (consecutive W-HC circuits at 30 qubits: 2.5-2.75 passes each instead of 4).
    void runSequence(const std::vector<Circuit>& circuits);
    void applyGate(const GateOp& gate);

    std::vector<std::complex<double>> getStateVector() const;
    std::vector<double> getProbabilities() const;

    std::vector<int> sample(int n_shots);  // without collapse
    int measureQubit(int qubit);           // reference semantics: StateVector::measure (F2)

    int getNumQubits() const { return state_.getNumQubits(); }
    size_t getStateSize() const { return state_.getSize(); }

    void setRunMode(RunMode m) { mode_ = m; }
    RunMode getRunMode() const { return mode_; }
    void setSeed(unsigned int seed) { state_.setSeed(seed); }
    void synchronize() const;
    StateVector& state() { return state_; }
    const StateVector& state() const { return state_; }

private:
    StateVector state_;
    RunMode mode_ = RunMode::Fused;
};

// Which gates CPUSimulator::applyGate acts on.  Reference: exactly the reference CPU path —
// every 1-qubit gate, CNOT, CZ and SWAP; CRY, CRZ and Toffoli are silent no-ops
// (src/Simulator.cu:214-220, 313-314).  Full: CRY / CRZ / Toffoli as the GPU kernels
// define them (src/Gates.cu:322-410), so CPU and GPU agree on every circuit.
enum class CpuGateSet { Reference, Full };

class CPUSimulator {
public:
    explicit CPUSimulator(int num_qubits, CpuGateSet gates = CpuGateSet::Reference);

    void reset();
    void run(const Circuit& circuit);  // std::invalid_argument on qubit-count mismatch
    void applyGate(const GateOp& gate);

    std::vector<std::complex<double>> getStateVector() const { return state_; }
    std::vector<double> getProbabilities() const;
    std::vector<int> sample(int n_shots);

    int getNumQubits() const { return num_qubits_; }
    size_t getStateSize() const { return state_.size(); }

    // Worker threads for the pair loops (a persistent pool; default min(hardware threads, 16);
    // states below 2^17 amplitudes always run on the calling thread).  1 = the reference's single
    // core.
    void setThreads(int threads);
    int getThreads() const { return threads_; }
    void setSeed(unsigned int seed) { rng_.seed(seed); }

private:
    int num_qubits_;
    CpuGateSet gate_set_;
    int threads_;
    std::vector<std::complex<double>> state_;
    std::mt19937 rng_;
    struct Pool;
    std::shared_ptr<Pool> pool_;
};

}  // namespace qsim
