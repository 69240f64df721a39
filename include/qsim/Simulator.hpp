// Simulator.hpp — circuit execution on one MI355X (reference include/Simulator.hpp:53-85).
//
// Drop-in for the reference `Simulator`: same constructor, run/applyGate, readout, sampling and
// measurement signatures and exception types.  run() is asynchronous like the reference
// (src/Simulator.cu:95-97); every readout synchronizes.  By default run() hands the whole circuit
// to the engine's fused-pass planner (RunMode::Fused); RunMode::PerGate reproduces the
// reference's one-launch-per-gate execution.  The reference's CPUSimulator is the parity oracle
// and lives in oracle/ (test infrastructure), not in this library.
#pragma once

#include <complex>
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

}  // namespace qsim
