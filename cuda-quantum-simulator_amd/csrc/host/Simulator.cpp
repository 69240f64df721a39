// Simulator.cpp — reference Simulator (src/Simulator.cu:22-189) over the C ABI.
#include "qsim/Simulator.hpp"

#include <stdexcept>

#include "abi_util.hpp"

namespace qsim {

using detail::check;

Simulator::Simulator(int num_qubits) : state_(num_qubits) {}

void Simulator::reset() { state_.initializeZero(); }

void Simulator::run(const Circuit& circuit) {
    if (circuit.getNumQubits() != state_.getNumQubits())
        throw std::invalid_argument("Circuit qubit count doesn't match simulator");
    const std::vector<qsim_gate> gates = detail::toAbi(circuit);
    check(qsim_run(state_.handle(), gates.data(), gates.size(),
                   mode_ == RunMode::Fused ? QSIM_RUN_FUSED : QSIM_RUN_PER_GATE));
}

void Simulator::runSequence(const std::vector<Circuit>& circuits) {
    std::vector<qsim_gate> gates;
    for (const Circuit& c : circuits) {
        if (c.getNumQubits() != state_.getNumQubits())
            throw std::invalid_argument("Circuit qubit count doesn't match simulator");
        const std::vector<qsim_gate> g = detail::toAbi(c);
        gates.insert(gates.end(), g.begin(), g.end());
    }
    check(qsim_run(state_.handle(), gates.data(), gates.size(),
                   mode_ == RunMode::Fused ? QSIM_RUN_FUSED : QSIM_RUN_PER_GATE));
}

void Simulator::applyGate(const GateOp& gate) {
    const qsim_gate g = detail::toAbi(gate);
    check(qsim_apply_gate(state_.handle(), &g));
}

std::vector<std::complex<double>> Simulator::getStateVector() const { return state_.toHost(); }
std::vector<double> Simulator::getProbabilities() const { return state_.getProbabilities(); }

std::vector<int> Simulator::sample(int n_shots) {
    if (n_shots == 0) return {};
    return state_.sample(n_shots);
}

int Simulator::measureQubit(int qubit) { return state_.measure(qubit); }

void Simulator::synchronize() const { check(qsim_state_sync(state_.handle())); }

}  // namespace qsim
