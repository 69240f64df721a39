// Circuit.hpp — circuit IR with the reference's fluent gate API.
//
// Same names, argument order, numbering and exceptions as the reference include/Circuit.hpp:
// GateType (:42-59, numbering shared with QSIM_GATE_* of qsim_hip.h), GateOp{type, qubits,
// parameter} (:64-84), Circuit (:89-131) and the factories (:138-144).  Host-only (g++).
#pragma once

#include <string>
#include <vector>

namespace qsim {

enum class GateType {
    X, Y, Z, H, S, T, Sdag, Tdag, Rx, Ry, Rz,
    CNOT, CZ, CRY, CRZ, SWAP,
    Toffoli
};

struct GateOp {
    GateType type;
    std::vector<int> qubits;  // [target] | [control, target] | [q1, q2] | [c1, c2, target]
    double parameter;         // radians for Rx/Ry/Rz/CRY/CRZ

    GateOp(GateType t, int q) : type(t), qubits{q}, parameter(0.0) {}
    GateOp(GateType t, int q, double p) : type(t), qubits{q}, parameter(p) {}
    GateOp(GateType t, int q1, int q2) : type(t), qubits{q1, q2}, parameter(0.0) {}
    GateOp(GateType t, int q1, int q2, double p) : type(t), qubits{q1, q2}, parameter(p) {}
    GateOp(GateType t, int q1, int q2, int q3) : type(t), qubits{q1, q2, q3}, parameter(0.0) {}
};

class Circuit {
public:
    explicit Circuit(int num_qubits);  // std::invalid_argument outside [1, 30]

    Circuit& x(int qubit);
    Circuit& y(int qubit);
    Circuit& z(int qubit);
    Circuit& h(int qubit);
    Circuit& s(int qubit);
    Circuit& t(int qubit);
    Circuit& sdag(int qubit);
    Circuit& tdag(int qubit);
    Circuit& rx(int qubit, double theta);
    Circuit& ry(int qubit, double theta);
    Circuit& rz(int qubit, double theta);
    Circuit& cnot(int control, int target);
    Circuit& cx(int control, int target) { return cnot(control, target); }
    Circuit& cz(int control, int target);
    Circuit& cry(int control, int target, double theta);
    Circuit& crz(int control, int target, double theta);
    Circuit& swap(int qubit1, int qubit2);
    Circuit& toffoli(int control1, int control2, int target);
    Circuit& ccx(int control1, int control2, int target) { return toffoli(control1, control2, target); }

    int getNumQubits() const { return num_qubits_; }
    const std::vector<GateOp>& getGates() const { return gates_; }
    size_t getDepth() const;
    size_t getGateCount() const { return gates_.size(); }

    void clear() { gates_.clear(); }
    std::string toString() const;

private:
    int num_qubits_;
    std::vector<GateOp> gates_;

    Circuit& add(GateType t, std::initializer_list<int> qubits, double param, bool has_param);
};

const char* gateTypeName(GateType t);

Circuit createBellCircuit();
Circuit createGHZCircuit(int num_qubits);
// Reference factory: mt19937(seed); per gate uniform_int(0,3) -> {H, X, CNOT, Rz}, then the
// qubit(s) (CNOT redraws q2 != q1), then the Rz angle uniform_real(0, 2*pi) (src/Circuit.cpp:252-282).
Circuit createRandomCircuit(int num_qubits, int depth, unsigned int seed = 42);
// Benchmark workload W-HC: same draw order, gate type uniform_int(0,1) -> {H, CNOT}.
Circuit createRandomHCCircuit(int num_qubits, int depth, unsigned int seed = 42);
// Benchmark workload W-REF: h(i % n) for i < 100 plus cnot(i%n, (i+1)%n) when i % 5 == 0
// (reference benchmarks/benchmark_scaling.cu:69-76; 120 gates).
Circuit createScalingBenchmarkCircuit(int num_qubits);

}  // namespace qsim
