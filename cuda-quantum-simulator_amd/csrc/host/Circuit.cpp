// Circuit.cpp — circuit IR, validation and factories (behaviour of reference src/Circuit.cpp).
//
// Validation rules and exception types: constructor std::invalid_argument outside [1,30]
// (:16-24); bad index std::out_of_range (:26-31); repeated qubit std::invalid_argument
// (:33-48); non-finite angle std::invalid_argument (:51-55).  Depth = longest chain of gates
// sharing a qubit (:183-201).  The random factories consume the mt19937 stream in the
// reference's draw order (type, q1, [q2 redraws], [angle]) so gate lists match libstdc++ builds.
#include "qsim/Circuit.hpp"

#include <algorithm>
#include <cmath>
#include <random>
#include <sstream>
#include <stdexcept>

#include "qsim/Constants.hpp"

namespace qsim {

namespace {
struct GateInfo {
    const char* name;
    int arity;
    bool param;
};
const GateInfo kGateInfo[] = {
    {"X", 1, false},    {"Y", 1, false},    {"Z", 1, false},    {"H", 1, false},
    {"S", 1, false},    {"T", 1, false},    {"Sdag", 1, false}, {"Tdag", 1, false},
    {"Rx", 1, true},    {"Ry", 1, true},    {"Rz", 1, true},    {"CNOT", 2, false},
    {"CZ", 2, false},   {"CRY", 2, true},   {"CRZ", 2, true},   {"SWAP", 2, false},
    {"Toffoli", 3, false},
};
const GateInfo& info(GateType t) { return kGateInfo[static_cast<int>(t)]; }
}  // namespace

const char* gateTypeName(GateType t) { return info(t).name; }

Circuit::Circuit(int num_qubits) : num_qubits_(num_qubits) {
    if (!isValidQubitCount(num_qubits))
        throw std::invalid_argument("Number of qubits must be between " +
                                    std::to_string(device_config::MIN_QUBITS) + " and " +
                                    std::to_string(device_config::MAX_QUBITS));
}

Circuit& Circuit::add(GateType t, std::initializer_list<int> qubits, double param, bool has_param) {
    for (int q : qubits)
        if (!isValidQubit(q, num_qubits_))
            throw std::out_of_range("Qubit index " + std::to_string(q) + " out of range [0, " +
                                    std::to_string(num_qubits_ - 1) + "]");
    const std::vector<int> qs(qubits);
    for (size_t i = 0; i < qs.size(); ++i)
        for (size_t j = i + 1; j < qs.size(); ++j)
            if (qs[i] == qs[j])
                throw std::invalid_argument(qs.size() == 2
                                                ? "Two-qubit gate requires distinct qubits"
                                                : "Three-qubit gate requires three distinct qubits");
    if (has_param && !std::isfinite(param))
        throw std::invalid_argument("Rotation angle must be a finite number");
    switch (qs.size()) {
        case 1: gates_.emplace_back(t, qs[0], param); break;
        case 2: gates_.emplace_back(t, qs[0], qs[1], param); break;
        default: gates_.emplace_back(t, qs[0], qs[1], qs[2]); break;
    }
    return *this;
}

Circuit& Circuit::x(int q) { return add(GateType::X, {q}, 0.0, false); }
Circuit& Circuit::y(int q) { return add(GateType::Y, {q}, 0.0, false); }
Circuit& Circuit::z(int q) { return add(GateType::Z, {q}, 0.0, false); }
Circuit& Circuit::h(int q) { return add(GateType::H, {q}, 0.0, false); }
Circuit& Circuit::s(int q) { return add(GateType::S, {q}, 0.0, false); }
Circuit& Circuit::t(int q) { return add(GateType::T, {q}, 0.0, false); }
Circuit& Circuit::sdag(int q) { return add(GateType::Sdag, {q}, 0.0, false); }
Circuit& Circuit::tdag(int q) { return add(GateType::Tdag, {q}, 0.0, false); }
Circuit& Circuit::rx(int q, double th) { return add(GateType::Rx, {q}, th, true); }
Circuit& Circuit::ry(int q, double th) { return add(GateType::Ry, {q}, th, true); }
Circuit& Circuit::rz(int q, double th) { return add(GateType::Rz, {q}, th, true); }
Circuit& Circuit::cnot(int c, int t) { return add(GateType::CNOT, {c, t}, 0.0, false); }
Circuit& Circuit::cz(int c, int t) { return add(GateType::CZ, {c, t}, 0.0, false); }
Circuit& Circuit::cry(int c, int t, double th) { return add(GateType::CRY, {c, t}, th, true); }
Circuit& Circuit::crz(int c, int t, double th) { return add(GateType::CRZ, {c, t}, th, true); }
Circuit& Circuit::swap(int a, int b) { return add(GateType::SWAP, {a, b}, 0.0, false); }
Circuit& Circuit::toffoli(int c1, int c2, int t) { return add(GateType::Toffoli, {c1, c2, t}, 0.0, false); }

size_t Circuit::getDepth() const {
    std::vector<size_t> level(num_qubits_, 0);
    size_t depth = 0;
    for (const GateOp& g : gates_) {
        size_t l = 0;
        for (int q : g.qubits) l = std::max(l, level[q]);
        for (int q : g.qubits) level[q] = l + 1;
        depth = std::max(depth, l + 1);
    }
    return depth;
}

std::string Circuit::toString() const {
    std::ostringstream os;
    os << "Circuit(" << num_qubits_ << " qubits, " << gates_.size() << " gates):\n";
    for (size_t i = 0; i < gates_.size(); ++i) {
        const GateOp& g = gates_[i];
        os << "  " << i << ": " << info(g.type).name << "(";
        for (size_t j = 0; j < g.qubits.size(); ++j) os << (j ? ", " : "") << g.qubits[j];
        if (info(g.type).param) os << ", " << g.parameter;
        os << ")\n";
    }
    return os.str();
}

Circuit createBellCircuit() {
    Circuit c(2);
    c.h(0).cnot(0, 1);
    return c;
}

Circuit createGHZCircuit(int num_qubits) {
    if (num_qubits < 2) throw std::invalid_argument("GHZ circuit requires at least 2 qubits");
    Circuit c(num_qubits);
    c.h(0);
    for (int q = 0; q + 1 < num_qubits; ++q) c.cnot(q, q + 1);
    return c;
}

namespace {
// Shared generator: `kinds` lists the gate chosen by each value of uniform_int(0, kinds-1).
enum class Pick { H, X, CNOT, Rz };
Circuit randomCircuit(int n, int depth, unsigned int seed, const std::vector<Pick>& kinds) {
    std::mt19937 rng(seed);
    std::uniform_int_distribution<int> qdist(0, n - 1);
    std::uniform_int_distribution<int> kdist(0, (int)kinds.size() - 1);
    std::uniform_real_distribution<double> adist(0.0, constants::TWO_PI);
    Circuit c(n);
    for (int d = 0; d < depth; ++d) {
        const Pick k = kinds[kdist(rng)];
        const int q1 = qdist(rng);
        switch (k) {
            case Pick::H: c.h(q1); break;
            case Pick::X: c.x(q1); break;
            case Pick::CNOT:
                if (n > 1) {
                    int q2 = qdist(rng);
                    while (q2 == q1) q2 = qdist(rng);
                    c.cnot(q1, q2);
                } else {
                    c.h(q1);
                }
                break;
            case Pick::Rz: c.rz(q1, adist(rng)); break;
        }
    }
    return c;
}
}  // namespace

Circuit createRandomCircuit(int n, int depth, unsigned int seed) {
    return randomCircuit(n, depth, seed, {Pick::H, Pick::X, Pick::CNOT, Pick::Rz});
}

Circuit createRandomHCCircuit(int n, int depth, unsigned int seed) {
    return randomCircuit(n, depth, seed, {Pick::H, Pick::CNOT});
}

Circuit createScalingBenchmarkCircuit(int n) {
    Circuit c(n);
    for (int i = 0; i < 100; ++i) {
        c.h(i % n);
        if (n > 1 && i % 5 == 0) c.cnot(i % n, (i + 1) % n);
    }
    return c;
}

}  // namespace qsim
