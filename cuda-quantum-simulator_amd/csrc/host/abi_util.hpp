// abi_util.hpp — helpers shared by the C++ API translation units: status-code -> exception
// mapping (reference exception conventions) and GateOp -> qsim_gate conversion.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "qsim/Circuit.hpp"
#include "qsim_hip.h"

namespace qsim {
namespace detail {

inline void check(int rc) {
    if (rc == QSIM_OK) return;
    const std::string msg = qsim_last_error();
    switch (rc) {
        case QSIM_ERR_INVALID_ARGUMENT: throw std::invalid_argument(msg);
        case QSIM_ERR_OUT_OF_RANGE: throw std::out_of_range(msg);
        default: throw std::runtime_error(msg);
    }
}

inline qsim_gate toAbi(const GateOp& g) {
    qsim_gate r{};
    r.type = static_cast<int>(g.type);
    r.nqubits = (int)g.qubits.size();
    for (size_t i = 0; i < g.qubits.size() && i < 3; ++i) r.qubits[i] = g.qubits[i];
    r.parameter = g.parameter;
    return r;
}

inline std::vector<qsim_gate> toAbi(const Circuit& c) {
    std::vector<qsim_gate> v;
    v.reserve(c.getGates().size());
    for (const GateOp& g : c.getGates()) v.push_back(toAbi(g));
    return v;
}

}  // namespace detail
}  // namespace qsim
