// circuit_capi.cpp — extern "C" wrappers of the C++ circuit factories (include/qsim_circuits.h).
#include <stdexcept>
#include <string>

#include "abi_util.hpp"
#include "qsim/Circuit.hpp"
#include "qsim_circuits.h"

static thread_local std::string g_circ_err;

extern "C" {

const char* qsim_circuits_last_error(void) { return g_circ_err.c_str(); }

int qsim_circuit_make(int kind, int n, int depth, unsigned int seed, qsim_gate* out, size_t cap,
                      size_t* count) {
    try {
        qsim::Circuit c = [&]() -> qsim::Circuit {
            switch (kind) {
                case QSIM_CIRCUIT_BELL: return qsim::createBellCircuit();
                case QSIM_CIRCUIT_GHZ: return qsim::createGHZCircuit(n);
                case QSIM_CIRCUIT_RANDOM: return qsim::createRandomCircuit(n, depth, seed);
                case QSIM_CIRCUIT_RANDOM_HC: return qsim::createRandomHCCircuit(n, depth, seed);
                case QSIM_CIRCUIT_SCALING: return qsim::createScalingBenchmarkCircuit(n);
            }
            throw std::invalid_argument("unknown circuit kind");
        }();
        const auto gates = qsim::detail::toAbi(c);
        if (count) *count = gates.size();
        for (size_t i = 0; i < gates.size() && i < cap; ++i) out[i] = gates[i];
        return QSIM_OK;
    } catch (const std::invalid_argument& e) {
        g_circ_err = e.what();
        return QSIM_ERR_INVALID_ARGUMENT;
    } catch (const std::out_of_range& e) {
        g_circ_err = e.what();
        return QSIM_ERR_OUT_OF_RANGE;
    } catch (const std::exception& e) {
        g_circ_err = e.what();
        return QSIM_ERR_RUNTIME;
    }
}

int qsim_circuit_depth(int n, const qsim_gate* gates, size_t count, size_t* depth) {
    try {
        qsim::Circuit c(n);
        for (size_t i = 0; i < count; ++i) {
            const qsim_gate& g = gates[i];
            const auto t = static_cast<qsim::GateType>(g.type);
            switch (g.nqubits) {
                case 1:
                    if (t == qsim::GateType::Rx) c.rx(g.qubits[0], g.parameter);
                    else if (t == qsim::GateType::Ry) c.ry(g.qubits[0], g.parameter);
                    else if (t == qsim::GateType::Rz) c.rz(g.qubits[0], g.parameter);
                    else c.h(g.qubits[0]);  // depth only depends on the qubits touched
                    break;
                case 2: c.cnot(g.qubits[0], g.qubits[1]); break;
                case 3: c.toffoli(g.qubits[0], g.qubits[1], g.qubits[2]); break;
                default: throw std::invalid_argument("bad arity");
            }
        }
        *depth = c.getDepth();
        return QSIM_OK;
    } catch (const std::invalid_argument& e) {
        g_circ_err = e.what();
        return QSIM_ERR_INVALID_ARGUMENT;
    } catch (const std::out_of_range& e) {
        g_circ_err = e.what();
        return QSIM_ERR_OUT_OF_RANGE;
    } catch (const std::exception& e) {
        g_circ_err = e.what();
        return QSIM_ERR_RUNTIME;
    }
}

}  // extern "C"
