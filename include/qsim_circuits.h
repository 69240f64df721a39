/*
 * qsim_circuits.h — C ABI of the C++ circuit factories in libqsim.so.
 *
 * Lets non-C++ hosts (the Python ctypes mirror, bench.py) obtain gate lists that are identical to
 * the reference's libstdc++ factories (std::mt19937 + uniform_*_distribution draw order of
 * src/Circuit.cpp:234-282), instead of re-implementing the distributions.
 */
#ifndef QSIM_CIRCUITS_H
#define QSIM_CIRCUITS_H

#include <stddef.h>

#include "qsim_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    QSIM_CIRCUIT_BELL = 0,      /* createBellCircuit()                    Circuit.cpp:234-238 */
    QSIM_CIRCUIT_GHZ = 1,       /* createGHZCircuit(n)                    Circuit.cpp:240-250 */
    QSIM_CIRCUIT_RANDOM = 2,    /* createRandomCircuit(n, depth, seed)    Circuit.cpp:252-282 */
    QSIM_CIRCUIT_RANDOM_HC = 3, /* W-HC: random {H, CNOT}, same draw order */
    QSIM_CIRCUIT_SCALING = 4    /* W-REF: benchmarks/benchmark_scaling.cu:69-76 */
};

/* Writes up to `cap` gates to `out` and the full gate count to *count (call with cap = 0 to size).
 * Returns QSIM_OK or a QSIM_ERR_* code (message in qsim_circuits_last_error()). */
int qsim_circuit_make(int kind, int n_qubits, int depth, unsigned int seed, qsim_gate* out,
                      size_t cap, size_t* count);
/* Circuit::getDepth() of a gate list (Circuit.cpp:183-201). */
int qsim_circuit_depth(int n_qubits, const qsim_gate* gates, size_t count, size_t* depth);
const char* qsim_circuits_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* QSIM_CIRCUITS_H */
