// oracle_capi.cpp — PARITY ORACLE C entry points for ctypes (tests/, smoke(), bench cpu_baseline).
// Test infrastructure only; see cpu_simulator.hpp.
#include <chrono>
#include <cstring>
#include <thread>

#include "cpu_simulator.hpp"
#include "qsim_hip.h"

using qsim_oracle::CPUSimulator;
using qsim_oracle::Mode;

extern "C" {

// Run `count` gates on |0..0> (or on `state` if init_from_state) and write 2*2^n doubles.
int qsim_oracle_run(int n, const qsim_gate* gates, size_t count, int strict_cpu,
                    int init_from_state, double* state) {
    if (n < 1 || n > 30) return QSIM_ERR_INVALID_ARGUMENT;
    CPUSimulator sim(n, strict_cpu ? Mode::StrictCpu : Mode::GpuSemantics);
    const size_t N = size_t(1) << n;
    if (init_from_state) std::memcpy((void*)sim.mutableState().data(), state, N * 2 * sizeof(double));
    for (size_t i = 0; i < count; ++i)
        sim.apply(gates[i].type, gates[i].qubits, gates[i].nqubits, gates[i].parameter);
    std::memcpy(state, sim.getStateVector().data(), N * 2 * sizeof(double));
    return QSIM_OK;
}

// As qsim_oracle_run with each gate's loop split over `threads` threads (disjoint pair ranges,
// joined before the next gate): the same result bit for bit, for the large-n parity tests.
int qsim_oracle_run_mt(int n, const qsim_gate* gates, size_t count, int strict_cpu, int init_from_state,
                       double* state, int threads) {
    if (n < 1 || n > 30 || threads < 1) return QSIM_ERR_INVALID_ARGUMENT;
    CPUSimulator sim(n, strict_cpu ? Mode::StrictCpu : Mode::GpuSemantics);
    const size_t N = size_t(1) << n;
    if (init_from_state) std::memcpy((void*)sim.mutableState().data(), state, N * 2 * sizeof(double));
    for (size_t i = 0; i < count; ++i) {
        const qsim_gate& g = gates[i];
        const size_t L = sim.loop_size(g.nqubits);
        const size_t T = std::min<size_t>((size_t)threads, std::max<size_t>(1, L >> 12));
        std::vector<std::thread> th;
        for (size_t t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                sim.apply_range(g.type, g.qubits, g.nqubits, g.parameter, L * t / T, L * (t + 1) / T);
            });
        for (std::thread& x : th) x.join();
    }
    std::memcpy(state, sim.getStateVector().data(), N * 2 * sizeof(double));
    return QSIM_OK;
}

// Reference-semantics sampling over a given state (lower_bound on the sequential CDF).
int qsim_oracle_sample(int n, const double* state, const double* uniforms, int shots, int64_t* out) {
    CPUSimulator sim(n);
    const size_t N = size_t(1) << n;
    std::memcpy((void*)sim.mutableState().data(), state, N * 2 * sizeof(double));
    std::vector<double> u(uniforms, uniforms + shots);
    const auto r = sim.sampleWith(u);
    for (int i = 0; i < shots; ++i) out[i] = r[i];
    return QSIM_OK;
}

// CPU baseline: apply gates of the circuit in order on |0..0> until `budget_s` seconds have
// elapsed (at least one gate).  Reports gates done and the seconds they took (single thread).
int qsim_oracle_time_prefix(int n, const qsim_gate* gates, size_t count, double budget_s,
                            size_t* done, double* seconds) {
    if (n < 1 || n > 30) return QSIM_ERR_INVALID_ARGUMENT;
    CPUSimulator sim(n);
    const auto t0 = std::chrono::steady_clock::now();
    size_t k = 0;
    double el = 0.0;
    while (k < count) {
        sim.apply(gates[k].type, gates[k].qubits, gates[k].nqubits, gates[k].parameter);
        ++k;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el >= budget_s) break;
    }
    *done = k;
    *seconds = el;
    return QSIM_OK;
}

}  // extern "C"
