// test_cpu_api.cpp — the product qsim::CPUSimulator (csrc/host/CPUSimulator.cpp; reference
// include/Simulator.hpp:91-112, src/Simulator.cu:195-345) against the test oracle, on the CPU.
// No GPU call is made: CPUSimulator is pure host code in libqsim.so.
#include <qsim/Circuit.hpp>
#include <qsim/Constants.hpp>
#include <qsim/Simulator.hpp>

#include <cmath>
#include <complex>
#include <map>
#include <numeric>
#include <random>
#include <stdexcept>
#include <vector>

#include "cpu_simulator.hpp"
#include "harness.hpp"

using cplx = std::complex<double>;

static std::vector<cplx> oracle_state(const qsim::Circuit& c, qsim_oracle::Mode m) {
    qsim_oracle::CPUSimulator o(c.getNumQubits(), m);
    o.run(c);
    return o.getStateVector();
}

static double max_diff(const std::vector<cplx>& a, const std::vector<cplx>& b) {
    double d = 0.0;
    for (size_t i = 0; i < a.size(); ++i)
        d = std::max(d, std::max(std::fabs(a[i].real() - b[i].real()), std::fabs(a[i].imag() - b[i].imag())));
    return d;
}

static qsim::Circuit mixed(int n, int depth, unsigned seed) {
    std::mt19937 rng(seed);
    qsim::Circuit c(n);
    std::uniform_real_distribution<double> ang(-3.0, 3.0);
    for (int i = 0; i < depth; ++i) {
        const int t = (int)(rng() % 17);
        std::vector<int> q(n);
        std::iota(q.begin(), q.end(), 0);
        std::shuffle(q.begin(), q.end(), rng);
        const int ar = t <= 10 ? 1 : (t <= 15 ? 2 : 3);
        q.resize(ar);
        const double th = ang(rng);
        switch (t) {
            case 0: c.x(q[0]); break;
            case 1: c.y(q[0]); break;
            case 2: c.z(q[0]); break;
            case 3: c.h(q[0]); break;
            case 4: c.s(q[0]); break;
            case 5: c.t(q[0]); break;
            case 6: c.sdag(q[0]); break;
            case 7: c.tdag(q[0]); break;
            case 8: c.rx(q[0], th); break;
            case 9: c.ry(q[0], th); break;
            case 10: c.rz(q[0], th); break;
            case 11: c.cnot(q[0], q[1]); break;
            case 12: c.cz(q[0], q[1]); break;
            case 13: c.cry(q[0], q[1], th); break;
            case 14: c.crz(q[0], q[1], th); break;
            case 15: c.swap(q[0], q[1]); break;
            default: c.toffoli(q[0], q[1], q[2]); break;
        }
    }
    return c;
}

TEST(CPUSimulator, BellAndGHZ) {  // tests/test_gates.cu:66-97 known answers on the CPU path
    qsim::CPUSimulator s(2);
    s.run(qsim::createBellCircuit());
    auto p = s.getProbabilities();
    EXPECT_NEAR(p[0], 0.5, 1e-12);
    EXPECT_NEAR(p[3], 0.5, 1e-12);
    qsim::CPUSimulator g(5);
    g.run(qsim::createGHZCircuit(5));
    auto pg = g.getProbabilities();
    EXPECT_NEAR(pg[0], 0.5, 1e-12);
    EXPECT_NEAR(pg[31], 0.5, 1e-12);
}

TEST(CPUSimulator, ReferenceGateSetMatchesStrictOracle) {  // F4: CRY/CRZ/CCX are no-ops
    for (int n : {3, 7, 12, 16})
        for (unsigned seed : {1u, 2u, 3u}) {
            const qsim::Circuit c = mixed(n, 120, seed * 7 + n);
            qsim::CPUSimulator s(n);
            s.run(c);
            EXPECT_TRUE(max_diff(s.getStateVector(), oracle_state(c, qsim_oracle::Mode::StrictCpu)) < 1e-12);
        }
}

TEST(CPUSimulator, FullGateSetMatchesGpuSemanticsOracle) {
    for (int n : {3, 8, 15})
        for (unsigned seed : {4u, 5u}) {
            const qsim::Circuit c = mixed(n, 150, seed * 11 + n);
            qsim::CPUSimulator s(n, qsim::CpuGateSet::Full);
            s.run(c);
            EXPECT_TRUE(max_diff(s.getStateVector(), oracle_state(c, qsim_oracle::Mode::GpuSemantics)) < 1e-12);
        }
}

TEST(CPUSimulator, ThreadsDoNotChangeResults) {  // each pair is owned by one thread: bitwise equal
    const qsim::Circuit c = qsim::createRandomCircuit(18, 200, 9);
    qsim::CPUSimulator a(18, qsim::CpuGateSet::Full), b(18, qsim::CpuGateSet::Full);
    a.setThreads(1);
    b.setThreads(8);
    a.run(c);
    b.run(c);
    EXPECT_TRUE(a.getStateVector() == b.getStateVector());
}

TEST(CPUSimulator, ScalingBenchmarkCircuit) {  // benchmarks/benchmark_scaling.cu:69-90 circuit
    for (int n = 10; n <= 16; n += 2) {
        qsim::Circuit c(n);
        for (int i = 0; i < 100; ++i) {
            c.h(i % n);
            if (i % 5 == 0) c.cnot(i % n, (i + 1) % n);
        }
        qsim::CPUSimulator s(n);
        s.run(c);
        EXPECT_TRUE(max_diff(s.getStateVector(), oracle_state(c, qsim_oracle::Mode::StrictCpu)) < 1e-12);
        auto p = s.getProbabilities();
        EXPECT_NEAR(std::accumulate(p.begin(), p.end(), 0.0), 1.0, 1e-10);
    }
}

TEST(CPUSimulator, SampleAndErrors) {
    qsim::CPUSimulator s(2);
    s.setSeed(5);
    s.run(qsim::createBellCircuit());
    std::map<int, int> h;
    for (int o : s.sample(4000)) ++h[o];
    EXPECT_EQ(h[1] + h[2], 0);
    EXPECT_TRUE(std::abs(h[0] - 2000) < 200);
    EXPECT_TRUE(s.sample(0).empty());
    EXPECT_THROW(qsim::CPUSimulator(0), std::invalid_argument);
    EXPECT_THROW(qsim::CPUSimulator(qsim::cuda_config::MAX_QUBITS + 1), std::invalid_argument);
    qsim::Circuit c3(3);
    EXPECT_THROW(s.run(c3), std::invalid_argument);
    s.reset();
    EXPECT_NEAR(s.getProbabilities()[0], 1.0, 0.0);
    EXPECT_EQ(s.getNumQubits(), 2);
}

TEST(Constants, CudaConfigAlias) {  // include/Constants.hpp:56-75 names keep compiling
    static_assert(qsim::cuda_config::MAX_QUBITS == 30, "MAX_QUBITS");
    static_assert(qsim::cuda_config::MIN_QUBITS == 1, "MIN_QUBITS");
    static_assert(qsim::cuda_config::DEFAULT_BLOCK_SIZE == 256, "DEFAULT_BLOCK_SIZE");
    EXPECT_TRUE(qsim::cuda_config::REDUCTION_BLOCK_SIZE > 0);
}

TH_MAIN
