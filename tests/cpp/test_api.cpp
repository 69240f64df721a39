// test_api.cpp — the reference's C++ test suites restated against the drop-in C++ API
// (include/qsim/*.hpp → libqsim.so → libqsim_hip.so).  Each case cites the reference test it
// mirrors.  Needs a GPU; the CPU oracle (tests only) is the header-only
// oracle/cpu_simulator.hpp.
#include <qsim/Circuit.hpp>
#include <qsim/DensityMatrix.hpp>
#include <qsim/NoiseModel.hpp>
#include <qsim/OptimizedGates.hpp>
#include <qsim/Simulator.hpp>
#include <qsim/StateVector.hpp>

#include <cmath>
#include <complex>
#include <numeric>
#include <stdexcept>
#include <utility>
#include <vector>

#include "cpu_simulator.hpp"
#include "harness.hpp"
#include "qsim_hip.h"

using cplx = std::complex<double>;
static const double kTol = 1e-10;          // tests/test_gates.cu:18
static const double kEquivTol = 1e-12;     // tests/test_gpu_cpu_equivalence.cu:26
static const double kS = 0.7071067811865476;

static std::vector<cplx> run_gpu(const qsim::Circuit& c, qsim::RunMode mode) {
    qsim::Simulator sim(c.getNumQubits());
    sim.setRunMode(mode);
    sim.run(c);
    return sim.getStateVector();
}

static void expect_state(const std::vector<cplx>& got, const std::vector<cplx>& want, double tol) {
    ASSERT_TRUE(got.size() == want.size());
    for (size_t i = 0; i < got.size(); ++i) {
        EXPECT_NEAR(got[i].real(), want[i].real(), tol);
        EXPECT_NEAR(got[i].imag(), want[i].imag(), tol);
    }
}

static void expect_matches_oracle(const qsim::Circuit& c, double tol = kEquivTol) {
    qsim_oracle::CPUSimulator cpu(c.getNumQubits());
    cpu.run(c);
    for (qsim::RunMode m : {qsim::RunMode::PerGate, qsim::RunMode::Fused})
        expect_state(run_gpu(c, m), cpu.getStateVector(), tol);
}

static std::vector<cplx> basis(int n, size_t k, cplx v = 1.0) {
    std::vector<cplx> s(size_t(1) << n, 0.0);
    s[k] = v;
    return s;
}

// ---- tests/test_gates.cu known answers ------------------------------------------------------
TEST(Gates, PauliX) {  // test_gates.cu:39-49
    qsim::Circuit c(1);
    c.x(0);
    expect_state(run_gpu(c, qsim::RunMode::Fused), basis(1, 1), kTol);
}
TEST(Gates, Hadamard) {  // :51-62
    qsim::Circuit c(1);
    c.h(0);
    expect_state(run_gpu(c, qsim::RunMode::Fused), {kS, kS}, kTol);
}
TEST(Gates, HadamardTwiceIsIdentity) {  // :64-74
    qsim::Circuit c(1);
    c.h(0).h(0);
    expect_state(run_gpu(c, qsim::RunMode::PerGate), basis(1, 0), kTol);
}
TEST(Gates, PauliZOnPlus) {  // :76-86
    qsim::Circuit c(1);
    c.h(0).z(0);
    expect_state(run_gpu(c, qsim::RunMode::Fused), {kS, -kS}, kTol);
}
TEST(Gates, PauliY) {  // :88-96
    qsim::Circuit c(1);
    c.y(0);
    expect_state(run_gpu(c, qsim::RunMode::Fused), {0.0, cplx(0, 1)}, kTol);
}
TEST(Gates, SAndT) {  // :98-116
    qsim::Circuit c(1);
    c.h(0).s(0);
    expect_state(run_gpu(c, qsim::RunMode::PerGate), {kS, cplx(0, kS)}, kTol);
    qsim::Circuit d(1);
    d.h(0).t(0);
    expect_state(run_gpu(d, qsim::RunMode::Fused), {kS, cplx(0.5, 0.5)}, kTol);
}
TEST(Gates, Rotations) {  // :118-152
    const double pi = std::acos(-1.0);
    qsim::Circuit rx(1), ry(1), rz(1);
    rx.rx(0, pi);
    ry.ry(0, pi);
    rz.rz(0, pi / 3);
    auto a = run_gpu(rx, qsim::RunMode::Fused);
    EXPECT_NEAR(std::abs(a[1]), 1.0, kTol);
    EXPECT_NEAR(a[1].imag(), -1.0, kTol);
    auto b = run_gpu(ry, qsim::RunMode::PerGate);
    EXPECT_NEAR(std::abs(b[1]), 1.0, kTol);
    auto z = run_gpu(rz, qsim::RunMode::Fused);
    EXPECT_NEAR(std::abs(z[0]), 1.0, kTol);
    EXPECT_NEAR(std::arg(z[0]), -pi / 6, kTol);
}
TEST(Gates, CnotAndBell) {  // :158-195
    qsim::Circuit c(2);
    c.x(0).cnot(0, 1);
    expect_state(run_gpu(c, qsim::RunMode::Fused), basis(2, 3), kTol);
    expect_state(run_gpu(qsim::createBellCircuit(), qsim::RunMode::Fused), {kS, 0, 0, kS}, kTol);
}
TEST(Gates, CzAndSwap) {  // :197-219
    qsim::Circuit c(2);
    c.x(0).x(1).cz(0, 1);
    expect_state(run_gpu(c, qsim::RunMode::PerGate), basis(2, 3, -1.0), kTol);
    qsim::Circuit s(2);
    s.x(0).swap(0, 1);
    expect_state(run_gpu(s, qsim::RunMode::Fused), basis(2, 2), kTol);
}
TEST(Gates, GhzAndUniform) {  // :225-252
    qsim::Simulator sim(4);
    sim.run(qsim::createGHZCircuit(4));
    auto p = sim.getProbabilities();
    EXPECT_NEAR(p[0], 0.5, kTol);
    EXPECT_NEAR(p[15], 0.5, kTol);
    qsim::Circuit h(4);
    for (int q = 0; q < 4; ++q) h.h(q);
    qsim::Simulator u(4);
    u.run(h);
    for (double v : u.getProbabilities()) EXPECT_NEAR(v, 1.0 / 16, kTol);
}
TEST(Gates, Toffoli) {  // :258-316 ("index = q0 + 2*q1 + 4*q2", :261)
    qsim::Circuit a(3), b(3), c(3), d(3);
    a.x(0).x(1).toffoli(0, 1, 2);
    b.x(0).toffoli(0, 1, 2);
    c.toffoli(0, 1, 2);
    d.x(0).x(1).x(2).toffoli(0, 1, 2);
    expect_state(run_gpu(a, qsim::RunMode::Fused), basis(3, 7), kTol);
    expect_state(run_gpu(b, qsim::RunMode::PerGate), basis(3, 1), kTol);
    expect_state(run_gpu(c, qsim::RunMode::Fused), basis(3, 0), kTol);
    expect_state(run_gpu(d, qsim::RunMode::PerGate), basis(3, 3), kTol);
}
TEST(Gates, ControlledRotations) {  // :318-386
    const double pi = std::acos(-1.0);
    qsim::Circuit off(2), on(2), rz(2);
    off.cry(0, 1, pi);
    on.x(0).cry(0, 1, pi);
    rz.x(0).h(1).crz(0, 1, pi / 2);
    expect_state(run_gpu(off, qsim::RunMode::Fused), basis(2, 0), kTol);
    expect_state(run_gpu(on, qsim::RunMode::Fused), basis(2, 3), kTol);
    auto s = run_gpu(rz, qsim::RunMode::PerGate);
    const cplx em = std::exp(cplx(0, -pi / 4)), ep = std::exp(cplx(0, pi / 4));
    expect_state(s, {0, kS * em, 0, kS * ep}, kTol);
}

// ---- tests/test_gpu_cpu_equivalence.cu -------------------------------------------------------
TEST(Equivalence, SingleQubitGatesOnSuperposition) {  // :122-152
    const double th = 0.7;
    for (int g = 0; g <= 10; ++g)
        for (int q = 0; q < 3; ++q) {
            qsim::Circuit c(3);
            c.h(0).h(1).h(2);
            switch (g) {
                case 0: c.x(q); break;
                case 1: c.y(q); break;
                case 2: c.z(q); break;
                case 3: c.h(q); break;
                case 4: c.s(q); break;
                case 5: c.t(q); break;
                case 6: c.sdag(q); break;
                case 7: c.tdag(q); break;
                case 8: c.rx(q, th); break;
                case 9: c.ry(q, th); break;
                default: c.rz(q, th); break;
            }
            expect_matches_oracle(c);
        }
}
TEST(Equivalence, TwoQubitGatesAllPairs) {  // :158-206
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            if (a == b) continue;
            qsim::Circuit c(4);
            c.h(0).h(1).h(2).h(3).t(a).s(b).cnot(a, b).cz(a, b).swap(a, b);
            expect_matches_oracle(c);
        }
}
TEST(Equivalence, RandomCircuits) {  // :227-251
    for (unsigned s = 0; s < 20; ++s)
        expect_matches_oracle(qsim::createRandomCircuit(3 + s % 3, 10 + s, s));
    for (unsigned s = 0; s < 10; ++s)
        expect_matches_oracle(qsim::createRandomCircuit(8 + s % 4, 50 + 5 * s, s));
}
TEST(Equivalence, DeepCircuitProbabilities) {  // :253-275
    for (unsigned s = 0; s < 5; ++s) {
        qsim::Circuit c = qsim::createRandomCircuit(4, 500, s);
        qsim_oracle::CPUSimulator cpu(4);
        cpu.run(c);
        qsim::Simulator sim(4);
        sim.run(c);
        auto p = sim.getProbabilities(), q = cpu.getProbabilities();
        for (size_t i = 0; i < p.size(); ++i) EXPECT_NEAR(p[i], q[i], 1e-10);
    }
}
TEST(Equivalence, FullGateSetWide) {  // all 17 gate types, targets across the 1 KiB lane boundary
    for (int n : {7, 12, 14}) {
        qsim::Circuit c(n);
        for (int i = 0; i < 60; ++i) {
            const int a = (7 * i + 1) % n, b = (5 * i + 3) % n == a ? (a + 1) % n : (5 * i + 3) % n;
            int d = (3 * i + 2) % n;
            while (d == a || d == b) d = (d + 1) % n;
            c.h(a).ry(b, 0.1 * i).cnot(a, b).rz(d, 0.3).cry(b, d, 0.2 * i).crz(d, a, -0.4)
                .toffoli(a, b, d).swap(a, d).t(b).sdag(a).cz(d, b).y(a).rx(d, 0.05 * i)
                .s(b).tdag(d).z(a).x(b);
        }
        expect_matches_oracle(c);
    }
}
TEST(Equivalence, RunSequence) {  // Simulator::runSequence (no reference counterpart) = run() in turn
    for (int n : {9, 14, 20}) {
        std::vector<qsim::Circuit> cs;
        for (unsigned s = 0; s < 3; ++s) cs.push_back(qsim::createRandomHCCircuit(n, 60, 100 + s));
        qsim::Simulator seq(n);
        seq.runSequence(cs);
        qsim_oracle::CPUSimulator cpu(n);
        for (const qsim::Circuit& c : cs) cpu.run(c);
        expect_state(seq.getStateVector(), cpu.getStateVector(), kEquivTol);
    }
    qsim::Simulator sim(3);
    EXPECT_THROW(sim.runSequence({qsim::Circuit(3), qsim::Circuit(4)}), std::invalid_argument);
}
TEST(Equivalence, EmptyAndTrivialCircuits) {  // :318-339
    qsim::Circuit e(3), one(3), two(3);
    one.h(1);
    two.h(1).h(1);
    expect_matches_oracle(e);
    expect_matches_oracle(one);
    expect_matches_oracle(two);
}

// ---- tests/test_boundary.cu -----------------------------------------------------------------
TEST(Boundary, Sizes) {  // :30-104
    for (int n : {1, 2, 16}) {
        qsim::Simulator sim(n);
        EXPECT_EQ(sim.getNumQubits(), n);
        EXPECT_EQ(sim.getStateSize(), size_t(1) << n);
    }
    qsim::Simulator big(20);
    big.run(qsim::createGHZCircuit(20));
    auto p = big.getProbabilities();
    EXPECT_NEAR(p[0], 0.5, kTol);
    EXPECT_NEAR(p[(size_t(1) << 20) - 1], 0.5, kTol);
}
TEST(Boundary, ErrorTypes) {  // :110-163, test_statevector.cu:229-242
    EXPECT_THROW(qsim::StateVector(31), std::invalid_argument);
    EXPECT_THROW(qsim::StateVector(0), std::invalid_argument);
    EXPECT_THROW(qsim::Circuit(0), std::invalid_argument);
    qsim::Circuit c(3);
    EXPECT_THROW(c.h(3), std::out_of_range);
    EXPECT_THROW(c.h(-1), std::out_of_range);
    EXPECT_THROW(c.cnot(1, 1), std::invalid_argument);
    EXPECT_THROW(c.toffoli(0, 1, 1), std::invalid_argument);
    EXPECT_THROW(c.rx(0, std::nan("")), std::invalid_argument);
    qsim::Simulator sim(2);
    EXPECT_THROW(sim.run(c), std::invalid_argument);
    EXPECT_THROW(sim.measureQubit(2), std::invalid_argument);
    EXPECT_THROW(sim.state().initializeBasis(4), std::invalid_argument);
    EXPECT_THROW(sim.state().sample(0), std::invalid_argument);
}
TEST(Boundary, NormalizedAfterLongCircuit) {  // :197-212
    qsim::Simulator sim(10);
    sim.run(qsim::createRandomCircuit(10, 1000, 7));
    EXPECT_TRUE(sim.state().isNormalized(1e-10));
    EXPECT_NO_THROW(sim.state().assertNormalized());
}
TEST(Boundary, ResetMoveAndCoexistence) {  // :237-315
    qsim::Simulator a(3), b(5);
    a.run(qsim::createGHZCircuit(3));
    b.run(qsim::createGHZCircuit(5));
    a.reset();
    expect_state(a.getStateVector(), basis(3, 0), kTol);
    EXPECT_NEAR(b.getProbabilities()[31], 0.5, kTol);
    qsim::StateVector s(4);
    qsim::StateVector t(std::move(s));
    EXPECT_EQ(t.getSize(), size_t(16));
    EXPECT_EQ(s.getSize(), size_t(0));
    EXPECT_TRUE(s.devicePtr() == nullptr);
}

// ---- tests/test_statevector.cu --------------------------------------------------------------
TEST(StateVector, InitAndBasis) {  // :20-95
    qsim::StateVector s(5);
    EXPECT_NEAR(s.getTotalProbability(), 1.0, kTol);
    s.initializeBasis(19);
    auto v = s.toHost();
    EXPECT_NEAR(v[19].real(), 1.0, kTol);
    EXPECT_NEAR(s.getTotalProbability(), 1.0, kTol);
}
TEST(StateVector, RawKernelEntry) {  // :151-159 launches applyH<<<>>> on devicePtr()
    qsim::StateVector s(3);
    qsim_gate g{QSIM_GATE_H, 1, {2, 0, 0}, 0, 0.0};
    void* stream = nullptr;
    ASSERT_TRUE(qsim_state_stream(s.handle(), &stream) == QSIM_OK);
    ASSERT_TRUE(qsim_apply_gate_raw(s.devicePtr(), 3, &g, stream) == QSIM_OK);
    auto p = s.getProbabilities();
    EXPECT_NEAR(p[0], 0.5, kTol);
    EXPECT_NEAR(p[4], 0.5, kTol);
}
TEST(StateVector, MeasureConventionF2) {  // src/StateVector.cu:87-89 (bit n-1-q)
    qsim::Simulator sim(2);
    qsim::Circuit c(2);
    c.x(0);
    sim.run(c);
    EXPECT_EQ(sim.measureQubit(1), 1);  // reads index bit 0
    EXPECT_EQ(sim.measureQubit(0), 0);  // reads index bit 1
    EXPECT_EQ(sim.state().measureBit(0), 1);
}
TEST(StateVector, SamplingBell) {  // :101-227 (±0.05)
    qsim::Simulator sim(2);
    sim.setSeed(11);
    sim.run(qsim::createBellCircuit());
    auto shots = sim.sample(4000);
    int ones = 0;
    for (int k : shots) {
        EXPECT_TRUE(k == 0 || k == 3);
        ones += k == 3;
    }
    EXPECT_NEAR(ones / 4000.0, 0.5, 0.05);
}
TEST(StateVector, GeneralMatrixEqualsY) {  // test_optimized_gates.cu general-1Q(Y)
    qsim::Circuit prep(6);
    for (int q = 0; q < 6; ++q) prep.ry(q, 0.3 + 0.1 * q);
    for (int t : {0, 5}) {
        qsim::Simulator a(6), b(6);
        a.run(prep);
        b.run(prep);
        qsim::Circuit y(6);
        y.y(t);
        a.run(y);
        const cplx m[4] = {0.0, cplx(0, -1), cplx(0, 1), 0.0};
        b.state().applyMatrix1Q(t, m);
        expect_state(b.getStateVector(), a.getStateVector(), 1e-12);
    }
}

// ---- tests/test_noise.cu (batched, noise-free) ----------------------------------------------
TEST(DensityMatrix, ReferenceSuite) {  // tests/test_density_matrix.cu:142-157, :251-265, :306-318
    qsim::DensityMatrixSimulator bell(2);
    bell.run(qsim::createBellCircuit());
    auto p = bell.getProbabilities();
    EXPECT_NEAR(p[0], 0.5, kTol);
    EXPECT_NEAR(p[3], 0.5, kTol);
    EXPECT_NEAR(bell.getPurity(), 1.0, kTol);
    qsim::NoiseModel nm;
    nm.addBitFlip(0.5);
    qsim::DensityMatrixSimulator flip(1, nm);
    qsim::Circuit x(1);
    x.x(0);
    flip.run(x);
    EXPECT_NEAR(flip.getProbabilities()[0], 0.5, 0.1);
    qsim::NoiseModel nm2;
    nm2.addDepolarizing(0.1);
    nm2.addAmplitudeDamping(0.05);
    qsim::DensityMatrixSimulator tr(2, nm2);
    qsim::Circuit c(2);
    c.h(0).h(1).cnot(0, 1).rz(0, 0.5);
    tr.run(c);
    EXPECT_NEAR(tr.getTrace(), 1.0, 1e-6);
    EXPECT_THROW(qsim::DensityMatrix(0), std::invalid_argument);
}
TEST(Noisy, BitFlipUndoesX) {  // tests/test_noise.cu:157-179
    qsim::NoiseModel nm;
    nm.addBitFlip({0}, 1.0);
    qsim::NoisySimulator sim(1, nm);
    sim.setSeed(42);
    qsim::Circuit x(1);
    x.x(0);
    sim.run(x);
    EXPECT_NEAR(sim.getProbabilities()[0], 1.0, kTol);
}
TEST(Batched, NoiseFreeBell) {  // :249-281, :313-339
    qsim::BatchedSimulator bs(2, 5);
    bs.run(qsim::createBellCircuit());
    for (int t = 0; t < 5; ++t) {
        auto p = bs.getProbabilities(t);
        EXPECT_NEAR(p[0], 0.5, kTol);
        EXPECT_NEAR(p[3], 0.5, kTol);
    }
    auto avg = bs.getAverageProbabilities();
    EXPECT_NEAR(avg[0] + avg[3], 1.0, kTol);
    EXPECT_EQ(bs.getTotalMemoryBytes(), size_t(5 * 4 * 16));
    auto h = bs.getHistogram(100);
    EXPECT_EQ(std::accumulate(h.begin(), h.end(), 0), 500);
    EXPECT_THROW(bs.getProbabilities(5), std::out_of_range);
}
TEST(Batched, DepolarizingKeepsNormalization) {  // :283-311, :449-462
    qsim::NoiseModel nm;
    nm.addDepolarizingAll(4, 0.05);
    qsim::BatchedSimulator bs(4, 64, nm);
    bs.setSeed(3);
    qsim::Circuit c(4);
    c.h(0).cnot(0, 1).ry(2, 0.4).cz(1, 3).x(2);
    bs.run(c);
    auto avg = bs.getAverageProbabilities();
    EXPECT_NEAR(std::accumulate(avg.begin(), avg.end(), 0.0), 1.0, 1e-10);
}

// benchmarks/benchmark_scaling.cu:69-90 (benchmarkGPUvsCPU): the W-REF circuit through the GPU
// Simulator and the API's CPUSimulator at n = 10..22 — the states agree at 1e-12.
TEST(Scaling, GpuMatchesCpuSimulator) {
    for (int n = 10; n <= 22; n += 2) {
        qsim::Circuit c(n);
        for (int i = 0; i < 100; ++i) {
            c.h(i % n);
            if (n > 1 && i % 5 == 0) c.cnot(i % n, (i + 1) % n);
        }
        qsim::Simulator gpu_sim(n);
        gpu_sim.run(c);
        qsim::CPUSimulator cpu_sim(n);
        cpu_sim.run(c);
        expect_state(gpu_sim.getStateVector(), cpu_sim.getStateVector(), kEquivTol);
    }
}

// src/OptimizedGates.cu:388-413 named dispatchers on StateVector::devicePtr() (the reference's
// tests/test_optimized_gates.cu drive them the same way) == the same gates via the simulator.
TEST(OptimizedGates, NamedDispatchers) {
    const int n = 9;
    qsim::StateVector sv(n);
    qsim::applyHadamardOptimized(sv.devicePtr(), n, 2);
    qsim::applyCNOTOptimized(sv.devicePtr(), n, 2, 7);
    const std::complex<double> x[4] = {0.0, 1.0, 1.0, 0.0};
    qsim::applyGate1QOptimized(sv.devicePtr(), n, 5, x);
    qsim::StateVector ref(n);
    qsim::Circuit c(n);
    c.h(2).cnot(2, 7).x(5);
    qsim::Simulator sim(n);
    sim.run(c);
    expect_state(sv.toHost(), sim.getStateVector(), kEquivTol);
}

// qsim_apply_matrix (k-qubit general matrix): a 3-qubit permutation matrix == the gates it encodes.
TEST(StateVector, GeneralMatrixK3) {
    const int n = 8;
    qsim::StateVector sv(n);
    qsim::Circuit prep(n);
    prep.h(0).h(3).h(5).ry(6, 0.3);
    qsim::Simulator sim(n);
    sim.run(prep);
    sv.fromHost(sim.getStateVector());
    // Toffoli(c1 = qubit 5 (bit 0), c2 = qubit 3 (bit 1), target = qubit 6 (bit 2)) as an 8x8
    std::vector<std::complex<double>> m(64, 0.0);
    for (int r = 0; r < 8; ++r) {
        const int c = (r & 3) == 3 ? r ^ 4 : r;
        m[r * 8 + c] = 1.0;
    }
    sv.applyMatrix({5, 3, 6}, m);
    qsim::Circuit t(n);
    t.toffoli(5, 3, 6);
    sim.applyGate(t.getGates()[0]);
    expect_state(sv.toHost(), sim.getStateVector(), kEquivTol);
}

TH_MAIN
