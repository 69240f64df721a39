// cpu_simulator.hpp — PARITY ORACLE (test infrastructure only).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this code, and
// only as the checker / the timed CPU baseline.  The product (libqsim_hip.so, libqsim.so) never
// links or calls it.
//
// Single-threaded C++17 restatement of the reference's CPU path `CPUSimulator`
// (src/Simulator.cu:191-345), written from the reference's behaviour, not its text:
//   * |0...0> start (:195-206); qubit q <-> index bit q (LSB-first);
//   * 1-qubit gates: loop over the 2^(n-1) pairs i0 = insert0(p, t), i1 = i0 | 1<<t with
//     std::complex<double> arithmetic and the reference's constants (:222-287);
//   * CNOT / CZ / SWAP: loop over all 2^n indices, act when the bit pattern selects the pair's
//     lower member (:289-317);
//   * CRY / CRZ / Toffoli: the reference CPUSimulator silently ignores them.  In
//     Mode::GpuSemantics (the default) they follow the reference GPU kernels
//     src/Gates.cu:322-410 instead, so the oracle covers the full gate set; Mode::StrictCpu
//     reproduces the no-ops.
// Parity was pinned against the reference's own known-answer tests (tests/golden/, generated
// from tests/test_gates.cu etc.) and an independent numpy einsum formulation (numpy_oracle.py);
// the reference itself could not be executed here (SURVEY §8(c) denial).
#pragma once

#include <algorithm>
#include <complex>
#include <cstddef>
#include <cstdint>
#include <numeric>
#include <stdexcept>
#include <vector>

namespace qsim_oracle {

using cplx = std::complex<double>;

// Reference GateType numbering (include/Circuit.hpp:42-59).
enum Gate { X, Y, Z, H, S, T, Sdag, Tdag, Rx, Ry, Rz, CNOT, CZ, CRY, CRZ, SWAP, Toffoli };

enum class Mode { GpuSemantics, StrictCpu };

class CPUSimulator {
public:
    explicit CPUSimulator(int num_qubits, Mode mode = Mode::GpuSemantics)
        : n_(num_qubits), size_(size_t(1) << num_qubits), mode_(mode), state_(size_) {
        reset();
    }

    void reset() {
        std::fill(state_.begin(), state_.end(), cplx(0.0, 0.0));
        state_[0] = cplx(1.0, 0.0);
    }

    // Any circuit type exposing getGates() with {type, qubits, parameter} (qsim::Circuit).
    template <class CircuitT>
    void run(const CircuitT& circuit) {
        for (const auto& g : circuit.getGates())
            apply(static_cast<int>(g.type), g.qubits.data(), (int)g.qubits.size(), g.parameter);
    }

    void apply(int type, const int* q, int nq, double theta) { apply_range(type, q, nq, theta, 0, loop_size(nq)); }

    // The gate's loop (pairs for one-qubit gates, indices otherwise) restricted to [begin, end).
    // Every iteration writes only the amplitudes of its own pair (two- and three-qubit gates act
    // from the pair's lower member only), so disjoint ranges may run on different threads and
    // produce exactly the single-threaded result (same operations per amplitude).
    size_t loop_size(int nq) const { return nq == 1 ? size_ >> 1 : size_; }
    void apply_range(int type, const int* q, int nq, double theta, size_t begin, size_t end) {
        if (nq == 1) one(type, q[0], theta, begin, end);
        else if (nq == 2) two(type, q[0], q[1], theta, begin, end);
        else if (nq == 3 && mode_ == Mode::GpuSemantics && type == Toffoli) toffoli(q[0], q[1], q[2], begin, end);
    }

    const std::vector<cplx>& getStateVector() const { return state_; }
    std::vector<cplx>& mutableState() { return state_; }
    int getNumQubits() const { return n_; }

    std::vector<double> getProbabilities() const {
        std::vector<double> p(size_);
        for (size_t i = 0; i < size_; ++i) p[i] = std::norm(state_[i]);
        return p;
    }

    // lower_bound over the sequential partial_sum CDF (src/Simulator.cu:164-185), with the
    // uniforms supplied by the caller.
    std::vector<int64_t> sampleWith(const std::vector<double>& uniforms) const {
        std::vector<double> cdf = getProbabilities();
        std::partial_sum(cdf.begin(), cdf.end(), cdf.begin());
        std::vector<int64_t> out;
        out.reserve(uniforms.size());
        for (double r : uniforms) out.push_back(std::lower_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
        return out;
    }

    // P(index bit == 0), sequential sum; and collapse (src/StateVector.cu:83-124 semantics).
    double probBitZero(int bit) const {
        double s = 0.0;
        for (size_t i = 0; i < size_; ++i)
            if (!((i >> bit) & 1)) s += std::norm(state_[i]);
        return s;
    }
    void collapse(int bit, int result, double scale) {
        for (size_t i = 0; i < size_; ++i)
            state_[i] = (int)((i >> bit) & 1) != result ? cplx(0.0, 0.0) : state_[i] * scale;
    }

private:
    int n_;
    size_t size_;
    Mode mode_;
    std::vector<cplx> state_;

    void one(int type, int t, double theta, size_t begin, size_t end) {
        const double r = 0.70710678118654752440;  // constants::INV_SQRT2
        const size_t low = (size_t(1) << t) - 1;
        const double c = std::cos(theta / 2.0), s = std::sin(theta / 2.0);
        for (size_t p = begin; p < end; ++p) {
            const size_t i0 = (p & low) | ((p & ~low) << 1), i1 = i0 | (size_t(1) << t);
            const cplx a0 = state_[i0], a1 = state_[i1];
            switch (type) {
                case X: state_[i0] = a1; state_[i1] = a0; break;
                case Y: state_[i0] = cplx(0, -1) * a1; state_[i1] = cplx(0, 1) * a0; break;
                case Z: state_[i1] = -a1; break;
                case H: state_[i0] = (a0 + a1) * r; state_[i1] = (a0 - a1) * r; break;
                case S: state_[i1] = cplx(0, 1) * a1; break;
                case T: state_[i1] = cplx(r, r) * a1; break;
                case Sdag: state_[i1] = cplx(0, -1) * a1; break;
                case Tdag: state_[i1] = cplx(r, -r) * a1; break;
                case Rx: state_[i0] = c * a0 - cplx(0, s) * a1; state_[i1] = -cplx(0, s) * a0 + c * a1; break;
                case Ry: state_[i0] = c * a0 - s * a1; state_[i1] = s * a0 + c * a1; break;
                case Rz: state_[i0] = cplx(c, -s) * a0; state_[i1] = cplx(c, s) * a1; break;
                default: break;
            }
        }
    }

    void two(int type, int q1, int q2, double theta, size_t begin, size_t end) {
        const double c = std::cos(theta / 2.0), s = std::sin(theta / 2.0);
        const size_t m1 = size_t(1) << q1, m2 = size_t(1) << q2;
        for (size_t i = begin; i < end; ++i) {
            const bool b1 = i & m1, b2 = i & m2;
            switch (type) {
                case CNOT:
                    if (b1 && !b2) std::swap(state_[i], state_[i ^ m2]);
                    break;
                case CZ:
                    if (b1 && b2) state_[i] = -state_[i];
                    break;
                case SWAP:
                    if (!b1 && b2) std::swap(state_[i], state_[i ^ m1 ^ m2]);
                    break;
                case CRY:  // Gates.cu:322-351 (no-op in the reference CPUSimulator, F4)
                    if (mode_ == Mode::GpuSemantics && b1 && !b2) {
                        const cplx a0 = state_[i], a1 = state_[i ^ m2];
                        state_[i] = c * a0 - s * a1;
                        state_[i ^ m2] = s * a0 + c * a1;
                    }
                    break;
                case CRZ:  // Gates.cu:353-386
                    if (mode_ == Mode::GpuSemantics && b1)
                        state_[i] = (b2 ? cplx(c, s) : cplx(c, -s)) * state_[i];
                    break;
                default: break;
            }
        }
    }

    void toffoli(int c1, int c2, int t, size_t begin, size_t end) {  // Gates.cu:392-410
        const size_t a = size_t(1) << c1, b = size_t(1) << c2, m = size_t(1) << t;
        for (size_t i = begin; i < end; ++i)
            if ((i & a) && (i & b) && !(i & m)) std::swap(state_[i], state_[i ^ m]);
    }
};

}  // namespace qsim_oracle
