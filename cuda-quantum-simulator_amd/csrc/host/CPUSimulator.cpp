// CPUSimulator.cpp — the API's host-side simulator (reference CPUSimulator,
// include/Simulator.hpp:91-112, src/Simulator.cu:195-345), for callers that time or check against
// the CPU (benchmarks/benchmark_scaling.cu:85).  Own implementation, not the test oracle:
//   * every gate is lowered once to an update rule on the pairs (i0, i1 = i0 | 1 << t) of its
//     target — a closed form for the fixed gates (the same arithmetic as the reference CPU path,
//     so results agree to the last bit for X/Y/Z/H/S/T/S†/T†/CNOT/CZ/SWAP) or a 2x2 complex
//     matrix for the rotations — with its controls as forced-1 bits of the pair index, so only
//     the control == 1 subspace is visited (the reference scans all 2^n indices for CNOT);
//   * the pair range is split into contiguous blocks over a persistent worker pool (states below
//     2^17 amplitudes stay on the calling thread).
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>

#include "qsim/Constants.hpp"
#include "qsim/Simulator.hpp"

namespace qsim {
namespace {

using cplx = std::complex<double>;

enum Rule { R_SWAP, R_Y, R_PHASE1, R_NEG1, R_H, R_MAT, R_SWAP2 };

struct Lowered {
    Rule rule = R_MAT;
    int target = 0, target2 = -1;
    uint64_t cmask = 0;  // control bits (must read 1)
    cplx m[4];           // R_MAT: [[m0, m1], [m2, m3]]; R_PHASE1: m[3] multiplies |1>
    bool noop = false;
};

Lowered lower(const GateOp& g, CpuGateSet set) {
    Lowered L;
    const double th = g.parameter;
    const double c = std::cos(th / 2.0), s = std::sin(th / 2.0);
    const double r = constants::INV_SQRT2;
    L.target = g.qubits.empty() ? 0 : g.qubits.back();
    switch (g.type) {
        case GateType::X: L.rule = R_SWAP; break;
        case GateType::Y: L.rule = R_Y; break;
        case GateType::Z: L.rule = R_NEG1; break;
        case GateType::H: L.rule = R_H; break;
        case GateType::S: L.rule = R_PHASE1; L.m[3] = cplx(0, 1); break;
        case GateType::T: L.rule = R_PHASE1; L.m[3] = cplx(r, r); break;
        case GateType::Sdag: L.rule = R_PHASE1; L.m[3] = cplx(0, -1); break;
        case GateType::Tdag: L.rule = R_PHASE1; L.m[3] = cplx(r, -r); break;
        case GateType::Rx:
            L.m[0] = c; L.m[1] = cplx(0, -s); L.m[2] = cplx(0, -s); L.m[3] = c;
            break;
        case GateType::Ry:
            L.m[0] = c; L.m[1] = -s; L.m[2] = s; L.m[3] = c;
            break;
        case GateType::Rz:
            L.m[0] = cplx(c, -s); L.m[1] = 0; L.m[2] = 0; L.m[3] = cplx(c, s);
            break;
        case GateType::CNOT:
            L.rule = R_SWAP; L.cmask = 1ull << g.qubits[0];
            break;
        case GateType::CZ:
            L.rule = R_NEG1; L.cmask = 1ull << g.qubits[0];
            break;
        case GateType::SWAP:
            L.rule = R_SWAP2; L.target = g.qubits[0]; L.target2 = g.qubits[1];
            break;
        case GateType::CRY:  // src/Gates.cu:322-351
            L.noop = set == CpuGateSet::Reference;
            L.cmask = 1ull << g.qubits[0];
            L.m[0] = c; L.m[1] = -s; L.m[2] = s; L.m[3] = c;
            break;
        case GateType::CRZ:  // src/Gates.cu:353-386
            L.noop = set == CpuGateSet::Reference;
            L.cmask = 1ull << g.qubits[0];
            L.m[0] = cplx(c, -s); L.m[1] = 0; L.m[2] = 0; L.m[3] = cplx(c, s);
            break;
        case GateType::Toffoli:  // src/Gates.cu:392-410
            L.noop = set == CpuGateSet::Reference;
            L.rule = R_SWAP;
            L.cmask = (1ull << g.qubits[0]) | (1ull << g.qubits[1]);
            break;
        default: throw std::runtime_error("Unknown gate type");
    }
    return L;
}

inline uint64_t insert_zeros(uint64_t k, const int* pos, int npos) {
    for (int i = 0; i < npos; ++i) {
        const uint64_t lo = k & ((1ull << pos[i]) - 1ull);
        k = ((k ^ lo) << 1) | lo;
    }
    return k;
}

constexpr uint64_t kSerialUnits = 1ull << 16;  // below this many pairs: the calling thread

}  // namespace

// Persistent worker pool: `run(parts, fn)` calls fn(part) for part in [0, parts) on the workers
// and the calling thread, and returns when all are done.  Waking parked threads costs a few
// microseconds, not the tens of a thread spawn per gate.
struct CPUSimulator::Pool {
    explicit Pool(int n) {
        for (int i = 1; i < n; ++i) workers.emplace_back([this, i] { loop(i); });
        size = n;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> l(mu);
            stop = true;
            ++gen;
        }
        cv.notify_all();
        for (auto& t : workers) t.join();
    }
    template <typename F>
    void run(int parts, F&& fn) {
        std::lock_guard<std::mutex> serial(run_mu);  // copies of one simulator share the pool
        {
            std::lock_guard<std::mutex> l(mu);
            job = [&fn](int p) { fn(p); };
            nparts = std::min(parts, size);
            pending = nparts - 1;
            ++gen;
        }
        cv.notify_all();
        fn(0);
        std::unique_lock<std::mutex> l(mu);
        done_cv.wait(l, [&] { return pending == 0; });
        job = nullptr;
    }
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(int)> j;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return gen != seen; });
                seen = gen;
                if (stop) return;
                if (id >= nparts) continue;
                j = job;
            }
            j(id);
            std::lock_guard<std::mutex> l(mu);
            if (--pending == 0) done_cv.notify_one();
        }
    }
    std::vector<std::thread> workers;
    std::mutex mu, run_mu;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    uint64_t gen = 0;
    int size = 1, nparts = 0, pending = 0;
    bool stop = false;
};

namespace {
template <typename P, typename F>
void parallel_blocks(P* pool, uint64_t units, F&& body) {
    if (!pool || pool->size <= 1 || units < kSerialUnits) {
        body(0, units);
        return;
    }
    const int parts = pool->size;
    const uint64_t per = (units + parts - 1) / parts;
    pool->run(parts, [&](int p) {
        const uint64_t b = per * (uint64_t)p, e = std::min(units, b + per);
        if (b < e) body(b, e);
    });
}
}  // namespace

CPUSimulator::CPUSimulator(int num_qubits, CpuGateSet gates)
    : num_qubits_(num_qubits), gate_set_(gates) {
    if (!isValidQubitCount(num_qubits))
        throw std::invalid_argument("Number of qubits must be between " +
                                    std::to_string(device_config::MIN_QUBITS) + " and " +
                                    std::to_string(device_config::MAX_QUBITS));
    const unsigned hc = std::thread::hardware_concurrency();
    setThreads((int)std::max(1u, std::min(16u, hc)));
    state_.assign(size_t(1) << num_qubits, cplx(0.0, 0.0));
    reset();
    rng_.seed(std::random_device{}());  // the reference seeds sample() from random_device
}

void CPUSimulator::setThreads(int threads) {
    threads_ = std::max(1, std::min(256, threads));
    pool_ = threads_ > 1 ? std::make_shared<Pool>(threads_) : nullptr;
}

void CPUSimulator::reset() {
    std::fill(state_.begin(), state_.end(), cplx(0.0, 0.0));
    state_[0] = cplx(1.0, 0.0);
}

void CPUSimulator::run(const Circuit& circuit) {
    if (circuit.getNumQubits() != num_qubits_)
        throw std::invalid_argument("Circuit qubit count doesn't match simulator");
    for (const GateOp& g : circuit.getGates()) applyGate(g);
}

void CPUSimulator::applyGate(const GateOp& gate) {
    for (int q : gate.qubits)
        if (q < 0 || q >= num_qubits_)
            throw std::out_of_range("Qubit index " + std::to_string(q) + " out of range [0, " +
                                    std::to_string(num_qubits_ - 1) + "]");
    if (gate.qubits.size() > 3 || gate.qubits.empty()) return;  // the reference dispatch ignores these
    const Lowered L = lower(gate, gate_set_);
    if (L.noop) return;
    cplx* st = state_.data();
    // fixed (zero-inserted) positions: target(s) and controls, ascending
    int pos[4], np = 0;
    uint64_t fixed = L.cmask | (1ull << L.target) | (L.target2 >= 0 ? 1ull << L.target2 : 0ull);
    for (int q = 0; q < num_qubits_; ++q)
        if ((fixed >> q) & 1ull) pos[np++] = q;
    const uint64_t units = 1ull << (num_qubits_ - np);
    const uint64_t tb = 1ull << L.target;
    const uint64_t set = L.cmask;
    const double r = constants::INV_SQRT2;
    auto body = [&](uint64_t b, uint64_t e) {
        for (uint64_t k = b; k < e; ++k) {
            const uint64_t i0 = insert_zeros(k, pos, np) | set;
            const uint64_t i1 = i0 | tb;
            switch (L.rule) {
                case R_SWAP: std::swap(st[i0], st[i1]); break;
                case R_Y: {
                    const cplx a0 = st[i0], a1 = st[i1];
                    st[i0] = cplx(0, -1) * a1;
                    st[i1] = cplx(0, 1) * a0;
                    break;
                }
                case R_NEG1: st[i1] = -st[i1]; break;
                case R_PHASE1: st[i1] = L.m[3] * st[i1]; break;
                case R_H: {
                    const cplx a0 = st[i0], a1 = st[i1];
                    st[i0] = (a0 + a1) * r;
                    st[i1] = (a0 - a1) * r;
                    break;
                }
                case R_SWAP2: {  // SWAP(q1, q2): exchange the 01 and 10 amplitudes
                    const uint64_t ia = i0 | (1ull << L.target2), ib = i0 | tb;
                    std::swap(st[ia], st[ib]);
                    break;
                }
                default: {
                    const cplx a0 = st[i0], a1 = st[i1];
                    st[i0] = L.m[0] * a0 + L.m[1] * a1;
                    st[i1] = L.m[2] * a0 + L.m[3] * a1;
                    break;
                }
            }
        }
    };
    parallel_blocks(pool_.get(), units, body);
}

std::vector<double> CPUSimulator::getProbabilities() const {
    std::vector<double> p(state_.size());
    const cplx* st = state_.data();
    double* out = p.data();
    parallel_blocks(pool_.get(), p.size(), [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; ++i) out[i] = std::norm(st[i]);
    });
    return p;
}

std::vector<int> CPUSimulator::sample(int n_shots) {
    // src/Simulator.cu:319-345: sequential partial_sum, one uniform per shot, lower_bound
    if (n_shots < 0) throw std::invalid_argument("n_shots must be non-negative");
    const std::vector<double> p = getProbabilities();
    std::vector<double> cdf(p.size());
    std::partial_sum(p.begin(), p.end(), cdf.begin());
    std::uniform_real_distribution<double> dist(0.0, 1.0);
    std::vector<int> out(n_shots);
    for (int& o : out) o = (int)(std::lower_bound(cdf.begin(), cdf.end(), dist(rng_)) - cdf.begin());
    return out;
}

}  // namespace qsim
