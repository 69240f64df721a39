// relabel.hip — layout-aware qubit relabeling for the fused passes (host code).
//
// A fused pass streams the state once, but how fast depends on WHICH 12 qubits its tile spans:
// gate-free probes of the same 32 GiB pass at 30 qubits take 5.15–9.05 ms depending on the
// tile's physical qubit positions (the memory system's address mapping; profiles/r02/layout/).
// Qubit labels are free to choose whenever the state is a computational basis state (|0..0> after
// construction or reset): relabeling a basis state is just another basis index.  So on the first
// fused run of a basis state the engine plans the circuit, picks a logical -> physical
// permutation that minimises the predicted cost of the plan's tiles (layout_cost.hpp, fitted to
// the probes by scripts/fit_layout_cost.py), and from then on applies every gate to the permuted
// qubits.  The permutation is undone by a fused SWAP network before anything reads or touches the
// amplitudes by index (capi.hip: canonicalize) — so results are exactly those of the
// unpermuted run up to the SWAPs' data movement (which is exact).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <random>
#include <vector>

#include "engine.hpp"
#include "layout_cost.hpp"

namespace qsim_hip {

// Policy: QSIM_RELABEL (0 off, 1 on: default), QSIM_RELABEL_MIN_QUBITS (default 26: the HBM-bound
// sizes the layout model was measured on; for the sharded engine the LOCAL qubit count);
// qsim_set_relabel overrides both.
static std::atomic<int> g_relabel{-1}, g_relabel_min{-1};
static void relabel_defaults() {
    if (g_relabel.load() < 0) {
        const char* e = std::getenv("QSIM_RELABEL");
        g_relabel.store(e ? std::atoi(e) : 1);
    }
    if (g_relabel_min.load() < 0) {
        const char* e = std::getenv("QSIM_RELABEL_MIN_QUBITS");
        g_relabel_min.store(e ? std::atoi(e) : 26);
    }
}
bool relabel_enabled(int n) {
    relabel_defaults();
    return g_relabel.load() != 0 && n >= g_relabel_min.load();
}
void relabel_configure(int mode, int min_qubits) {
    relabel_defaults();
    if (mode >= 0) g_relabel.store(mode);
    if (min_qubits >= 0) g_relabel_min.store(min_qubits);
}

double layout_cost_us(uint64_t tile) {
    using namespace layout_cost;
    double c = kBase;
    int q[64];
    int k = 0;
    for (uint64_t m = tile; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        if (b >= kQ0 && b < kN) q[k++] = b;
    }
    for (int i = 0; i < k; ++i) {
        c += kW1[q[i]];
        for (int j = i + 1; j < k; ++j) c += kW2[q[i]][q[j]];
    }
    return c;
}

std::vector<uint64_t> plan_tiles(const Plan& plan) {
    std::vector<uint64_t> t;
    for (const FusedPass& p : plan.passes) {
        if (p.single >= 0 || p.h < 4) continue;
        uint64_t m = (1ull << p.r0) - 1ull;
        for (int i = 0; i < 6 + p.h - p.r0; ++i) m |= 1ull << p.hpos[i];
        t.push_back(m);
    }
    return t;
}

double plan_layout_cost_us(const Plan& plan) {
    double c = 0.0;
    for (uint64_t t : plan_tiles(plan)) c += layout_cost_us(t);
    return c;
}

static uint64_t map_mask(uint64_t m, const std::vector<int>& pi) {
    uint64_t r = 0;
    for (; m; m &= m - 1) r |= 1ull << pi[__builtin_ctzll(m)];
    return r;
}

// Simulated annealing over permutations of the qubits >= kFixed (the contiguous run bits every
// tile contains stay put), deterministic (fixed seeds).  Returns an empty vector when nothing
// beats the identity by at least min_gain (fraction).
std::vector<int> choose_relabel(const std::vector<uint64_t>& tiles, int n, double* before, double* after,
                                double min_gain) {
    constexpr int kFixed = 4;
    std::vector<int> id(n);
    for (int q = 0; q < n; ++q) id[q] = q;
    auto total = [&](const std::vector<int>& pi) {
        double c = 0.0;
        for (uint64_t t : tiles) c += layout_cost_us(map_mask(t, pi));
        return c;
    };
    const double c0 = total(id);
    if (before) *before = c0;
    if (after) *after = c0;
    if (tiles.empty() || n - kFixed < 2) return {};
    std::vector<int> best = id;
    double bc = c0;
    for (int restart = 0; restart < 6; ++restart) {
        std::mt19937 rng(0x5eed + restart);
        std::vector<int> pi = id;
        if (restart > 0) std::shuffle(pi.begin() + kFixed, pi.end(), rng);
        double cur = total(pi), T = 200.0;  // microseconds
        std::uniform_int_distribution<int> pick(kFixed, n - 1);
        std::uniform_real_distribution<double> u01(0.0, 1.0);
        for (int it = 0; it < 6000; ++it) {
            const int a = pick(rng), b = pick(rng);
            if (a == b) continue;
            std::swap(pi[a], pi[b]);
            const double c = total(pi);
            if (c < cur || u01(rng) < std::exp((cur - c) / T)) cur = c;
            else std::swap(pi[a], pi[b]);
            T *= 0.999;
            if (cur < bc) {
                bc = cur;
                best = pi;
            }
        }
    }
    if (bc > c0 * (1.0 - min_gain)) return {};
    if (after) *after = bc;
    return best;
}

}  // namespace qsim_hip
