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
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
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
bool relabel_mode_on() {
    relabel_defaults();
    return g_relabel.load() != 0;
}
void relabel_configure(int mode, int min_qubits) {
    relabel_defaults();
    if (mode >= 0) g_relabel.store(mode);
    if (min_qubits >= 0) g_relabel_min.store(min_qubits);
}

// Process-wide memo of layout choices: the same circuit on a reset state (trajectory loops,
// one state per shot batch, benchmark repetitions) re-uses the decision instead of planning the
// candidates again.  Keyed by (n, kind, tile height, tile-constant controls on / off, the exact
// gate bytes); LRU of kMemo entries.
namespace {
struct MemoEntry {
    int n, kind;
    std::vector<unsigned char> key;
    std::vector<int> perm;
    int h;  // the tile height decided with the labels (cross-height calibration), or -1
    uint64_t used;
};
std::mutex g_memo_mu;
std::vector<MemoEntry> g_memo;
uint64_t g_memo_clock = 0;
constexpr size_t kMemo = 16;
}  // namespace

bool layout_memo_get(int n, int kind, const void* gates, size_t bytes, std::vector<int>& perm, int* h) {
    std::lock_guard<std::mutex> l(g_memo_mu);
    // a choice made for one tile height only, unless the height was chosen with it (h != null)
    kind = (kind * 16 + (h ? 15 : tile_height_default())) * 2 + (tile_ctrl_out() ? 1 : 0);
    for (MemoEntry& e : g_memo)
        if (e.n == n && e.kind == kind && e.key.size() == bytes && std::memcmp(e.key.data(), gates, bytes) == 0) {
            e.used = ++g_memo_clock;
            perm = e.perm;
            if (h) *h = e.h;
            return true;
        }
    // a decision another process made on this machine (cache.hip), taken into this process's memo
    int dh = -1;
    std::vector<int> dp;
    if (!layout_cache_load(n, kind, gates, bytes, dp, &dh)) return false;
    if (g_memo.size() >= kMemo)
        g_memo.erase(std::min_element(g_memo.begin(), g_memo.end(),
                                      [](const MemoEntry& a, const MemoEntry& b) { return a.used < b.used; }));
    const unsigned char* p = static_cast<const unsigned char*>(gates);
    g_memo.push_back(MemoEntry{n, kind, std::vector<unsigned char>(p, p + bytes), dp, dh, ++g_memo_clock});
    perm = dp;
    if (h) *h = dh;
    return true;
}
void layout_memo_put(int n, int kind, const void* gates, size_t bytes, const std::vector<int>& perm, int h) {
    std::lock_guard<std::mutex> l(g_memo_mu);
    if (g_memo.size() >= kMemo)
        g_memo.erase(std::min_element(g_memo.begin(), g_memo.end(),
                                      [](const MemoEntry& a, const MemoEntry& b) { return a.used < b.used; }));
    kind = (kind * 16 + (h >= 0 ? 15 : tile_height_default())) * 2 + (tile_ctrl_out() ? 1 : 0);
    const unsigned char* p = static_cast<const unsigned char*>(gates);
    g_memo.push_back(MemoEntry{n, kind, std::vector<unsigned char>(p, p + bytes), perm, h, ++g_memo_clock});
    layout_cache_store(n, kind, gates, bytes, h, perm);
}

// Cross-height calibration (QSIM_CALIBRATE_HEIGHTS, default 1; needs layout calibration, i.e.
// inline compilation): the first run of a basis state also times 13-qubit-tile candidates
// against 12-qubit ones (or the reverse) unless a tile height was set explicitly.
bool calibrate_heights(int n) {
    static const int v = [] {
        const char* e = std::getenv("QSIM_CALIBRATE_HEIGHTS");
        return e ? std::atoi(e) : 1;
    }();
    return v != 0 && relabel_calibrate(n) && !tile_height_is_set();
}

static std::atomic<int> g_calib{-1}, g_calib_min{-1};
bool relabel_calibrate(int n) {
    if (g_calib.load() < 0) {
        const char* e = std::getenv("QSIM_RELABEL_CALIBRATE");
        g_calib.store(e ? std::atoi(e) : 1);
    }
    if (g_calib_min.load() < 0) {
        const char* e = std::getenv("QSIM_RELABEL_CALIBRATE_MIN_QUBITS");
        g_calib_min.store(e ? std::atoi(e) : 26);
    }
    return g_calib.load() != 0 && n >= g_calib_min.load() && jit_mode() == 2;
}
bool calibrate_mode_on() {
    relabel_calibrate(0);  // defaults first
    return g_calib.load() != 0;
}
void calibrate_configure(int mode, int min_qubits) {
    relabel_calibrate(0);  // defaults first
    if (mode >= 0) g_calib.store(mode);
    if (min_qubits >= 0) g_calib_min.store(min_qubits);
}

int relabel_tries() {
    static const int v = [] {
        const char* e = std::getenv("QSIM_RELABEL_TRIES");
        return e ? std::max(0, std::atoi(e)) : 7;
    }();
    return v;
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
    // The model was fitted on 12-qubit tiles; a 13-qubit tile (one 128 KiB workgroup per CU,
    // persistent pipelined kernel) streams ~1.2-1.3x slower per pass (profiles/r02/h7s/).
    // QSIM_LAYOUT_T13 scales its predicted cost, steering the label search toward plans whose
    // passes fit 12-qubit tiles (mixed heights): 1.25 gave W-HC 30q seed 42 at h = 7 4 224 gates/s
    // but 28q 16.2 k instead of 18.3 k (profiles/r02/mix2/), so the default stays 1.
    if (__builtin_popcountll(tile) >= 13) c *= layout_t13();
    return c;
}
static thread_local double t_t13 = -1.0;  // LayoutT13Scope of the calling thread
double layout_t13() {
    if (t_t13 >= 0.0) return t_t13;
    static const double env = [] {
        const char* e = std::getenv("QSIM_LAYOUT_T13");
        return e ? std::atof(e) : 1.0;
    }();
    return env;
}
LayoutT13Scope::LayoutT13Scope(double f) : prev_(t_t13) { t_t13 = f; }
LayoutT13Scope::~LayoutT13Scope() { t_t13 = prev_; }

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

// Full layout choice for one circuit.  The labels also steer the pass planner (its run bits are
// physical qubits 0..r0-1, and its searches break ties by position): W-HC at 28 qubits plans into
// 6 passes as labelled but into 5 under about half of all random relabelings.  So: plan the
// circuit under the identity and `tries` seeded random permutations (in parallel), keep the
// fewest-pass candidates, anneal each one's layout (positions >= 4) on the cost model, and take
// the cheapest; accepted only when it plans into fewer passes than the identity, or as many and
// >= 3 % cheaper.  `lower` maps the caller's gates through a permutation and lowers them exactly
// as the caller will (so the returned plan can be cached under the same key).
LayoutChoice choose_layout(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                           int tries, size_t want_alts, double stage_us) {
    const int h = tile_height_default();  // the calling thread's height, for the worker threads too
    const double t13 = layout_t13();      // and its 13-qubit tile cost factor
    const bool ctrl_out = tile_ctrl_out();  // (CtrlOutOff is per thread: carried into the workers)
    struct Cand {
        std::vector<int> pi;
        size_t passes = 0;
        std::vector<uint64_t> tiles;
        double cost = 0.0;
    };
    std::vector<Cand> cand(1 + std::max(0, tries));
    for (size_t k = 0; k < cand.size(); ++k) {
        cand[k].pi.resize(n);
        for (int q = 0; q < n; ++q) cand[k].pi[q] = q;
        if (k > 0) {
            std::mt19937 rng(0x1abe1u + (unsigned)k);
            std::shuffle(cand[k].pi.begin(), cand[k].pi.end(), rng);
        }
    }
    auto plan_cand = [&](Cand& c) {
        try {  // (worker threads must not throw; a failed candidate just never wins)
            const Plan p = plan_fused(lower(c.pi), n, h);
            c.passes = p.passes.size();
            c.tiles = plan_tiles(p);
            c.cost = 0.0;
            for (uint64_t t : c.tiles) c.cost += layout_cost_us(t);
        } catch (...) {
            c.passes = SIZE_MAX;
        }
    };
    {
        std::vector<std::thread> th;
        for (size_t k = 0; k < cand.size(); ++k)
            th.emplace_back([&, k] {
                const LayoutT13Scope sc(t13);
                std::unique_ptr<CtrlOutOff> off;  // (the caller's tile-control rule, per thread)
                if (!ctrl_out) off = std::make_unique<CtrlOutOff>();
                plan_cand(cand[k]);
            });
        for (auto& t : th) t.join();
    }
    LayoutChoice out;
    if (cand[0].passes == SIZE_MAX) return out;  // the caller's own planning reports the error
    out.passes_before = cand[0].passes;
    out.cost_before = out.cost_after = cand[0].cost;
    size_t best_passes = cand[0].passes;
    for (const Cand& c : cand) best_passes = std::min(best_passes, c.passes);
    // anneal the layout of every fewest-pass candidate (positions 0..3 stay where it put them)
    std::vector<size_t> pool;
    for (size_t k = 0; k < cand.size(); ++k)
        if (cand[k].passes == best_passes) pool.push_back(k);
    std::vector<std::vector<int>> total(pool.size());
    std::vector<double> pred(pool.size());
    {
        std::vector<std::thread> th;
        for (size_t i = 0; i < pool.size(); ++i)
            th.emplace_back([&, i] {
                const LayoutT13Scope sc(t13);
                std::unique_ptr<CtrlOutOff> off;
                if (!ctrl_out) off = std::make_unique<CtrlOutOff>();
                const Cand& c = cand[pool[i]];
                double b = 0.0, a = 0.0;
                std::vector<int> sigma;
                try {
                    sigma = choose_relabel(c.tiles, n, &b, &a, 0.0);
                } catch (...) {
                }
                total[i] = c.pi;
                if (!sigma.empty())
                    for (int q = 0; q < n; ++q) total[i][q] = sigma[c.pi[q]];
                pred[i] = sigma.empty() ? c.cost : a;
            });
        for (auto& t : th) t.join();
    }
    if (stage_us > 0.0) {  // rank by the annealed plans' cost + stages (see the declaration)
        std::vector<std::thread> th;
        for (size_t i = 0; i < pool.size(); ++i)
            th.emplace_back([&, i] {
                const LayoutT13Scope sc(t13);
                std::unique_ptr<CtrlOutOff> off;
                if (!ctrl_out) off = std::make_unique<CtrlOutOff>();
                try {
                    const Plan p = plan_fused(lower(total[i]), n, h);
                    int st = 0;
                    for (const FusedPass& fp : p.passes) st += fp.stage_end - fp.stage_begin;
                    pred[i] = plan_layout_cost_us(p) + stage_us * st;
                } catch (...) {
                    pred[i] = 1e300;
                }
            });
        for (auto& t : th) t.join();
    }
    std::vector<size_t> order(pool.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return pred[a] < pred[b]; });
    bool chosen = false;  // the first acceptable candidate; then up to want_alts alternatives
    for (size_t i : order) {
        // the annealed labels may steer the planner differently: verify, else the candidate as is
        for (int variant = 0; variant < 2; ++variant) {
            const std::vector<int>& pi = variant == 0 ? total[i] : cand[pool[i]].pi;
            std::vector<Op> ops = lower(pi);
            Plan plan = plan_fused(ops, n, h);
            const double cost = plan_layout_cost_us(plan);
            const bool fewer = plan.passes.size() < out.passes_before;
            const bool cheaper = plan.passes.size() == out.passes_before && cost < out.cost_before * 0.97;
            if (plan.passes.size() > best_passes || !(fewer || cheaper)) continue;
            bool identity = true;
            for (int q = 0; q < n; ++q) identity = identity && pi[q] == q;
            if (identity) return out;
            if (!chosen) {
                out.perm = pi;
                out.ops = std::move(ops);
                out.plan = std::move(plan);
                out.cost_after = cost;
                chosen = true;
            } else if (plan.passes.size() == out.plan.passes.size() && pi != out.perm) {
                out.alts.push_back(LayoutChoice::Alt{pi, std::move(ops), std::move(plan)});
            }
            break;
        }
        if (chosen && out.alts.size() >= want_alts) break;
    }
    return out;
}

}  // namespace qsim_hip
