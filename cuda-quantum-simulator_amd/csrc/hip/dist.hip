// dist.hip — state vector sharded over the GPUs of one node, one process per GPU, RCCL over xGMI.
//
// The reference is single-GPU (README.md:361-367); SURVEY §8(e) specifies this extension.
//
// Layout: W = 2^g ranks, L = n - g local qubits.  Rank r owns the 2^L amplitudes whose top g
// PHYSICAL index bits equal r.  Every rank keeps the same logical->physical qubit map `perm`:
//   * SWAP gates only exchange two map entries (zero data movement);
//   * controls on global (rank) bits are resolved per rank (the op is dropped on ranks whose bit
//     is 0, the control is dropped on the others); a diagonal gate whose target is global becomes a
//     uniform phase on the rank's shard;
//   * a gate whose TARGET is global needs data from another rank: before it, the planner remaps
//     qubits — the g logical qubits whose next use as a target lies furthest ahead become global —
//     and executes the remap as one all-to-all: pack (gather the 2^k - 1 outgoing chunks by their
//     local bits) -> grouped ncclSend/ncclRecv with the 2^k - 1 peers -> unpack.  With k = g all
//     W - 1 xGMI links of every GPU carry 1/W of its shard concurrently.
// Local work between remaps is the single-GPU engine (fused tile passes) on the 2^L shard.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "device_ops.hpp"
#include "engine.hpp"
#include "qsim_hip.h"

using namespace qsim_hip;

namespace qsim_hip {

struct DStep {
    int kind = 0;  // 0 ops, 1 exchange
    int k = 0;
    int gpos[8] = {0}, lpos[8] = {0};
    std::vector<Op> ops;
    // Overlap of a remap with local work (mark_overlap): an exchange with pivots (pmask != 0, up
    // to kMaxPivots local physical positions) runs as 2^m part-exchanges, one per value of the
    // pivot bits.  An ops step with role bit 1 runs the trailing passes of its fused plan that
    // avoid the pivots of the exchange after it per part (so part j's transfer overlaps the later
    // parts' passes); role bit 2: the leading passes that avoid the pivots of the exchange before
    // it run per part, each as soon as its part has landed.  The step's plan is the same one-piece
    // fused plan either way (no extra passes).  `pivot`: the lowest pivot (-1: none).
    int pivot = -1, role = 0;
    uint64_t pmask = 0;
    // Coarse parts (round 5; exchange steps): a subset of pmask that the step before's passes just
    // ahead of its per-part tail leave untouched.  Those passes (which do touch the other pivots)
    // run per value of these bits, each coarse part followed at once by the tail of its fine parts,
    // so the first part can leave after 1/2^|coarse| of them instead of after all of them.  Parts
    // are exchanged in coarse-major order (part_order).  0: none.
    uint64_t coarse = 0;
    // planning only: the circuit gates emitted into this step (rank-independent), their physical
    // qubit masks, and for each op the index of the gate (in this list) it came from
    std::vector<uint64_t> gmask;
    std::vector<int> op_gate;
};

constexpr int kMaxPivots = 4;
constexpr int kMaxParts = 1 << kMaxPivots;  // part-exchanges of one overlapped remap
// QSIM_DIST_COARSE=0: no coarse parts (DStep::coarse; read once)
static bool coarse_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("QSIM_DIST_COARSE");
        return e == nullptr || std::atoi(e) != 0;
    }();
    return v;
}
// QSIM_DIST_CARRY=1 (experimental, off by default; read per call so tests can switch it): a run's
// last step is left pending and merged into the next run's first step (qsim_dist_run).
bool carry_enabled() {
    const char* e = std::getenv("QSIM_DIST_CARRY");
    return e != nullptr && std::atoi(e) != 0;
}
// The positions of `mask` that pass p's tile touches (all of them for a per-gate step or a tile
// below 4 free bits: such passes never run as sub-space launches).
static uint64_t pass_touches(const FusedPass& p, uint64_t mask) {
    if (p.single >= 0 || p.h < 4) return mask;
    uint64_t t = 0;
    for (int i = 0; i < 6 + p.h - p.r0; ++i) t |= mask & (1ull << p.hpos[i]);
    return t;
}
// Coarse split of the passes [lo, hi) of a plan just ahead of its per-part tail, for pivots `set`:
// the count c of passes (ending at hi) and the coarse bits (pivots none of them touches) that
// minimise the exposed work (hi - lo - c) + c / 2^|coarse| (in passes).  *cb = 0, 0: none.
static int coarse_split(const Plan& pl, int lo, int hi, uint64_t set, uint64_t* cb) {
    int best_c = 0;
    uint64_t best_cb = 0, U = 0;
    double best = (double)(hi - lo);
    for (int c = 1; c <= hi - lo; ++c) {
        U |= pass_touches(pl.passes[hi - c], set);
        const uint64_t b = set & ~U;
        if (!b) break;
        const double e = (double)(hi - lo - c) + (double)c / (double)(1 << __builtin_popcountll(b));
        if (e < best - 1e-9) {
            best = e;
            best_c = c;
            best_cb = b;
        }
    }
    *cb = best_cb;
    return best_c;
}
// Exchange order of the K parts of an overlapped remap with pivots pmask and coarse bits cb:
// coarse-major (part index bit j = the j-th pivot; the coarse pivots' bits vary slowest), so the
// parts of the first coarse part, whose passes finish first, leave first.  Rank-independent.
static void part_order(uint64_t pmask, uint64_t cb, int* order) {
    const int m = __builtin_popcountll(pmask), K = 1 << m;
    uint64_t ch = 0;  // coarse pivots as part-index bits
    {
        int j = 0;
        for (uint64_t mm = pmask; mm; mm &= mm - 1, ++j)
            if ((cb >> __builtin_ctzll(mm)) & 1ull) ch |= 1ull << j;
    }
    const uint64_t fh = (uint64_t)(K - 1) & ~ch;
    const int Kc = 1 << __builtin_popcountll(ch), Kf = K / Kc;
    int i = 0;
    for (int cv = 0; cv < Kc; ++cv)
        for (int f = 0; f < Kf; ++f) {
            uint64_t h = 0;
            int a = 0, b = 0;
            for (int j = 0; j < m; ++j) {
                if ((ch >> j) & 1ull) h |= (uint64_t)((cv >> a++) & 1) << j;
                else h |= (uint64_t)((f >> b++) & 1) << j;
            }
            order[i++] = (int)h;
        }
    (void)fh;
}
static bool pass_avoids(const FusedPass& p, uint64_t pmask) {
    if (p.single >= 0 || p.h < 4) return false;
    for (int i = 0; i < 6 + p.h - p.r0; ++i)
        if ((pmask >> p.hpos[i]) & 1ull) return false;
    return true;
}
static uint64_t deposit_bits(uint64_t v, uint64_t mask) {  // bit j of v -> j-th set bit of mask
    uint64_t r = 0;
    for (int j = 0; mask; mask &= mask - 1, ++j) r |= ((v >> j) & 1ull) << __builtin_ctzll(mask);
    return r;
}

// Choose, for every exchange between two ops steps, its pivots (QSIM_DIST_OVERLAP=0 disables).
// The ops steps are not split: each rank plans a step as one fused plan (tiles padded away from
// the pivots) and runs per part only the passes at its ends that avoid them (qsim_dist_run).
// Time model of one remap between steps A and B (pass time 1, transfer time R, K = 2^m parts,
// t trailing passes of A and h leading passes of B avoiding the pivots):
//     T = max(R + (nA - t) + (nB - h) + (t + h) / K,  nA + nB + R / K)
// with R = 50 / world (an HBM pass at ~6 TB/s over a remap that sends 1/world of the shard per
// link at ~60 GB/s).  Pivots are local positions >= 6 (never a tile's contiguous run) outside the
// exchanged positions, added greedily (up to kMaxPivots) while T drops; each candidate set is
// scored by planning both steps with it avoided, in parallel, on RANK 0's ops (`ref`: the same
// skeleton on every rank), so every rank picks the same pivots.  Everything else the score reads
// is rank-independent too: the positions the step before must also avoid come from this rank's
// own marks (`steps`, set by the same decisions on every rank), never from `ref`'s roles (which
// are only marked when `ref` aliases `steps`, i.e. on rank 0).  QSIM_DIST_PIVOTS caps m
// (default kMaxPivots); QSIM_DIST_PIVOT_PLAN=0: one pivot by the cheaper gate-level score
// (trailing / leading gates that do not touch the position).
// carry: pivots of the previous run's last exchange whose parts are still in flight when this
// run starts (qsim_dist_run merges that run's last step into this one's first): the first ops
// step's leading passes that avoid them run per part too (role bit 2 on step 0).
// next_ops: the first ops step of the NEXT run of the circuit (from this run's end map, rank 0's
// lowering): the last remap's pivots are also scored by the passes of it they let run per part
// (carried into the next run, qsim_dist_run).
static void mark_overlap(std::vector<DStep>& steps, int L, int world, const std::vector<DStep>& ref,
                         uint64_t carry = 0, const std::vector<Op>* next_ops = nullptr) {
    static const int enabled = [] {
        const char* e = std::getenv("QSIM_DIST_OVERLAP");
        return e ? std::atoi(e) : 1;
    }();
    static const int by_plan = [] {
        const char* e = std::getenv("QSIM_DIST_PIVOT_PLAN");
        return e ? std::atoi(e) : 1;
    }();
    static const int max_piv = [] {
        const char* e = std::getenv("QSIM_DIST_PIVOTS");
        return e ? std::max(1, std::min(kMaxPivots, std::atoi(e))) : kMaxPivots;
    }();
    if (!enabled || L < 8) return;
    if (carry && !steps.empty() && steps[0].kind == 0) steps[0].role |= 2;
    const int min_gates = 4;
    static const double r_scale = [] {  // QSIM_DIST_MODEL_R (experiments): R x world, default 50
        const char* e = std::getenv("QSIM_DIST_MODEL_R");
        return e ? std::atof(e) : 50.0;
    }();
    const double R = r_scale / std::max(2, world);
    for (size_t i = 1; i + 1 < steps.size(); ++i) {
        DStep& ex = steps[i];
        DStep& A = steps[i - 1];
        DStep& B = steps[i + 1];
        if (ex.kind != 1 || A.kind != 0 || B.kind != 0) continue;
        uint64_t lmask = 0;
        for (int j = 0; j < ex.k; ++j) lmask |= 1ull << ex.lpos[j];
        int best_p = -1, best = 0;
        std::vector<int> cand;
        for (int p = 6; p < L; ++p) {
            if ((lmask >> p) & 1ull) continue;
            cand.push_back(p);
            const uint64_t bit = 1ull << p;
            int a = 0, b = 0;
            while (a < (int)A.gmask.size() && !(A.gmask[A.gmask.size() - 1 - a] & bit)) ++a;
            while (b < (int)B.gmask.size() && !(B.gmask[b] & bit)) ++b;
            if (a + b > best) {
                best_p = p;
                best = a + b;
            }
        }
        uint64_t pmask = best_p >= 0 && best >= min_gates ? 1ull << best_p : 0ull;
        const DStep& rA = ref[i - 1];
        const DStep& rB = ref[i + 1];
        if (by_plan && !rA.ops.empty() && !rB.ops.empty() && !cand.empty()) {
            const uint64_t avoidA0 = (A.role & 2) ? (i >= 2 ? steps[i - 2].pmask : carry) : 0ull;
            // T of a pivot set (pass counts in units of one pass); +inf when planning failed;
            // *cb_out: the coarse bits of that set (coarse_split)
            auto model = [&](uint64_t set, uint64_t* cb_out = nullptr) {
                const Plan pA = plan_fused(rA.ops, L, -1, set, avoidA0);
                const Plan pB = plan_fused(rB.ops, L, -1, 0, set);
                const int na = (int)pA.passes.size(), nb = (int)pB.passes.size();
                int t = 0, h = 0, ha = 0;
                // A's leading passes that run per part of the exchange before it (or of the
                // previous run's last one, `carry`) are hidden behind that exchange; the trailing
                // ones that avoid this set feed this one (a pass counts once: head first, as the
                // run splits a step)
                if (avoidA0)
                    while (ha < na && pass_avoids(pA.passes[ha], avoidA0)) ++ha;
                while (t < na - ha && pass_avoids(pA.passes[na - 1 - t], set)) ++t;
                while (h < nb && pass_avoids(pB.passes[h], set)) ++h;
                const double K = (double)(1 << __builtin_popcountll(set));
                if (t + h == 0) return 1e30;
                // The next run's first pass, if it avoids the set, is hidden behind this remap too
                // (carried, qsim_dist_run); at most one is credited — more would only shorten that
                // run's own tail, whose remap hides it anyway (crediting them all makes the greedy
                // pick few pivots: big parts, a long exposed last part).  A's leading `ha` passes
                // were hidden behind the remap before this one and cost nothing here.
                int hn = 0;
                if (next_ops && !next_ops->empty() && i + 2 == steps.size() && h == nb && !(B.role & 1)) {
                    const Plan pN = plan_fused(*next_ops, L, -1, set);
                    hn = !pN.passes.empty() && pass_avoids(pN.passes[0], set) ? 1 : 0;
                }
                // the passes just ahead of the tail run per coarse part (coarse_split)
                uint64_t cb = 0;
                const int c = coarse_enabled() ? coarse_split(pA, ha, na - t, set, &cb) : 0;
                if (cb_out) *cb_out = cb;
                const double exposed = (double)(na - t - ha - c) + (c ? (double)c / (double)(1 << __builtin_popcountll(cb)) : 0.0);
                return std::max(R + exposed + (nb - h) + (t + h + hn) / K - hn, na + nb + R / K);
            };
            auto score_all = [&](uint64_t base, const std::vector<int>& cs) {
                std::vector<double> sc(cs.size(), 1e30);
                std::vector<std::thread> th;
                for (size_t c = 0; c < cs.size(); ++c)
                    th.emplace_back([&, c] {
                        try {  // (worker threads must not throw; a failed candidate just loses)
                            sc[c] = model(base | (1ull << cs[c]));
                        } catch (...) {
                        }
                    });
                for (auto& t : th) t.join();
                return sc;
            };
            // round 1: every single position; later rounds: a beam of the kBeam best sets, each
            // grown by one of the kPool best singles (the greedy of round 4 kept one set: it missed
            // sets whose first pass leaves a pivot untouched, i.e. coarse parts, round 5)
            constexpr size_t kBeam = 4, kPool = 10;
            std::vector<double> sc1 = score_all(0, cand);
            std::vector<size_t> order(cand.size());
            for (size_t c = 0; c < order.size(); ++c) order[c] = c;
            std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return sc1[a] < sc1[b]; });
            double bestT = sc1[order[0]];
            uint64_t set = bestT < 1e29 ? 1ull << cand[order[0]] : 0ull;
            std::vector<int> pool;
            std::vector<std::pair<double, uint64_t>> beam;
            for (size_t c = 0; c < order.size() && pool.size() < kPool; ++c)
                if (sc1[order[c]] < 1e29) {
                    pool.push_back(cand[order[c]]);
                    if (beam.size() < kBeam) beam.push_back({sc1[order[c]], 1ull << cand[order[c]]});
                }
            for (int m = 1; set && m < max_piv && !beam.empty(); ++m) {
                std::vector<uint64_t> sets;
                for (const auto& b : beam)
                    for (int q : pool) {
                        const uint64_t s2 = b.second | (1ull << q);
                        if (s2 != b.second && std::find(sets.begin(), sets.end(), s2) == sets.end()) sets.push_back(s2);
                    }
                std::vector<double> sc(sets.size(), 1e30);
                {
                    std::vector<std::thread> th;
                    const size_t nt = std::min<size_t>(sets.size(), 16);
                    for (size_t w = 0; w < nt; ++w)
                        th.emplace_back([&, w] {
                            for (size_t c = w; c < sets.size(); c += nt) try {
                                    sc[c] = model(sets[c]);
                                } catch (...) {
                                }
                        });
                    for (auto& t : th) t.join();
                }
                std::vector<size_t> o2(sets.size());
                for (size_t c = 0; c < o2.size(); ++c) o2[c] = c;
                std::sort(o2.begin(), o2.end(), [&](size_t a, size_t b) {
                    return sc[a] != sc[b] ? sc[a] < sc[b] : sets[a] < sets[b];  // (deterministic)
                });
                beam.clear();
                for (size_t c = 0; c < o2.size() && beam.size() < kBeam; ++c)
                    if (sc[o2[c]] < 1e29) beam.push_back({sc[o2[c]], sets[o2[c]]});
                if (!beam.empty() && beam[0].first < bestT - 1e-9) {
                    bestT = beam[0].first;
                    set = beam[0].second;
                }
            }
            if (set) {
                pmask = set;
                try {
                    (void)model(set, &ex.coarse);
                } catch (...) {
                    ex.coarse = 0;
                }
            }
        }
        if (!pmask) continue;
        ex.pmask = pmask;
        ex.pivot = __builtin_ctzll(pmask);
        A.role |= 1;
        B.role |= 2;
    }
}

// Logical target that must be local for gate g (2x2 ops), or -1 (diagonal, SWAP).
static int needs_local(const qsim_gate& g) {
    switch (g.type) {
        case QSIM_GATE_X: case QSIM_GATE_Y: case QSIM_GATE_H: case QSIM_GATE_RX: case QSIM_GATE_RY:
            return g.qubits[0];
        case QSIM_GATE_CNOT: case QSIM_GATE_CRY:
            return g.qubits[1];
        case QSIM_GATE_TOFFOLI:
            return g.qubits[2];
        default:
            return -1;
    }
}

// QSIM_DIST_FULL_REMAP=0 lets a remap move only the globals that must leave (fewer bytes, fewer
// links); the default swaps all of them (see plan_dist).
static bool full_remap() {
    static const bool v = [] {
        const char* e = std::getenv("QSIM_DIST_FULL_REMAP");
        return e == nullptr || std::atoi(e) != 0;
    }();
    return v;
}

static uint64_t gate_qmask(const qsim_gate& g) {
    uint64_t m = 0;
    for (int j = 0; j < g.nqubits; ++j) m |= 1ull << g.qubits[j];
    return m;
}

// Gates of `window` (indices into `gates`, in program order) that can run before any further
// remap when the logical qubits in `glob` are global: a gate runs unless its target is global or
// an earlier gate that shares a qubit with it could not run.  SWAPs relabel `glob`.
static int count_runnable(const qsim_gate* gates, const std::vector<uint64_t>& qm,
                          const std::vector<int>& window, size_t upto, uint64_t glob) {
    uint64_t blocked = 0;
    int cnt = 0;
    for (size_t w = 0; w < upto; ++w) {
        const int i = window[w];
        const qsim_gate& gt = gates[i];
        if (qm[i] & blocked) {
            blocked |= qm[i];
            continue;
        }
        if (gt.type == QSIM_GATE_SWAP) {
            const uint64_t a = 1ull << gt.qubits[0], b = 1ull << gt.qubits[1];
            if (((glob & a) != 0) != ((glob & b) != 0)) glob ^= a | b;
            continue;
        }
        const int tq = needs_local(gt);
        if (tq >= 0 && ((glob >> tq) & 1ull)) {
            blocked |= qm[i];
            continue;
        }
        ++cnt;
    }
    return cnt;
}

// The logical qubits to make global at a remap.  Scored, in order, by the gates that can then run
// before the next remap (i) in the rest of this circuit and (ii) over the rest plus one more run
// of the circuit (a benchmark or trajectory loop re-runs it from the map this run ends with), then
// by the physical positions of the incoming qubits (high positions give long pack runs).
// Exhaustive over the candidate g-sets when that is cheap (C(27,3) = 2925 at 30 qubits on 8
// ranks), greedy one qubit at a time otherwise.
static uint64_t choose_globals(const qsim_gate* gates, size_t count, const std::vector<uint64_t>& qm,
                               const std::vector<char>& done, const std::vector<int>& perm, int n,
                               int g, int L, bool full) {
    std::vector<int> window;
    for (size_t i = 0; i < count; ++i)
        if (!done[i]) window.push_back((int)i);
    const size_t rest = window.size();
    const size_t cap = std::max<size_t>(rest, 1024);
    for (size_t i = 0; i < count && window.size() < cap; ++i) window.push_back((int)i);
    std::vector<int> cand;  // full remap: every current global leaves, so only locals may enter
    for (int q = 0; q < n; ++q)
        if (!full || perm[q] < L) cand.push_back(q);
    struct Score {
        int a = -1, b = -1, c = -1;
        bool operator<(const Score& o) const {
            return a != o.a ? a < o.a : (b != o.b ? b < o.b : c < o.c);
        }
    };
    auto score = [&](uint64_t set) {
        Score s;
        s.a = count_runnable(gates, qm, window, rest, set);
        s.b = count_runnable(gates, qm, window, window.size(), set);
        s.c = 0;
        for (int q = 0; q < n; ++q)
            if ((set >> q) & 1ull) s.c += perm[q];
        return s;
    };
    const int m = (int)cand.size();
    double combos = 1.0;
    for (int j = 0; j < g; ++j) combos = combos * (m - j) / (j + 1);
    uint64_t best_set = 0;
    Score best;
    if (combos <= 20000.0) {
        std::vector<int> idx(g);
        for (int j = 0; j < g; ++j) idx[j] = j;
        for (;;) {
            uint64_t set = 0;
            for (int j = 0; j < g; ++j) set |= 1ull << cand[idx[j]];
            const Score s = score(set);
            if (best < s) {
                best = s;
                best_set = set;
            }
            int j = g - 1;
            while (j >= 0 && idx[j] == m - g + j) --j;
            if (j < 0) break;
            ++idx[j];
            for (int k = j + 1; k < g; ++k) idx[k] = idx[k - 1] + 1;
        }
    } else {
        for (int j = 0; j < g; ++j) {
            uint64_t pick = 0;
            Score bj;
            for (int q : cand) {
                if ((best_set >> q) & 1ull) continue;
                const Score s = score(best_set | (1ull << q));
                if (bj < s) {
                    bj = s;
                    pick = 1ull << q;
                }
            }
            best_set |= pick;
        }
    }
    return best_set;
}

// Host plan of one run for one rank.  Gates are reordered only past gates on disjoint qubits
// (exact).  Each sweep in program order runs every gate whose target is local and whose earlier
// qubit-sharing gates have all run; when a sweep leaves gates, one remap brings in the targets
// (choose_globals) and the next sweep continues.  W-HC at 30 qubits on 8 ranks needs one remap
// per run this way (two in plain program order).
static std::vector<DStep> plan_dist_core(const qsim_gate* gates, size_t count, int n, int g, int rank,
                                         std::vector<int>& perm) {
    const int L = n - g;
    auto rank_bit = [&](int p) { return (rank >> (p - L)) & 1; };
    std::vector<DStep> steps;
    DStep cur;
    auto flush = [&]() {
        if (!cur.ops.empty() || !cur.gmask.empty()) steps.push_back(cur);
        cur = DStep();
    };
    for (size_t i = 0; i < count; ++i) validate_gate(gates[i], n);
    std::vector<uint64_t> qm(count);
    for (size_t i = 0; i < count; ++i) qm[i] = gate_qmask(gates[i]);
    auto emit = [&](size_t i) {
        const qsim_gate& gt = gates[i];
        if (gt.type == QSIM_GATE_SWAP) {  // relabel only
            std::swap(perm[gt.qubits[0]], perm[gt.qubits[1]]);
            return;
        }
        uint64_t pm = 0;  // physical positions the gate touches (rank-independent)
        for (int j = 0; j < gt.nqubits; ++j) pm |= 1ull << perm[gt.qubits[j]];
        cur.gmask.push_back(pm);
        qsim_gate pg = gt;
        for (int j = 0; j < gt.nqubits; ++j) pg.qubits[j] = perm[gt.qubits[j]];
        Op op = lower_gate(pg, n);
        op.src = (int)i;
        bool skip = false;
        for (int c = L; c < n; ++c)
            if ((op.cmask >> c) & 1ull) {
                if (!rank_bit(c)) skip = true;
                op.cmask &= ~(1ull << c);
            }
        if (skip) return;
        if (op.kind == K_DIAG && op.t0 >= L) {
            const int b = rank_bit(op.t0);
            if (!b && op.d0_one) return;  // factor 1 on this rank
            const double fr = b ? op.m[2] : op.m[0], fi = b ? op.m[3] : op.m[1];
            int t = 0;
            while (t < L - 1 && ((op.cmask >> t) & 1ull)) ++t;
            op.t0 = t;
            op.sub = S_GEN;
            op.d0_one = false;
            op.m[0] = op.m[2] = fr;
            op.m[1] = op.m[3] = fi;
        }
        if (op.t0 >= L || (op.kind == K_SWAP && op.t1 >= L))
            fail(QSIM_ERR_RUNTIME, "distributed planner left a global target");
        cur.ops.push_back(op);
        cur.op_gate.push_back((int)cur.gmask.size() - 1);
    };
    std::vector<char> done(count, 0);
    size_t left = count;
    for (;;) {
        uint64_t blocked = 0;
        for (size_t i = 0; i < count; ++i) {
            if (done[i]) continue;
            if (qm[i] & blocked) {
                blocked |= qm[i];
                continue;
            }
            const int tq = needs_local(gates[i]);
            if (tq >= 0 && perm[tq] >= L) {
                blocked |= qm[i];
                continue;
            }
            emit(i);
            done[i] = 1;
            --left;
        }
        if (left == 0) break;
        flush();
        const bool full = full_remap();
        const uint64_t want = choose_globals(gates, count, qm, done, perm, n, g, L, full);
        std::vector<int> out, in;
        for (int q = 0; q < n; ++q) {
            const bool w = (want >> q) & 1ull;
            if (perm[q] >= L && !w) out.push_back(q);
            if (perm[q] < L && w) in.push_back(q);
        }
        if (out.empty() || out.size() != in.size())
            fail(QSIM_ERR_RUNTIME, "distributed planner: no remap makes progress");
        DStep ex;
        ex.kind = 1;
        ex.k = (int)out.size();
        for (int j = 0; j < ex.k; ++j) {
            ex.gpos[j] = perm[out[j]];
            ex.lpos[j] = perm[in[j]];
            perm[out[j]] = ex.lpos[j];
            perm[in[j]] = ex.gpos[j];
        }
        steps.push_back(ex);
    }
    flush();
    // an exchange needs an ops step on both sides to overlap with (possibly empty)
    std::vector<DStep> framed;
    for (size_t i = 0; i < steps.size(); ++i) {
        if (steps[i].kind == 1 && (framed.empty() || framed.back().kind == 1)) framed.push_back(DStep());
        framed.push_back(std::move(steps[i]));
    }
    if (!framed.empty() && framed.back().kind == 1) framed.push_back(DStep());
    steps.swap(framed);
    return steps;
}

// Pivots chosen for a (gate list, start map, n, g): every shard of a virtual run, and every run
// that starts from the same map, reuses the decision instead of re-planning the candidates.
namespace {
struct PivotMemo {
    int n, g;
    uint64_t carry;
    std::vector<qsim_gate> gates;
    std::vector<int> perm;
    std::vector<uint64_t> pmask;   // per step (0: none)
    std::vector<uint64_t> coarse;  // per step
    uint64_t used;
};
std::mutex g_pivot_mu;
std::vector<PivotMemo> g_pivots;
uint64_t g_pivot_clock = 0;
}  // namespace

// ---- steady-state cycle pivots (the cross-run carry, QSIM_DIST_CARRY) ---------------------
// A benchmark or trajectory loop re-runs one circuit, and the runs' start maps soon cycle (the remap
// planner is deterministic; W-HC 30q on 8 ranks: two maps).  With the carry on, run j's last step B_j
// and run j+1's leading passes run per part of run j's exchange X_j, so X_j's pivots P_j shape TWO
// runs: run j (A_j's tail and B_j avoid P_j) and run j+1 (A_{j+1}'s head avoids P_j).  mark_overlap
// chooses P_j for run j alone (at most one pass of the next run credited), and on the alternate
// runs of seed 42 A's first pass then touches the carried pivots and runs whole and exposed.  Here
// the pivots of every exchange of the cycle are chosen together: coordinate descent over the
// cycle, each P_j by the beam search of mark_overlap on the cost T_j + T_{j+1} (the run-time model
// of mark_overlap with the carry: per-part passes of both neighbouring runs, whole passes exposed),
// every plan from rank 0's lowering (rank-independent), plans memoised by (step, avoid sets).
namespace {
struct CycleMemo {
    int n, g;
    std::vector<qsim_gate> gates;
    std::vector<std::vector<int>> maps;  // start map of each run of the cycle
    std::vector<uint64_t> piv;           // pivots of each run's exchange
    uint64_t used;
};
std::vector<CycleMemo> g_cycles;  // (under g_pivot_mu)
}  // namespace

// The pass touch masks of step `ops` planned with tail avoid set `pa` and head avoid set `pb`
// (all ones for a pass that never runs per part).
static std::vector<uint64_t> pass_masks(const std::vector<Op>& ops, int L, uint64_t pa, uint64_t pb) {
    const Plan pl = plan_fused(ops, L, -1, pa, pb);
    std::vector<uint64_t> m;
    for (const FusedPass& fp : pl.passes) {
        if (fp.single >= 0 || fp.h < 4) {
            m.push_back(~0ull);
            continue;
        }
        uint64_t t = 0;
        for (int i = 0; i < 6 + fp.h - fp.r0; ++i) t |= 1ull << fp.hpos[i];
        m.push_back(t);
    }
    return m;
}

// Per pass of the unconstrained plan of `ops`: the positions its gates act on (targets and
// controls; padding excluded — a tile may be padded elsewhere), all ones for a per-gate pass.
static std::vector<uint64_t> pass_forced(const std::vector<Op>& ops, int L) {
    const Plan pl = plan_fused(ops, L);
    std::vector<uint64_t> m;
    for (const FusedPass& fp : pl.passes) {
        if (fp.single >= 0 || fp.h < 4) {
            m.push_back(~0ull);
            continue;
        }
        int b = fp.op_begin, e = fp.op_end;
        if (fp.stage_end > fp.stage_begin) {
            b = pl.stages[fp.stage_begin].op_begin;
            e = pl.stages[fp.stage_end - 1].op_end;
        }
        uint64_t f = 0;
        for (int i = b; i < e; ++i) {
            const Op& o = ops[pl.order[i]];
            f |= (1ull << o.t0) | o.cmask;
            if (o.t1 >= 0) f |= 1ull << o.t1;
        }
        m.push_back(f);
    }
    return m;
}

static bool cycle_pivots(const qsim_gate* gates, size_t count, int n, int g, const std::vector<int>& perm_in,
                         uint64_t* piv_out) {
    const int L = n - g;
    auto same_gates = [&](const CycleMemo& m) {
        return m.n == n && m.g == g && m.gates.size() == count &&
               (count == 0 || std::memcmp(m.gates.data(), gates, count * sizeof(qsim_gate)) == 0);
    };
    {
        std::lock_guard<std::mutex> l(g_pivot_mu);
        for (CycleMemo& m : g_cycles)
            if (same_gates(m))
                for (size_t j = 0; j < m.maps.size(); ++j)
                    if (m.maps[j] == perm_in) {
                        m.used = ++g_pivot_clock;
                        *piv_out = m.piv[j];
                        return true;
                    }
    }
    // the runs from perm_in (rank 0's lowering), until a start map repeats
    std::vector<std::vector<int>> maps;
    std::vector<std::vector<DStep>> runs;
    std::vector<int> p = perm_in;
    int cyc = -1;
    for (int r = 0; r < 8 && cyc < 0; ++r) {
        maps.push_back(p);
        runs.push_back(plan_dist_core(gates, count, n, g, 0, p));
        for (size_t j = 0; j < maps.size(); ++j)
            if (maps[j] == p) cyc = (int)j;
    }
    if (cyc != 0) return false;  // (perm_in is a transient map, or no cycle within 8 runs)
    const int C = (int)runs.size();
    for (const std::vector<DStep>& st : runs)
        if (st.size() != 3 || st[0].kind != 0 || st[1].kind != 1 || st[2].kind != 0 || st[0].ops.empty() ||
            st[2].ops.empty())
            return false;  // (one remap per run between two ops steps: the case the model prices)
    static const double r_scale = [] {  // (mark_overlap's QSIM_DIST_MODEL_R)
        const char* e = std::getenv("QSIM_DIST_MODEL_R");
        return e ? std::atof(e) : 50.0;
    }();
    // a pass run per part (sub-space launches) costs rP whole-shard passes (virtual 30q / 8:
    // 5.15 vs 6.4 TB/s, profiles/r04/dist_virtual/)
    static const double rP = [] {
        const char* e = std::getenv("QSIM_DIST_MODEL_PART");
        return e ? std::atof(e) : 1.243;
    }();
    const double R = r_scale / std::max(2, 1 << g);
    std::mutex mu;
    std::map<std::tuple<int, int, uint64_t, uint64_t>, std::vector<uint64_t>> cache;
    auto masks = [&](int j, int which, uint64_t pa, uint64_t pb) {
        const auto key = std::make_tuple(j, which, pa, pb);
        {
            std::lock_guard<std::mutex> l(mu);
            auto it = cache.find(key);
            if (it != cache.end()) return it->second;
        }
        std::vector<uint64_t> m = pass_masks(runs[j][which].ops, L, pa, pb);
        std::lock_guard<std::mutex> l(mu);
        cache.emplace(key, m);
        return m;
    };
    // B_j's (passes, leading passes avoiding P_j, parts)
    struct BInfo {
        int nb, h;
        double K;
    };
    auto binfo = [&](int j, uint64_t P) {
        const std::vector<uint64_t> mb = masks(j, 2, 0, P);
        int h = 0;
        if (P)
            while (h < (int)mb.size() && !(mb[h] & P)) ++h;
        return BInfo{(int)mb.size(), h, (double)(1 << __builtin_popcountll(P))};
    };
    // T of a run from its A's pass masks, the previous run's B info, carried pivots Pp, own P
    auto t_of = [&](const std::vector<uint64_t>& ma, const BInfo& bp, uint64_t Pp, uint64_t P) {
        const int na = (int)ma.size();
        int hA = 0, t = 0;
        if (Pp)
            while (hA < na && !(ma[hA] & Pp)) ++hA;
        if (P)
            while (t < na - hA && !(ma[na - 1 - t] & P)) ++t;
        int c = 0;
        uint64_t cb = 0;
        if (P && coarse_enabled()) {  // (coarse_split on the masks)
            double best = (double)(na - t - hA);
            uint64_t U = 0;
            for (int cc = 1; cc <= na - t - hA; ++cc) {
                U |= ma[na - t - cc] & P;
                const uint64_t b = P & ~U;
                if (!b) break;
                const double e = (double)(na - t - hA - cc) + (double)cc / (double)(1 << __builtin_popcountll(b));
                if (e < best - 1e-9) {
                    best = e;
                    c = cc;
                    cb = b;
                }
            }
        }
        const double K = (double)(1 << __builtin_popcountll(P)), Kc = (double)(1 << __builtin_popcountll(cb));
        const int whole = (na - hA - t - c) + (bp.nb - bp.h);
        const double exposed = (bp.h + hA) * rP / bp.K + (na - hA - t - c) + c * rP / Kc + t * rP / K + (bp.nb - bp.h);
        return std::max(R + exposed, whole + (hA + t + c + bp.h) * rP + R / K);
    };
    // T_j: run j with carried pivots Pp (of X_{j-1}) and its own P, from the plans under those sets
    auto tj = [&](int j, uint64_t Pp, uint64_t P) {
        const int jp = (j + C - 1) % C;
        return t_of(masks(j, 0, P, Pp), binfo(jp, Pp), Pp, P);
    };
    std::vector<uint64_t> P(C, 0);
    auto cost_j = [&](int j, uint64_t Pj) {  // the terms P_j enters
        std::vector<uint64_t> Q = P;
        Q[j] = Pj;
        const int jn = (j + 1) % C;
        if (jn == j) return tj(j, Pj, Pj);
        return tj(j, Q[(j + C - 1) % C], Pj) + tj(jn, Pj, Q[jn]);
    };
    auto optimise = [&](int j) {
        uint64_t lmask = 0;
        for (int i = 0; i < runs[j][1].k; ++i) lmask |= 1ull << runs[j][1].lpos[i];
        std::vector<int> cand;
        for (int q = 6; q < L; ++q)
            if (!((lmask >> q) & 1ull)) cand.push_back(q);
        auto score = [&](const std::vector<uint64_t>& sets) {
            std::vector<double> sc(sets.size(), 1e30);
            std::vector<std::thread> th;
            const size_t nt = std::min<size_t>(sets.size(), 16);
            for (size_t w = 0; w < nt; ++w)
                th.emplace_back([&, w] {
                    for (size_t c = w; c < sets.size(); c += nt) try {
                            sc[c] = cost_j(j, sets[c]);
                        } catch (...) {
                        }
                });
            for (auto& t : th) t.join();
            return sc;
        };
        std::vector<uint64_t> singles;
        for (int q : cand) singles.push_back(1ull << q);
        std::vector<double> s1 = score(singles);
        double bestT = cost_j(j, 0);
        uint64_t best = 0;
        std::vector<size_t> o(singles.size());
        for (size_t c = 0; c < o.size(); ++c) o[c] = c;
        std::sort(o.begin(), o.end(), [&](size_t a, size_t b) { return s1[a] != s1[b] ? s1[a] < s1[b] : a < b; });
        constexpr size_t kBeam = 4, kPool = 10;
        std::vector<int> pool;
        std::vector<uint64_t> beam;
        for (size_t c = 0; c < o.size() && pool.size() < kPool; ++c)
            if (s1[o[c]] < 1e29) {
                pool.push_back(cand[o[c]]);
                if (beam.size() < kBeam) beam.push_back(singles[o[c]]);
                if (s1[o[c]] < bestT - 1e-9) {
                    bestT = s1[o[c]];
                    best = singles[o[c]];
                }
            }
        // (the current choice competes too: a sweep never makes P_j worse)
        if (P[j]) {
            const double cur = cost_j(j, P[j]);
            if (cur < bestT - 1e-9) {
                bestT = cur;
                best = P[j];
            }
        }
        for (int m = 1; m < kMaxPivots && !beam.empty(); ++m) {
            std::vector<uint64_t> sets;
            for (uint64_t b : beam)
                for (int q : pool) {
                    const uint64_t s2 = b | (1ull << q);
                    if (s2 != b && std::find(sets.begin(), sets.end(), s2) == sets.end()) sets.push_back(s2);
                }
            std::vector<double> sc = score(sets);
            std::vector<size_t> o2(sets.size());
            for (size_t c = 0; c < o2.size(); ++c) o2[c] = c;
            std::sort(o2.begin(), o2.end(),
                      [&](size_t a, size_t b) { return sc[a] != sc[b] ? sc[a] < sc[b] : sets[a] < sets[b]; });
            beam.clear();
            for (size_t c = 0; c < o2.size() && beam.size() < kBeam; ++c)
                if (sc[o2[c]] < 1e29) beam.push_back(sets[o2[c]]);
            if (!o2.empty() && sc[o2[0]] < bestT - 1e-9) {
                bestT = sc[o2[0]];
                best = sets[o2[0]];
            }
        }
        P[j] = best;
    };
    // Constructive start: every split of each run's A into a head (avoids the carried pivots) and a
    // tail (avoids its own), the passes between them whole or coarse.  Under fixed splits P_j may
    // take any position outside the exchanged ones, B_j's passes, A_j's tail and A_{j+1}'s head
    // (masks of the unconstrained plans); the up-to-4 such positions used by the fewest passes of
    // the cycle form P_j.  Splits are ranked by the model on the unconstrained masks, the best few
    // re-priced on the plans under their sets, and the best becomes the descent's start.
    // (QSIM_DIST_CYCLE_CONSTRUCT=1, measured not kept: W-HC 30q / 8, the carry model over seeds
    // 42 / 1-3 gives 4.03 / 3.98 / 4.11 / 3.97x with it against 4.18 / 4.00 / 4.11 / 4.22x from the
    // descent alone — W-HC tiles are dense, a split's free positions number one or two, and the
    // plans re-padded under the chosen sets lose the split anyway)
    static const bool construct = [] {
        const char* e = std::getenv("QSIM_DIST_CYCLE_CONSTRUCT");
        return e != nullptr && std::atoi(e) != 0;
    }();
    if (C <= 3 && construct) {
        std::vector<std::vector<uint64_t>> mA(C), mB(C);
        std::vector<int> use(64, 0);
        for (int j = 0; j < C; ++j) {
            mA[j] = pass_forced(runs[j][0].ops, L);
            mB[j] = pass_forced(runs[j][2].ops, L);
            for (const auto* v : {&mA[j], &mB[j]})
                for (uint64_t x : *v)
                    for (int q = 0; q < L; ++q) use[q] += (int)((x >> q) & 1ull);
        }
        uint64_t all = 0;
        for (int q = 6; q < L; ++q) all |= 1ull << q;
        std::vector<std::vector<std::pair<int, int>>> splits(C);
        for (int j = 0; j < C; ++j)
            for (int h = 0; h <= std::min(1, (int)mA[j].size()); ++h)  // (the planner steers the first pass only)
                for (int t = 0; h + t <= (int)mA[j].size(); ++t) splits[j].push_back({h, t});
        struct Combo {
            double pred;
            std::vector<uint64_t> P;
        };
        std::vector<Combo> combos;
        std::vector<size_t> idx(C, 0);
        for (;;) {
            std::vector<uint64_t> Q(C, 0);
            for (int j = 0; j < C; ++j) {
                const int jn = (j + 1) % C;
                const int t = splits[j][idx[j]].second, hn = splits[jn][idx[jn]].first;
                uint64_t forbid = 0;
                for (int i = 0; i < runs[j][1].k; ++i) forbid |= 1ull << runs[j][1].lpos[i];
                for (uint64_t x : mB[j]) forbid |= x;
                for (int i = 0; i < t; ++i) forbid |= mA[j][mA[j].size() - 1 - i];
                for (int i = 0; i < hn; ++i) forbid |= mA[jn][i];
                std::vector<int> ok;
                for (int q = 6; q < L; ++q)
                    if (((all & ~forbid) >> q) & 1ull) ok.push_back(q);
                std::stable_sort(ok.begin(), ok.end(), [&](int a, int b) { return use[a] < use[b]; });
                for (size_t i = 0; i < ok.size() && i < (size_t)kMaxPivots; ++i) Q[j] |= 1ull << ok[i];
            }
            double pred = 0.0;
            for (int j = 0; j < C; ++j) {
                const int jp = (j + C - 1) % C;
                int hb = 0;
                if (Q[jp])
                    while (hb < (int)mB[jp].size() && !(mB[jp][hb] & Q[jp])) ++hb;
                pred += t_of(mA[j], BInfo{(int)mB[jp].size(), hb, (double)(1 << __builtin_popcountll(Q[jp]))},
                             Q[jp], Q[j]);
            }
            combos.push_back({pred, Q});
            int j = 0;
            while (j < C && ++idx[j] == splits[j].size()) idx[j++] = 0;
            if (j == C) break;
        }
        std::sort(combos.begin(), combos.end(), [](const Combo& a, const Combo& b) {
            return a.pred != b.pred ? a.pred < b.pred : a.P < b.P;
        });
        std::vector<std::vector<uint64_t>> tops;
        for (const Combo& cb : combos) {
            if (tops.size() >= 12) break;
            if (std::find(tops.begin(), tops.end(), cb.P) == tops.end()) tops.push_back(cb.P);
        }
        std::vector<double> sc(tops.size(), 1e30);
        {
            std::vector<std::thread> th;
            for (size_t c = 0; c < tops.size(); ++c)
                th.emplace_back([&, c] {
                    try {
                        double tot = 0.0;
                        for (int j = 0; j < C; ++j) tot += tj(j, tops[c][(j + C - 1) % C], tops[c][j]);
                        sc[c] = tot;
                    } catch (...) {
                    }
                });
            for (auto& t : th) t.join();
        }
        size_t bi = 0;
        for (size_t c = 1; c < tops.size(); ++c)
            if (sc[c] < sc[bi] - 1e-9) bi = c;
        if (std::getenv("QSIM_DIST_DEBUG_CYCLE"))
            for (size_t c = 0; c < tops.size(); ++c) {
                double pr = 0;
                for (const Combo& cb : combos)
                    if (cb.P == tops[c]) {
                        pr = cb.pred;
                        break;
                    }
                std::fprintf(stderr, "[cycle] combo %zu pred %.3f real %.3f:", c, pr, sc[c]);
                for (uint64_t x : tops[c]) std::fprintf(stderr, " %#llx", (unsigned long long)x);
                for (int j = 0; j < C; ++j) {
                    std::fprintf(stderr, " | A%d", j);
                    for (uint64_t x : masks(j, 0, tops[c][j], tops[c][(j + C - 1) % C]))
                        std::fprintf(stderr, " %#llx", (unsigned long long)x);
                    std::fprintf(stderr, " B%d", j);
                    for (uint64_t x : masks(j, 2, 0, tops[c][j])) std::fprintf(stderr, " %#llx", (unsigned long long)x);
                }
                std::fprintf(stderr, "\n");
            }
        if (!tops.empty() && sc[bi] < 1e29) P = tops[bi];
    }
    static const int sweeps = [] {
        const char* e = std::getenv("QSIM_DIST_CYCLE_SWEEPS");
        return e ? std::max(0, std::atoi(e)) : 2;
    }();
    for (int sw = 0; sw < sweeps; ++sw)
        for (int j = 0; j < C; ++j) optimise(j);
    static const bool dbg = std::getenv("QSIM_DIST_DEBUG_CYCLE") != nullptr;
    if (dbg) {
        double tot = 0.0;
        for (int j = 0; j < C; ++j) tot += tj(j, P[(j + C - 1) % C], P[j]);
        std::fprintf(stderr, "[cycle] %d runs, model %.3f passes per run, pivots", C, tot / C);
        for (uint64_t x : P) std::fprintf(stderr, " %#llx", (unsigned long long)x);
        std::fprintf(stderr, "\n");
        for (int j = 0; j < C; ++j) {
            const uint64_t Pp = P[(j + C - 1) % C];
            std::fprintf(stderr, "[cycle] run %d T %.3f | A (head %#llx, tail %#llx):", j, tj(j, Pp, P[j]),
                         (unsigned long long)Pp, (unsigned long long)P[j]);
            for (uint64_t x : masks(j, 0, P[j], Pp)) std::fprintf(stderr, " %#llx", (unsigned long long)x);
            std::fprintf(stderr, " | A free:");
            for (uint64_t x : masks(j, 0, 0, 0)) std::fprintf(stderr, " %#llx", (unsigned long long)x);
            std::fprintf(stderr, " | B:");
            for (uint64_t x : masks(j, 2, 0, P[j])) std::fprintf(stderr, " %#llx", (unsigned long long)x);
            std::fprintf(stderr, " | X lpos");
            for (int i = 0; i < runs[j][1].k; ++i) std::fprintf(stderr, " %d", runs[j][1].lpos[i]);
            std::fprintf(stderr, "\n");
        }
    }
    *piv_out = P[0];
    std::lock_guard<std::mutex> l(g_pivot_mu);
    CycleMemo m{n, g, std::vector<qsim_gate>(gates, gates + count), maps, P, ++g_pivot_clock};
    if (g_cycles.size() >= 8)
        g_cycles.erase(std::min_element(g_cycles.begin(), g_cycles.end(),
                                        [](const CycleMemo& a, const CycleMemo& b) { return a.used < b.used; }));
    g_cycles.push_back(std::move(m));
    return true;
}

static std::vector<DStep> plan_dist(const qsim_gate* gates, size_t count, int n, int g, int rank,
                                    std::vector<int>& perm, uint64_t carry = 0) {
    const std::vector<int> perm_in = perm;
    std::vector<DStep> steps = plan_dist_core(gates, count, n, g, rank, perm);
    const int L = n - g;
    static const int overlap = [] {
        const char* e = std::getenv("QSIM_DIST_OVERLAP");
        return e ? std::atoi(e) : 1;
    }();
    if (!overlap || L < 8 || steps.empty() || steps[0].kind != 0) carry = 0;
    auto same = [&](const PivotMemo& m) {
        return m.n == n && m.g == g && m.carry == carry && m.perm == perm_in && m.gates.size() == count &&
               (count == 0 || std::memcmp(m.gates.data(), gates, count * sizeof(qsim_gate)) == 0);
    };
    {
        std::lock_guard<std::mutex> l(g_pivot_mu);
        for (PivotMemo& m : g_pivots)
            if (same(m) && m.pmask.size() == steps.size()) {
                m.used = ++g_pivot_clock;
                if (carry) steps[0].role |= 2;
                for (size_t k = 0; k < steps.size(); ++k)
                    if (m.pmask[k]) {
                        steps[k].pmask = m.pmask[k];
                        steps[k].coarse = m.coarse[k];
                        steps[k].pivot = __builtin_ctzll(m.pmask[k]);
                        steps[k - 1].role |= 1;
                        steps[k + 1].role |= 2;
                    }
                return steps;
            }
    }
    // carry on and the start map on a cycle of one-remap runs: the cycle's jointly chosen pivots
    uint64_t cyc_piv = 0;
    if (carry_enabled() && overlap && L >= 8 && steps.size() == 3 && steps[0].kind == 0 && steps[1].kind == 1 &&
        steps[2].kind == 0 && cycle_pivots(gates, count, n, g, perm_in, &cyc_piv) && cyc_piv) {
        DStep& A = steps[0];
        DStep& ex = steps[1];
        ex.pmask = cyc_piv;
        ex.pivot = __builtin_ctzll(cyc_piv);
        A.role |= 1;
        steps[2].role |= 2;
        if (carry) A.role |= 2;
        // coarse bits for this run's actual carry, on rank 0's lowering (rank-independent)
        ex.coarse = 0;
        if (coarse_enabled()) {
            std::vector<int> p0 = perm_in;
            const std::vector<DStep> ref = plan_dist_core(gates, count, n, g, 0, p0);
            if (ref.size() == 3 && !ref[0].ops.empty()) {
                const Plan pA = plan_fused(ref[0].ops, L, -1, cyc_piv, carry);
                const int na = (int)pA.passes.size();
                int ha = 0, t = 0;
                if (carry)
                    while (ha < na && pass_avoids(pA.passes[ha], carry)) ++ha;
                while (t < na - ha && pass_avoids(pA.passes[na - 1 - t], cyc_piv)) ++t;
                (void)coarse_split(pA, ha, na - t, cyc_piv, &ex.coarse);
            }
        }
        PivotMemo m{n, g, carry, std::vector<qsim_gate>(gates, gates + count), perm_in, {}, {}, 0};
        for (const DStep& st : steps) {
            m.pmask.push_back(st.kind == 1 ? st.pmask : 0ull);
            m.coarse.push_back(st.kind == 1 ? st.coarse : 0ull);
        }
        std::lock_guard<std::mutex> l(g_pivot_mu);
        m.used = ++g_pivot_clock;
        if (g_pivots.size() >= 16)
            g_pivots.erase(std::min_element(g_pivots.begin(), g_pivots.end(),
                                            [](const PivotMemo& a, const PivotMemo& b) { return a.used < b.used; }));
        g_pivots.push_back(std::move(m));
        return steps;
    }
    // the next run's first ops step (rank 0's lowering, from this run's end map: the same on every
    // rank), for scoring the last remap's pivots by the passes it can carry
    std::vector<Op> next_ops;
    if (carry_enabled() && overlap && L >= 8) {
        std::vector<int> pn = perm;
        const std::vector<DStep> nxt = plan_dist_core(gates, count, n, g, 0, pn);
        if (!nxt.empty() && nxt[0].kind == 0) next_ops = nxt[0].ops;
    }
    if (rank == 0) {
        mark_overlap(steps, L, 1 << g, steps, carry, &next_ops);
    } else {
        std::vector<int> p0 = perm_in;
        const std::vector<DStep> ref = plan_dist_core(gates, count, n, g, 0, p0);
        if (ref.size() != steps.size()) fail(QSIM_ERR_RUNTIME, "exchange skeleton mismatch");
        mark_overlap(steps, L, 1 << g, ref, carry, &next_ops);
    }
    PivotMemo m{n, g, carry, std::vector<qsim_gate>(gates, gates + count), perm_in, {}, {}, 0};
    for (const DStep& st : steps) {
        m.pmask.push_back(st.kind == 1 ? st.pmask : 0ull);
        m.coarse.push_back(st.kind == 1 ? st.coarse : 0ull);
    }
    std::lock_guard<std::mutex> l(g_pivot_mu);
    m.used = ++g_pivot_clock;
    if (g_pivots.size() >= 16)
        g_pivots.erase(std::min_element(g_pivots.begin(), g_pivots.end(),
                                        [](const PivotMemo& a, const PivotMemo& b) { return a.used < b.used; }));
    g_pivots.push_back(std::move(m));
    return steps;
}

// ---- exchange kernels ---------------------------------------------------------------------
struct XArgs {
    double2* st;
    double2* buf;
    uint64_t chunk;     // 2^(L-k) amplitudes
    int chunk_log;
    int k;
    int my_c;
    int nsorted;        // zero-insertion positions: lpos, plus the pivots of a part exchange
    int sorted[12];     // ascending
    int lpos[8];        // chunk bit j <-> lpos[j]
    uint64_t orval;     // part exchange: the pivot bits' values
};

// Local amplitude index of element e of the slab buffer (slab c = e >> chunk_log): the offset's
// bits are spread around the zero-inserted positions, then slab bits go to lpos and the part's
// pivot values are or-ed in.  Host and device: qsim_dist_slab_map exports the same map.
__host__ __device__ __forceinline__ uint64_t xlocal(const XArgs& a, uint64_t e) {
    const uint64_t c = e >> a.chunk_log;
    uint64_t off = e & (a.chunk - 1);
#pragma unroll
    for (int j = 0; j < 12; ++j)
        if (j < a.nsorted) {
            const uint64_t lo = off & ((1ull << a.sorted[j]) - 1ull);
            off = ((off ^ lo) << 1) | lo;
        }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < a.k) off |= ((c >> j) & 1ull) << a.lpos[j];
    return off | a.orval;
}

// Pack (state -> send slabs) or unpack (receive slabs -> state) the offsets [lo, lo + 2^sub_log)
// of every slab (one pipeline part of a remap); the own slab never moves.
template <bool PACK>
__global__ __launch_bounds__(256) void k_exchange_copy(XArgs a, uint64_t lo, int sub_log) {
    const uint64_t total = (uint64_t)1 << (sub_log + a.k);
    const uint64_t sub_mask = ((uint64_t)1 << sub_log) - 1;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += step) {
        const uint64_t c = x >> sub_log;
        if ((int)c == a.my_c) continue;
        const uint64_t e = (c << a.chunk_log) | (lo + (x & sub_mask));
        const uint64_t i = xlocal(a, e);
        if (PACK) a.buf[e] = a.st[i];
        else a.st[i] = a.buf[e];
    }
}

}  // namespace qsim_hip

// ncclInProgress is the normal return of a non-blocking communicator (the call is queued; the
// communicator settles before the next use, comm_settle below).
#define QSIM_NCCLCHK(call)                                                              \
    do {                                                                                \
        ncclResult_t r_ = (call);                                                       \
        if (r_ != ncclSuccess && r_ != ncclInProgress)                                  \
            fail(QSIM_ERR_DEVICE, std::string("RCCL error: ") + ncclGetErrorString(r_)); \
    } while (0)

// A prepared ops step (see prepare_step): its plan, kernels and the pass ranges around pivots.
struct StepRun {
    const Plan* plan = nullptr;
    const JitModule* jm = nullptr;
    size_t j1 = 0, j2 = 0, np = 0;
};

// One rank's share: its amplitudes and the exchange staging buffers.
struct Shard {
    int rank = 0;
    double2* d = nullptr;
    double2* sendbuf = nullptr;
    double2* recvbuf = nullptr;
};

// Every mode runs the same per-shard code (planning per rank, pack / unpack, the slab posts of
// one remap part); only the transport that carries the posts differs:
//   T_RCCL    one shard per process, grouped ncclSend / ncclRecv over xGMI (production);
//   T_VIRTUAL all W shards in this process on one GPU (qsim_dist_create_virtual): the posts of
//             the W shards are paired by RCCL's matching rule and moved by device copies, or by
//             ncclSend / ncclRecv to rank 0 of a world-1 communicator (qsim_dist_virtual_rccl);
//   T_HOSTED  one shard per process, the posts staged through host memory and handed to a
//             caller-supplied function (qsim_dist_create_hosted: multi-process runs without RCCL,
//             e.g. several ranks on one GPU in tests).
struct qsim_dist {
    enum Transport { T_RCCL = 0, T_VIRTUAL = 1, T_HOSTED = 2 };
    int n = 0, g = 0, L = 0, world = 1, device = 0;
    bool virt = false;
    Transport transport = T_RCCL;
    qsim_dist_transport_fn host_fn = nullptr;
    void* host_ctx = nullptr;
    char* h_stage = nullptr;  // hosted: pinned staging (send half, receive half), grow-only
    size_t h_stage_bytes = 0;
    std::vector<Shard> shards;
    double* d_partials = nullptr;
    double* d_result = nullptr;
    hipStream_t stream = nullptr;       // compute: passes, pack / unpack
    hipStream_t comm_stream = nullptr;  // remap transfers (RCCL or, virtual, device copies)
    hipStream_t copy_stream = nullptr;  // pack / unpack of overlapped (half) remaps
    std::vector<hipEvent_t> events;     // remap pipeline: packed part p, transferred part p
    // overlapped remap, per part h < kMaxParts: tail done (pev[h]), packed (kMaxParts + h), sent
    // (2 kMaxParts + h), unpacked (3 kMaxParts + h)
    hipEvent_t pev[4 * kMaxParts] = {};
    int order[kMaxParts] = {};  // exchange order of the pending overlapped remap's parts (part_order)
    int overlapped = 0;                 // remaps of the last run that overlapped local work
    ncclComm_t comm = nullptr;
    bool aborted = false;  // the communicator was aborted after an RCCL / HIP error or a timeout
    bool fresh = true;     // |0..0> with the identity map (create / reset): local labels are free
    std::vector<int> perm;
    DevBuf ops, stages;
    // Plans of recent runs, keyed by (gate list, map at the start of the run): a repeated circuit
    // alternates between a few start maps, each with its own segment plans and compiled kernels.
    // Fused remap (QSIM_DIST_FUSED_PACK, default on): the last pass before an exchange stores
    // its tiles straight into the send buffer's slab layout and the step after it plans in that
    // layout, loading from the receive buffer, its last pass storing back to the standard one —
    // no pack / unpack kernels.  Per shard: the two plans, their compiled kernels, the decision.
    struct FusedVariant {
        Plan plan;
        JitState jit;
        bool ok = false;
    };
    struct RunPlan {
        std::vector<qsim_gate> gates;
        std::vector<int> perm_in, perm_out;
        uint64_t carry_in = 0;  // pivots of the previous run's exchange still in flight at the start
        bool in_use = false;    // a deferred step of this plan is pending (never evicted then)
        std::vector<std::vector<DStep>> steps;              // per shard
        std::vector<std::vector<std::unique_ptr<PlanCache>>> fplans;  // per shard, per step
        std::vector<std::unique_ptr<FusedVariant>> fpack, funpack;    // per shard (the first exchange)
        bool fused_decided = false;
        uint64_t used = 0;
    };
    int fused_remaps = 0;  // exchanges of the last run whose pack / unpack ran inside the passes
    // Cross-run overlap: a run whose last step is the per-part head of an overlapped remap (every
    // pass of it avoids the pivots) leaves that step pending; the next run of a circuit runs its
    // first step's leading passes per part too, interleaved with it (part h of both as soon as
    // part h has landed), so the remap also hides the next run's first passes.  Anything else
    // that touches the state runs it first (flush_carry).
    struct Carry {
        bool active = false;
        uint64_t pmask = 0;  // the remap's pivots (the run's standard positions)
        int parts = 0;
        RunPlan* rp = nullptr;
        size_t step = 0;
        std::vector<StepRun> runs;
        std::vector<uint64_t> pbs;
        std::vector<double2*> homes, alts;
    } carry;
    int carried = 0;  // runs of this object whose first step merged a carried step
    std::vector<std::unique_ptr<RunPlan>> run_plans;
    uint64_t run_clock = 0;
    Timer timer;
    ~qsim_dist() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (comm) {  // flush, bounded wait (non-blocking comm), then destroy; abort on trouble
            bool ok = ncclCommFinalize(comm) == ncclSuccess;
            if (!ok) {
                ncclResult_t st = ncclInProgress;
                const auto t0 = std::chrono::steady_clock::now();
                while (ncclCommGetAsyncError(comm, &st) == ncclSuccess && st == ncclInProgress &&
                       std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60))
                    std::this_thread::yield();
                ok = st == ncclSuccess;
            }
            if (ok) (void)ncclCommDestroy(comm);
            else (void)ncclCommAbort(comm);
        }
        for (Shard& s : shards)
            for (void* p : {(void*)s.d, (void*)s.sendbuf, (void*)s.recvbuf})
                if (p) (void)hipFree(p);
        if (d_partials) (void)hipFree(d_partials);
        if (d_result) (void)hipFree(d_result);
        if (comm_stream) (void)hipStreamSynchronize(comm_stream);
        for (hipEvent_t e : events)
            if (e) (void)hipEventDestroy(e);
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        for (hipEvent_t e : pev)
            if (e) (void)hipEventDestroy(e);
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        if (comm_stream) (void)hipStreamDestroy(comm_stream);
        if (stream) (void)hipStreamDestroy(stream);
        if (h_stage) (void)hipHostFree(h_stage);
    }
    // this rank's remap traffic in the last run (bytes sent; the same are received)
    double sent_bytes = 0.0;
};

namespace {
template <typename F>
int dguard(F&& f) {
    try {
        f();
        return QSIM_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return QSIM_ERR_RUNTIME;
    }
}
void need(const qsim_dist* d) {
    if (!d) fail(QSIM_ERR_INVALID_ARGUMENT, "null dist handle");
    if (d->aborted)
        fail(QSIM_ERR_DEVICE, "distributed state unusable: its RCCL communicator was aborted "
                              "after an earlier error");
}
// Entry points that touch the communicator: any RCCL / HIP failure (or a timeout) aborts it, so
// peers blocked in a collective with this rank are released instead of hanging.
template <typename F>
int dguard_comm(qsim_dist* d, F&& f) {
    const int rc = dguard(std::forward<F>(f));
    if (rc == QSIM_ERR_DEVICE && d && d->comm && !d->aborted) {
        (void)ncclCommAbort(d->comm);
        d->comm = nullptr;
        d->aborted = true;
    }
    return rc;
}
double env_seconds(const char* k, double dflt) {
    const char* e = std::getenv(k);
    const double v = e ? std::atof(e) : dflt;
    return v > 0 ? v : dflt;
}
// Wait until a non-blocking communicator has finished queuing its last call (init, group end,
// collective); a communicator error or QSIM_DIST_TIMEOUT seconds without progress fails (the
// caller's dguard_comm then aborts the communicator).
void comm_settle(ncclComm_t comm, const char* what, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        QSIM_NCCLCHK(ncclCommGetAsyncError(comm, &st));
        if (st == ncclSuccess) return;
        if (st != ncclInProgress)
            fail(QSIM_ERR_DEVICE, std::string("RCCL error during ") + what + ": " + ncclGetErrorString(st));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            fail(QSIM_ERR_DEVICE, std::string("RCCL timeout during ") + what);
        std::this_thread::yield();
    }
}
void comm_settle(qsim_dist* d, const char* what) {
    if (d->comm) comm_settle(d->comm, what, env_seconds("QSIM_DIST_TIMEOUT", 600.0));
}
// hipStreamSynchronize with a watchdog: while the stream drains, a communicator error or
// QSIM_DIST_TIMEOUT seconds fail (and abort the communicator) instead of blocking forever.
void stream_wait(qsim_dist* d, hipStream_t s) {
    if (!d->comm) {
        QSIM_HIPCHK(hipStreamSynchronize(s));
        return;
    }
    const double timeout_s = env_seconds("QSIM_DIST_TIMEOUT", 600.0);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) QSIM_HIPCHK(q);
        ncclResult_t st = ncclSuccess;
        QSIM_NCCLCHK(ncclCommGetAsyncError(d->comm, &st));
        if (st != ncclSuccess && st != ncclInProgress)
            fail(QSIM_ERR_DEVICE, std::string("RCCL error while waiting: ") + ncclGetErrorString(st));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            fail(QSIM_ERR_DEVICE, "timeout waiting for the distributed state's streams");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
int log2_exact(int w) {
    if (w < 1) fail(QSIM_ERR_INVALID_ARGUMENT, "world size must be positive");
    int g = 0;
    while ((1 << g) < w) ++g;
    if ((1 << g) != w) fail(QSIM_ERR_INVALID_ARGUMENT, "world size must be a power of two");
    return g;
}
void check_sizes(int n, int g) {
    if (n < QSIM_MIN_QUBITS || n > QSIM_MAX_QUBITS_DIST)
        fail(QSIM_ERR_INVALID_ARGUMENT, "Number of qubits out of range");
    if (n - g < std::max(1, g))
        fail(QSIM_ERR_INVALID_ARGUMENT, "too few qubits per rank for this world size");
}
void alloc_shards(qsim_dist* d, const std::vector<int>& ranks) {
    const size_t bytes = sizeof(double2) << d->L;
    for (int r : ranks) {
        Shard s;
        s.rank = r;
        QSIM_HIPCHK(hipMalloc((void**)&s.d, bytes));
        if (d->world > 1) {
            QSIM_HIPCHK(hipMalloc((void**)&s.sendbuf, bytes));
            QSIM_HIPCHK(hipMalloc((void**)&s.recvbuf, bytes));
        }
        d->shards.push_back(s);
    }
    QSIM_HIPCHK(hipMalloc((void**)&d->d_partials, 4096 * sizeof(double)));
    QSIM_HIPCHK(hipMalloc((void**)&d->d_result, sizeof(double)));
}
void init_zero(qsim_dist* d) {
    for (int q = 0; q < d->n; ++q) d->perm[q] = q;
    d->fresh = true;
    for (Shard& s : d->shards) launch_init_basis(s.d, d->L, 1, s.rank == 0 ? 0 : ~0ull, d->stream);
    QSIM_HIPCHK(hipStreamSynchronize(d->stream));
}

// The slab layout of one remap (or one part of an overlapped remap) on one rank: the pack /
// unpack map (XArgs) and the rank each slab goes to and comes from.  Host-only and rank-local;
// qsim_dist_slab_map exports it for the CPU tests.
struct XPlan {
    XArgs a;
    int peer_of[256];
};
// part < 0: the whole shard; part j: the amplitudes whose pivot bits hold the bits of j.
XPlan xplan(int L, int rank, const DStep& ex, int part = -1) {
    XPlan x{};
    XArgs& a = x.a;
    a.k = ex.k;
    const bool h = part >= 0;
    a.chunk_log = L - ex.k - (h ? __builtin_popcountll(ex.pmask) : 0);
    a.chunk = 1ull << a.chunk_log;
    for (int j = 0; j < ex.k; ++j) {
        a.lpos[j] = ex.lpos[j];
        a.sorted[j] = ex.lpos[j];
        a.my_c |= ((rank >> (ex.gpos[j] - L)) & 1) << j;
    }
    a.nsorted = ex.k;
    if (h) {
        for (uint64_t m = ex.pmask; m; m &= m - 1) a.sorted[a.nsorted++] = __builtin_ctzll(m);
        a.orval = deposit_bits((uint64_t)part, ex.pmask);
    }
    std::sort(a.sorted, a.sorted + a.nsorted);
    for (int c = 0; c < (1 << ex.k); ++c) {
        int peer = rank;
        for (int j = 0; j < ex.k; ++j) {
            const int b = ex.gpos[j] - L;
            peer = (peer & ~(1 << b)) | (((c >> j) & 1) << b);
        }
        x.peer_of[c] = peer;
    }
    return x;
}
XPlan xplan(const qsim_dist* d, const Shard& sh, const DStep& ex, int part = -1) {
    XPlan x = xplan(d->L, sh.rank, ex, part);
    x.a.st = sh.d;
    return x;
}
void copy_kernel(bool pack, XArgs a, uint64_t lo, int sub_log, hipStream_t s) {
    const uint64_t total = (uint64_t)1 << (sub_log + a.k);
    const unsigned blocks = (unsigned)std::min<uint64_t>((total + 255) / 256, 256 * 64);
    if (pack) hipLaunchKernelGGL(k_exchange_copy<true>, dim3(blocks), dim3(256), 0, s, a, lo, sub_log);
    else hipLaunchKernelGGL(k_exchange_copy<false>, dim3(blocks), dim3(256), 0, s, a, lo, sub_log);
    QSIM_HIPCHK(hipGetLastError());
}
// Pipeline parts of a remap (QSIM_DIST_PIPELINE, default 4): slab offsets are split into parts
// so that part p's transfer overlaps the packing of later parts and the unpacking of earlier
// ones (pack and unpack run on the compute stream, transfers on the comm stream, ordered by
// events).  Parts below 1 MiB of amplitudes are not split further.
static int pipeline_parts(uint64_t chunk) {
    static const int want = [] {
        const char* e = std::getenv("QSIM_DIST_PIPELINE");
        const int v = e ? std::atoi(e) : 4;
        return v < 1 ? 1 : (v > 16 ? 16 : v);
    }();
    int parts = 1;
    while (parts * 2 <= want && (chunk / (uint64_t)(parts * 2)) >= (1ull << 16)) parts *= 2;
    return parts;
}
// Qubit remap: rank r sends its amplitudes with local bits lpos == c to the rank whose bits at
// gpos are c, and stores what that rank sends at local bits == c (the swap of the two qubit
// sets, SURVEY §8(e) "global<->local qubit swap by all-to-all").
//
// One point-to-point transfer posted by a shard: `amps` amplitudes at `send` go to rank `peer`
// and `amps` amplitudes from `peer` land at `recv` — one ncclSend / ncclRecv pair of a group on
// the multi-rank path.  Posts pair up by RCCL's rule: the k-th post of rank r naming q matches
// the k-th post of rank q naming r (and must carry the same count).
struct Post {
    int rank, peer;
    const double2* send;
    double2* recv;
    uint64_t amps;
};
// The posts of one remap part of shard `sh`: slab c (c != my_c) is the `amps` amplitudes at
// base + c * stride of the send / receive buffers; it goes to and comes from rank peer_of[c].
// Every transport runs this same per-shard loop (one shard per process, or all of them).
void slab_posts(std::vector<Post>& out, const Shard& sh, const XPlan& x, int k, uint64_t base,
                uint64_t stride, uint64_t amps) {
    for (int c = 0; c < (1 << k); ++c) {
        if (c == x.a.my_c) continue;
        const uint64_t at = base + (uint64_t)c * stride;
        out.push_back({sh.rank, x.peer_of[c], sh.sendbuf + at, sh.recvbuf + at, amps});
    }
}
// Virtual transport: move one matched slab inside this process — a device copy, or, with a
// world-1 communicator attached (qsim_dist_virtual_rccl), an ncclSend / ncclRecv pair to rank 0
// itself inside the caller's group (RCCL matches them in issue order).
void virt_move(qsim_dist* d, double2* dst, const double2* src, uint64_t amps) {
    if (!d->comm) {
        QSIM_HIPCHK(hipMemcpyAsync(dst, src, amps * sizeof(double2), hipMemcpyDeviceToDevice, d->comm_stream));
        return;
    }
    QSIM_NCCLCHK(ncclSend(src, (size_t)amps * 2, ncclDouble, 0, d->comm, d->comm_stream));
    QSIM_NCCLCHK(ncclRecv(dst, (size_t)amps * 2, ncclDouble, 0, d->comm, d->comm_stream));
}
// Hosted transport: hand host-staged copies of this rank's posts to the caller's function (which
// must move them between the rank processes with the same matching rule) and copy what arrived
// back.  Synchronous on the comm stream; for tests, not for speed.
void host_call(qsim_dist* d, const std::vector<qsim_dist_post>& hp, const char* what) {
    const int rc = d->host_fn(d->host_ctx, hp.data(), hp.size());
    if (rc != 0) fail(QSIM_ERR_DEVICE, std::string("host transport failed (") + std::to_string(rc) + ") during " + what);
}
char* host_stage(qsim_dist* d, size_t bytes) {
    if (bytes > d->h_stage_bytes) {
        if (d->h_stage) QSIM_HIPCHK(hipHostFree(d->h_stage));
        d->h_stage = nullptr;
        d->h_stage_bytes = 0;
        QSIM_HIPCHK(hipHostMalloc((void**)&d->h_stage, bytes, hipHostMallocDefault));
        d->h_stage_bytes = bytes;
    }
    return d->h_stage;
}
void host_transfers(qsim_dist* d, const std::vector<Post>& posts, const char* what) {
    size_t total = 0;
    for (const Post& p : posts) total += p.amps * sizeof(double2);
    char* snd = host_stage(d, 2 * total);
    char* rcv = snd + total;
    std::vector<qsim_dist_post> hp(posts.size());
    size_t at = 0;
    for (size_t i = 0; i < posts.size(); ++i) {
        const size_t b = posts[i].amps * sizeof(double2);
        QSIM_HIPCHK(hipMemcpyAsync(snd + at, posts[i].send, b, hipMemcpyDeviceToHost, d->comm_stream));
        hp[i] = {posts[i].peer, 0, (uint64_t)b, snd + at, rcv + at};
        at += b;
    }
    QSIM_HIPCHK(hipStreamSynchronize(d->comm_stream));
    host_call(d, hp, what);
    at = 0;
    for (size_t i = 0; i < posts.size(); ++i) {
        const size_t b = posts[i].amps * sizeof(double2);
        QSIM_HIPCHK(hipMemcpyAsync(posts[i].recv, rcv + at, b, hipMemcpyHostToDevice, d->comm_stream));
        at += b;
    }
    QSIM_HIPCHK(hipStreamSynchronize(d->comm_stream));
}
// Carry the posts of one remap part on d->comm_stream (which has already waited for the packs).
void post_transfers(qsim_dist* d, const std::vector<Post>& posts, const char* what) {
    if (posts.empty()) return;
    double sent = 0.0;
    for (const Post& p : posts) sent += (double)p.amps * sizeof(double2);
    d->sent_bytes += sent / (double)d->shards.size();
    TimedLaunch tl(&d->timer, "xgmi_transfer", 2.0 * sent / (double)d->shards.size(), d->comm_stream);
    switch (d->transport) {
        case qsim_dist::T_RCCL:
            QSIM_NCCLCHK(ncclGroupStart());
            for (const Post& p : posts) {
                QSIM_NCCLCHK(ncclSend(p.send, (size_t)p.amps * 2, ncclDouble, p.peer, d->comm, d->comm_stream));
                QSIM_NCCLCHK(ncclRecv(p.recv, (size_t)p.amps * 2, ncclDouble, p.peer, d->comm, d->comm_stream));
            }
            QSIM_NCCLCHK(ncclGroupEnd());
            comm_settle(d, what);
            return;
        case qsim_dist::T_HOSTED:
            host_transfers(d, posts, what);
            return;
        case qsim_dist::T_VIRTUAL: {
            // pair shard r's k-th post naming q with shard q's k-th post naming r; what r sends
            // lands where q receives (a mismatch is exactly what would hang a multi-rank run)
            std::map<std::pair<int, int>, std::vector<size_t>> by_pair;
            for (size_t i = 0; i < posts.size(); ++i) by_pair[{posts[i].rank, posts[i].peer}].push_back(i);
            if (d->comm) QSIM_NCCLCHK(ncclGroupStart());
            for (const auto& kv : by_pair) {
                const auto it = by_pair.find({kv.first.second, kv.first.first});
                if (it == by_pair.end() || it->second.size() != kv.second.size())
                    fail(QSIM_ERR_RUNTIME, std::string("unmatched slab transfer during ") + what);
                for (size_t j = 0; j < kv.second.size(); ++j) {
                    const Post& s = posts[kv.second[j]];
                    const Post& r = posts[it->second[j]];
                    if (s.amps != r.amps) fail(QSIM_ERR_RUNTIME, std::string("slab size mismatch during ") + what);
                    virt_move(d, r.recv, s.send, s.amps);
                }
            }
            if (d->comm) {
                QSIM_NCCLCHK(ncclGroupEnd());
                comm_settle(d, what);
            }
            return;
        }
    }
}

// A fused shard's own slab of part `base`: the pass wrote it to the send buffer, the step after
// reads the receive buffer (the slab never leaves the GPU: one device copy of 1 / 2^k of it).
void own_slab_copy(qsim_dist* d, const Shard& sh, const XPlan& x, uint64_t base, uint64_t stride, uint64_t amps,
                   hipStream_t s) {
    const uint64_t at = base + (uint64_t)x.a.my_c * stride;
    QSIM_HIPCHK(hipMemcpyAsync(sh.recvbuf + at, sh.sendbuf + at, amps * sizeof(double2), hipMemcpyDeviceToDevice, s));
}

void exchange(qsim_dist* d, const DStep& ex, const std::vector<char>& fused) {
    if (ex.k == 0) return;
    const uint64_t total = 1ull << d->L;
    const uint64_t chunk = total >> ex.k;
    const double bytes = 2.0 * 16.0 * (double)(total - chunk) * (double)d->shards.size();
    TimedLaunch tl(&d->timer, "alltoall_remap", bytes, d->stream);
    const int parts = pipeline_parts(chunk);
    int sub_log = d->L - ex.k;
    for (int p = parts; p > 1; p >>= 1) --sub_log;
    const uint64_t sub = 1ull << sub_log;
    if ((int)d->events.size() < 2 * parts) {
        const size_t have = d->events.size();
        d->events.resize(2 * parts, nullptr);
        for (size_t i = have; i < d->events.size(); ++i)
            QSIM_HIPCHK(hipEventCreateWithFlags(&d->events[i], hipEventDisableTiming));
    }
    std::vector<XPlan> xs;
    for (Shard& sh : d->shards) xs.push_back(xplan(d, sh, ex));
    for (int p = 0; p < parts; ++p) {
        for (size_t i = 0; i < d->shards.size(); ++i) {
            if (fused[i]) {  // (the pass before stored the slabs; the own slab moves on the device)
                own_slab_copy(d, d->shards[i], xs[i], (uint64_t)p * sub, chunk, sub, d->stream);
                continue;
            }
            XArgs a = xs[i].a;
            a.buf = d->shards[i].sendbuf;
            copy_kernel(true, a, (uint64_t)p * sub, sub_log, d->stream);
        }
        QSIM_HIPCHK(hipEventRecord(d->events[p], d->stream));
    }
    for (int p = 0; p < parts; ++p) {
        QSIM_HIPCHK(hipStreamWaitEvent(d->comm_stream, d->events[p], 0));
        std::vector<Post> posts;
        for (size_t i = 0; i < d->shards.size(); ++i)
            slab_posts(posts, d->shards[i], xs[i], ex.k, (uint64_t)p * sub, chunk, sub);
        post_transfers(d, posts, "remap send/recv");
        QSIM_HIPCHK(hipEventRecord(d->events[parts + p], d->comm_stream));
    }
    for (int p = 0; p < parts; ++p) {
        QSIM_HIPCHK(hipStreamWaitEvent(d->stream, d->events[parts + p], 0));
        for (size_t i = 0; i < d->shards.size(); ++i) {
            if (fused[i]) continue;  // (the step after loads the receive buffer itself)
            XArgs a = xs[i].a;
            a.buf = d->shards[i].recvbuf;
            copy_kernel(false, a, (uint64_t)p * sub, sub_log, d->stream);
        }
    }
}
// One overlapped remap: the K = 2^m parts of every shard (the values of the m pivot bits) are
// exchanged one after the other — pack and unpack on copy_stream, transfers on comm_stream —
// each part waiting for its local work (event pev[j], recorded on the compute stream after the
// role-1 step's part) and signalling pev[3 kMaxParts + j] when unpacked (the role-2 step's part waits for
// it).  Part j uses part j of the send / receive buffers, so all parts can be in flight.
// Part count of an overlapped remap with pivot mask pmask; the event array pev holds kMaxParts
// slots per kind, so a larger count is a planner bug, reported instead of overrunning it (round 4:
// a segfault when the pivot limit rose to 4 while pev still had 8 slots per kind).
int part_count(uint64_t pmask) {
    const int m = __builtin_popcountll(pmask);
    if (m > kMaxPivots) fail(QSIM_ERR_RUNTIME, "overlapped remap with " + std::to_string(m) + " pivots (at most " +
                                                   std::to_string(kMaxPivots) + ")");
    return 1 << m;
}
void exchange_parts(qsim_dist* d, const DStep& ex, const std::vector<char>& fused) {
    const int K = part_count(ex.pmask);
    const uint64_t part_amps = 1ull << (d->L - __builtin_popcountll(ex.pmask));
    const uint64_t chunk = part_amps >> ex.k;
    const double bytes = 2.0 * 16.0 * (double)(part_amps - chunk) * (double)d->shards.size();
    part_order(ex.pmask, ex.coarse & ex.pmask, d->order);  // (the same on every rank: RCCL pairs posts in order)
    for (int oi = 0; oi < K; ++oi) {
        const int h = d->order[oi];
        TimedLaunch tl(&d->timer, "alltoall_remap", bytes, d->copy_stream);
        std::vector<XPlan> xs;
        for (Shard& sh : d->shards) xs.push_back(xplan(d, sh, ex, h));
        QSIM_HIPCHK(hipStreamWaitEvent(d->copy_stream, d->pev[h], 0));
        for (size_t i = 0; i < d->shards.size(); ++i) {
            if (fused[i]) {  // (the tail pass of part h stored its slabs; own slab on the device)
                own_slab_copy(d, d->shards[i], xs[i], (uint64_t)h * part_amps, chunk, chunk, d->copy_stream);
                continue;
            }
            XArgs a = xs[i].a;
            a.buf = d->shards[i].sendbuf + (uint64_t)h * part_amps;
            copy_kernel(true, a, 0, xs[i].a.chunk_log, d->copy_stream);
        }
        QSIM_HIPCHK(hipEventRecord(d->pev[kMaxParts + h], d->copy_stream));
        QSIM_HIPCHK(hipStreamWaitEvent(d->comm_stream, d->pev[kMaxParts + h], 0));
        std::vector<Post> posts;
        for (size_t i = 0; i < d->shards.size(); ++i)
            slab_posts(posts, d->shards[i], xs[i], ex.k, (uint64_t)h * part_amps, chunk, chunk);
        post_transfers(d, posts, "overlapped remap send/recv");
        QSIM_HIPCHK(hipEventRecord(d->pev[2 * kMaxParts + h], d->comm_stream));
        QSIM_HIPCHK(hipStreamWaitEvent(d->copy_stream, d->pev[2 * kMaxParts + h], 0));
        for (size_t i = 0; i < d->shards.size(); ++i) {
            if (fused[i]) continue;  // (the step after loads part h from the receive buffer)
            XArgs a = xs[i].a;
            a.buf = d->shards[i].recvbuf + (uint64_t)h * part_amps;
            copy_kernel(false, a, 0, xs[i].a.chunk_log, d->copy_stream);
        }
        QSIM_HIPCHK(hipEventRecord(d->pev[3 * kMaxParts + h], d->copy_stream));
    }
}

// Sum of one double over the ranks (virtual: `local` already sums every shard; with a world-1
// communicator the all-reduce below runs anyway, as an identity).  Hosted: every rank sends its
// value to every other and sums in rank order (the same order, so the same result, everywhere).
double allreduce_sum(qsim_dist* d, double local) {
    if (d->transport == qsim_dist::T_HOSTED) {
        const int me = d->shards[0].rank;
        std::vector<double> vals(d->world, 0.0);
        vals[me] = local;
        std::vector<qsim_dist_post> hp;
        for (int r = 0; r < d->world; ++r)
            if (r != me) hp.push_back({r, 0, sizeof(double), &local, &vals[r]});
        host_call(d, hp, "all-reduce");
        double s = 0.0;
        for (double v : vals) s += v;
        return s;
    }
    if (!d->comm) return local;
    QSIM_HIPCHK(hipMemcpyAsync(d->d_result, &local, sizeof(double), hipMemcpyHostToDevice, d->stream));
    QSIM_NCCLCHK(ncclAllReduce(d->d_result, d->d_result, 1, ncclDouble, ncclSum, d->comm, d->stream));
    comm_settle(d, "all-reduce");
    double out = 0.0;
    QSIM_HIPCHK(hipMemcpyAsync(&out, d->d_result, sizeof(double), hipMemcpyDeviceToHost, d->stream));
    stream_wait(d, d->stream);
    return out;
}
// One ops step on one shard, split by passes around the neighbouring half-exchanges:
//   head   passes [0, j1) that avoid pivot pb (the exchange before): per half, each after its half
//          of the exchange has landed;
//   middle passes [j1, j2): whole shard, after both halves landed;
//   tail   passes [j2, P) that avoid pivot pa (the exchange after): per half, each followed by the
//          event its half-exchange waits for.
// The plan is the step's ordinary fused plan with tiles padded away from both pivots, so the
// split costs no extra HBM pass.  Per-gate mode (or a plan without such passes) runs whole.
StepRun prepare_step(qsim_dist* d, const std::vector<Op>& ops, int flags, PlanCache& pc, uint64_t pb,
                     uint64_t pa) {
    StepRun r;
    if (ops.empty() || !(flags & QSIM_RUN_FUSED)) return r;
    PlanCache::Entry& pe = pc.get(ops, d->L, d->stream, pa, pb);
    r.plan = &pe.plan;
    r.jm = jit_for(pe.jit, pe.plan, d->L);
    r.np = pe.plan.passes.size();
    if (pb)
        while (r.j1 < r.np && pass_avoids(pe.plan.passes[r.j1], pb)) ++r.j1;
    r.j2 = r.np;
    if (pa)
        while (r.j2 > r.j1 && pass_avoids(pe.plan.passes[r.j2 - 1], pa)) --r.j2;
    return r;
}
// Launch passes [first, last) of a prepared step (part >= 0: the part whose pivot bits `pmask`
// hold the bits of part); per-gate mode: the whole op list when called for the middle part.
// home / alt: where the step's passes read, and where a relayout pass (fused remap) writes
// (null: the shard's state, no second buffer).
void run_part(qsim_dist* d, Shard& sh, const std::vector<Op>& ops, const StepRun& r, size_t first,
              size_t last, uint64_t pmask = 0, int part = -1, double2* home = nullptr, double2* alt = nullptr) {
    if (ops.empty() || first >= last) return;
    if (!r.plan) {
        for (const Op& op : ops) launch_op(sh.d, d->L, 1, op, d->stream, &d->timer);
        return;
    }
    d->ops.upload(r.plan->ops.data(), r.plan->ops.size() * sizeof(TileOp), d->stream);
    d->stages.upload(r.plan->stages.data(), r.plan->stages.size() * sizeof(Stage), d->stream);
    FusedRange rg;
    rg.first = first;
    rg.last = last;
    rg.alt = alt;
    if (part >= 0) {
        rg.fix_mask = pmask;
        rg.fix_val = deposit_bits((uint64_t)part, pmask);
    }
    launch_fused(home ? home : sh.d, d->L, 1, *r.plan, (const TileOp*)d->ops.ptr, (const Stage*)d->stages.ptr,
                 d->stream, &d->timer, r.jm, nullptr, rg);
}

// The slab layout of exchange `ex` as a permutation of the local positions (the inverse of
// xlocal): positions outside lpos and the pivots ascending -> 0 .. L-k-m-1, lpos[j] -> L-m-k+j,
// the pivots ascending -> L-m .. L-1.  Part h of slab c is then the contiguous block at
// h * 2^(L-m) + c * 2^(L-m-k) of the send / receive buffers.
std::vector<int> slab_sigma(int L, const DStep& ex) {
    std::vector<int> s(L, -1);
    uint64_t moved = ex.pmask;
    for (int j = 0; j < ex.k; ++j) moved |= 1ull << ex.lpos[j];
    const int m = __builtin_popcountll(ex.pmask);
    int k = 0;
    for (int p = 0; p < L; ++p)
        if (!((moved >> p) & 1ull)) s[p] = k++;
    for (int j = 0; j < ex.k; ++j) s[ex.lpos[j]] = L - m - ex.k + j;
    int i = 0;
    for (uint64_t mm = ex.pmask; mm; mm &= mm - 1) s[__builtin_ctzll(mm)] = L - m + i++;
    return s;
}
bool fused_pack_enabled() {
    const char* e = std::getenv("QSIM_DIST_FUSED_PACK");  // (read per run: tests switch it)
    return e == nullptr || std::atoi(e) != 0;
}
Op map_op_positions(Op op, const std::vector<int>& sg) {
    op.t0 = sg[op.t0];
    if (op.kind == K_SWAP) op.t1 = sg[op.t1];
    uint64_t cm = 0;
    for (uint64_t m = op.cmask; m; m &= m - 1) cm |= 1ull << sg[__builtin_ctzll(m)];
    op.cmask = cm;
    return op;
}
// Per shard, whether the first exchange of run plan `rp` runs fused (steps [A, X, B] at the
// start of the run, fused ops plans on both sides; exchanged positions below 6 only cost the
// storing pass some coalescing: its lanes are the tile bits with the lowest store positions),
// and the two plans: A's with its last pass storing into
// the slab layout, B's planned on positions sigma(p) (the receive buffer's layout) with its last
// pass storing back to the standard positions.  The slab layout is the unfused exchange's, so
// shards decide independently.
// The variants are built the first time a run of this plan may use them (fused mode, fused pack
// on); whether a run uses them is decided per run from its own flags (fused_now), so a per-gate
// run of a cached plan never runs them and a fused run after a per-gate one still gets them.
bool fused_now(int flags) {
    return (flags & QSIM_RUN_FUSED) && fused_pack_enabled();
}
void decide_fused(qsim_dist* d, qsim_dist::RunPlan& rp, int flags) {
    const size_t S = d->shards.size();
    rp.fpack.resize(S);
    rp.funpack.resize(S);
    if (rp.fused_decided || !fused_now(flags)) return;
    rp.fused_decided = true;
    const std::vector<DStep>& st0 = rp.steps[0];
    if (st0.size() < 3 || st0[0].kind != 0 || st0[1].kind != 1 || st0[2].kind != 0 || (st0[2].role & 1))
        return;
    const DStep& ex = st0[1];
    if (ex.pmask & 0x3full) return;  // (pivots are >= 6 by construction)
    const std::vector<int> sg = slab_sigma(d->L, ex);
    std::vector<int> inv(d->L);
    for (int p = 0; p < d->L; ++p) inv[sg[p]] = p;
    uint64_t pm_sigma = 0;
    for (uint64_t m = ex.pmask; m; m &= m - 1) pm_sigma |= 1ull << sg[__builtin_ctzll(m)];
    for (size_t i = 0; i < S; ++i) {
        const DStep& A = rp.steps[i][0];
        const DStep& B = rp.steps[i][2];
        if (A.ops.empty() || B.ops.empty()) continue;
        auto pk = std::make_unique<qsim_dist::FusedVariant>();
        auto up = std::make_unique<qsim_dist::FusedVariant>();
        try {
            const uint64_t pa = (A.role & 1) ? ex.pmask : 0ull;
            const uint64_t pb = (A.role & 2) ? rp.carry_in : 0ull;
            pk->plan = plan_fused(A.ops, d->L, -1, pa, pb);
            const FusedPass& la = pk->plan.passes.back();
            if (la.single >= 0 || la.h < 4) continue;
            relayout_last_pass(pk->plan, d->L, sg.data());
            std::vector<Op> bops;
            for (const Op& op : B.ops) bops.push_back(map_op_positions(op, sg));
            up->plan = plan_fused(bops, d->L, -1, 0ull, (B.role & 2) ? pm_sigma : 0ull);
            const FusedPass& lb = up->plan.passes.back();
            if (lb.single >= 0 || lb.h < 4) continue;
            relayout_last_pass(up->plan, d->L, inv.data());
        } catch (const Error&) {
            continue;  // (this shard keeps the pack / unpack kernels)
        }
        pk->ok = up->ok = true;
        rp.fpack[i] = std::move(pk);
        rp.funpack[i] = std::move(up);
    }
}
StepRun prepare_variant(qsim_dist* d, qsim_dist::FusedVariant& v, uint64_t pb, uint64_t pa) {
    StepRun r;
    r.plan = &v.plan;
    r.jm = jit_for(v.jit, v.plan, d->L);
    r.np = v.plan.passes.size();
    if (pb)
        while (r.j1 < r.np && pass_avoids(v.plan.passes[r.j1], pb)) ++r.j1;
    r.j2 = r.np;
    if (pa)
        while (r.j2 > r.j1 && pass_avoids(v.plan.passes[r.j2 - 1], pa)) --r.j2;
    return r;
}
// The cached plan of this run (same gates, same start map), or a new one (LRU of 8).
qsim_dist::RunPlan& run_plan(qsim_dist* d, const qsim_gate* gates, size_t count, uint64_t carry) {
    for (auto& rp : d->run_plans)
        if (rp->perm_in == d->perm && rp->carry_in == carry && rp->gates.size() == count &&
            (count == 0 || std::memcmp(rp->gates.data(), gates, count * sizeof(qsim_gate)) == 0)) {
            rp->used = ++d->run_clock;
            return *rp;
        }
    auto rp = std::make_unique<qsim_dist::RunPlan>();
    rp->gates.assign(gates, gates + count);
    rp->perm_in = d->perm;
    rp->carry_in = carry;
    // Plan per shard (ranks differ only in which global controls/phases apply).
    for (const Shard& sh : d->shards) {
        std::vector<int> perm = d->perm;
        rp->steps.push_back(plan_dist(gates, count, d->n, d->g, sh.rank, perm, carry));
        rp->perm_out = perm;
        rp->fplans.emplace_back();
        for (const DStep& s : rp->steps.back())
            rp->fplans.back().push_back(s.kind == 0 ? std::make_unique<PlanCache>() : nullptr);
    }
    rp->used = ++d->run_clock;
    if (d->run_plans.size() >= 8) {
        auto lru = std::min_element(d->run_plans.begin(), d->run_plans.end(), [](const auto& a, const auto& b) {
            return a->in_use != b->in_use ? !a->in_use : a->used < b->used;  // (a pending step's plan stays)
        });
        QSIM_HIPCHK(hipStreamSynchronize(d->stream));  // its compiled kernels may still be queued
        d->run_plans.erase(lru);
    }
    d->run_plans.push_back(std::move(rp));
    return *d->run_plans.back();
}
// Run the carried step (the per-part head of the previous run's last remap) now, part by part as
// each part lands; every entry that touches the state, or a run that cannot merge it, calls this.
// A shard whose carried step has passes that touch the pivots (j1 < np: its lowering differs from
// rank 0's, e.g. gates dropped by a global control) runs those whole once every part has landed.
void flush_carry(qsim_dist* d) {
    qsim_dist::Carry& c = d->carry;
    if (!c.active) return;
    if (c.parts > kMaxParts) fail(QSIM_ERR_RUNTIME, "carried remap with too many parts");
    for (int oi = 0; oi < c.parts; ++oi) {
        const int h = d->order[oi];
        QSIM_HIPCHK(hipStreamWaitEvent(d->stream, d->pev[3 * kMaxParts + h], 0));
        for (size_t i = 0; i < d->shards.size(); ++i)
            if (c.runs[i].plan)
                run_part(d, d->shards[i], c.rp->steps[i][c.step].ops, c.runs[i], 0, c.runs[i].j1, c.pbs[i], h,
                         c.homes[i], c.alts[i]);
    }
    for (size_t i = 0; i < d->shards.size(); ++i)
        if (c.runs[i].plan && c.runs[i].j1 < c.runs[i].np)
            run_part(d, d->shards[i], c.rp->steps[i][c.step].ops, c.runs[i], c.runs[i].j1, c.runs[i].np, 0, -1,
                     c.homes[i], c.alts[i]);
    c.active = false;
    c.rp->in_use = false;
    c.rp = nullptr;
}
// Physical (rank-major) amplitudes -> logical index order (dst: 2 * 2^n doubles).  The map
// i -> p(i) moves bit q to perm[q], so p is the OR of per-11-bit-chunk tables; threads split i.
void unpermute(const qsim_dist* d, const std::vector<double2>& phys, double* dst) {
    const int n = d->n, nch = (n + 10) / 11;
    std::vector<uint64_t> tab((size_t)nch << 11, 0);
    for (int c = 0; c < nch; ++c)
        for (uint64_t v = 0; v < 2048; ++v)
            for (int b = 0; b < 11 && c * 11 + b < n; ++b)
                if ((v >> b) & 1ull) tab[((size_t)c << 11) + v] |= 1ull << d->perm[c * 11 + b];
    const uint64_t N = 1ull << n;
    const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(16, N >> 16));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (uint64_t i = N * t / T; i < N * (t + 1) / T; ++i) {
                uint64_t p = 0;
                for (int c = 0; c < nch; ++c) p |= tab[((size_t)c << 11) + ((i >> (11 * c)) & 2047)];
                dst[2 * i] = phys[p].x;
                dst[2 * i + 1] = phys[p].y;
            }
        });
    for (auto& x : th) x.join();
}
}  // namespace

extern "C" {

int qsim_dist_unique_id(void* id_out) {
    return dguard([&] {
        if (!id_out) fail(QSIM_ERR_INVALID_ARGUMENT, "null id buffer");
        static_assert(sizeof(ncclUniqueId) <= QSIM_DIST_UNIQUE_ID_BYTES, "unique id size");
        ncclUniqueId id;
        QSIM_NCCLCHK(ncclGetUniqueId(&id));
        std::memset(id_out, 0, QSIM_DIST_UNIQUE_ID_BYTES);
        std::memcpy(id_out, &id, sizeof(id));
    });
}

int qsim_dist_create(int n_qubits, int rank, int world, const void* unique_id, int device,
                     qsim_dist** out) {
    return dguard([&] {
        if (!out || !unique_id) fail(QSIM_ERR_INVALID_ARGUMENT, "null argument");
        *out = nullptr;
        const int g = log2_exact(world);
        if (rank < 0 || rank >= world) fail(QSIM_ERR_INVALID_ARGUMENT, "rank out of range");
        check_sizes(n_qubits, g);
        auto d = std::make_unique<qsim_dist>();
        d->n = n_qubits;
        d->g = g;
        d->L = n_qubits - g;
        d->world = world;
        d->device = device;
        d->perm.resize(n_qubits);
        QSIM_HIPCHK(hipSetDevice(device));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
        for (hipEvent_t& e : d->pev) QSIM_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        d->timer.stream = d->stream;
        alloc_shards(d.get(), {rank});
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        // Non-blocking communicator (QSIM_RCCL_BLOCKING=1 selects a blocking one): the init and
        // every later call can then be bounded by a timeout and aborted, so a rank that never
        // arrives (or dies) makes its peers fail instead of hanging.
        const char* bl = std::getenv("QSIM_RCCL_BLOCKING");
        const bool blocking = bl && std::atoi(bl) != 0;
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = blocking ? 1 : 0;
        const ncclResult_t ir = ncclCommInitRankConfig(&d->comm, world, id, rank, &cfg);
        if (ir != ncclSuccess && ir != ncclInProgress) {
            if (d->comm) (void)ncclCommAbort(d->comm);
            d->comm = nullptr;
            fail(QSIM_ERR_DEVICE, std::string("RCCL error: ") + ncclGetErrorString(ir));
        }
        try {
            comm_settle(d->comm, "communicator init", env_seconds("QSIM_DIST_INIT_TIMEOUT", 300.0));
        } catch (...) {
            (void)ncclCommAbort(d->comm);
            d->comm = nullptr;
            throw;
        }
        init_zero(d.get());
        *out = d.release();
    });
}

int qsim_dist_create_virtual(int n_qubits, int world, int device, qsim_dist** out) {
    return dguard([&] {
        if (!out) fail(QSIM_ERR_INVALID_ARGUMENT, "null argument");
        *out = nullptr;
        const int g = log2_exact(world);
        check_sizes(n_qubits, g);
        auto d = std::make_unique<qsim_dist>();
        d->n = n_qubits;
        d->g = g;
        d->L = n_qubits - g;
        d->world = world;
        d->device = device;
        d->virt = true;
        d->transport = qsim_dist::T_VIRTUAL;
        d->perm.resize(n_qubits);
        QSIM_HIPCHK(hipSetDevice(device));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
        for (hipEvent_t& e : d->pev) QSIM_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        d->timer.stream = d->stream;
        std::vector<int> ranks(world);
        for (int r = 0; r < world; ++r) ranks[r] = r;
        alloc_shards(d.get(), ranks);
        init_zero(d.get());
        *out = d.release();
    });
}

int qsim_dist_create_hosted(int n_qubits, int rank, int world, int device, qsim_dist_transport_fn fn,
                            void* ctx, qsim_dist** out) {
    return dguard([&] {
        if (!out || !fn) fail(QSIM_ERR_INVALID_ARGUMENT, "null argument");
        *out = nullptr;
        const int g = log2_exact(world);
        if (rank < 0 || rank >= world) fail(QSIM_ERR_INVALID_ARGUMENT, "rank out of range");
        check_sizes(n_qubits, g);
        auto d = std::make_unique<qsim_dist>();
        d->n = n_qubits;
        d->g = g;
        d->L = n_qubits - g;
        d->world = world;
        d->device = device;
        d->transport = qsim_dist::T_HOSTED;
        d->host_fn = fn;
        d->host_ctx = ctx;
        d->perm.resize(n_qubits);
        QSIM_HIPCHK(hipSetDevice(device));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
        for (hipEvent_t& e : d->pev) QSIM_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        d->timer.stream = d->stream;
        alloc_shards(d.get(), {rank});
        init_zero(d.get());
        *out = d.release();
    });
}

int qsim_dist_virtual_rccl(qsim_dist* d, const void* unique_id) {
    return dguard([&] {
        need(d);
        if (!d->virt || d->comm) fail(QSIM_ERR_INVALID_ARGUMENT, "needs a virtual object without a communicator");
        if (!unique_id) fail(QSIM_ERR_INVALID_ARGUMENT, "null argument");
        QSIM_HIPCHK(hipSetDevice(d->device));
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        const char* bl = std::getenv("QSIM_RCCL_BLOCKING");
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = bl && std::atoi(bl) != 0 ? 1 : 0;
        const ncclResult_t ir = ncclCommInitRankConfig(&d->comm, 1, id, 0, &cfg);
        if (ir != ncclSuccess && ir != ncclInProgress) {
            if (d->comm) (void)ncclCommAbort(d->comm);
            d->comm = nullptr;
            fail(QSIM_ERR_DEVICE, std::string("RCCL error: ") + ncclGetErrorString(ir));
        }
        try {
            comm_settle(d->comm, "communicator init", env_seconds("QSIM_DIST_INIT_TIMEOUT", 300.0));
        } catch (...) {
            (void)ncclCommAbort(d->comm);
            d->comm = nullptr;
            throw;
        }
    });
}

int qsim_dist_destroy(qsim_dist* d) {
    return dguard([&] { delete d; });
}

int qsim_dist_reset(qsim_dist* d) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        init_zero(d);
    });
}

int qsim_dist_run(qsim_dist* d, const qsim_gate* gates, size_t count, int flags) {
    return dguard_comm(d, [&] {
        need(d);
        if (!gates && count) fail(QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        QSIM_HIPCHK(hipSetDevice(d->device));
        if ((flags & QSIM_RUN_FUSED) && d->fresh && count > 0 && relabel_enabled(d->L)) {
            // Layout-aware relabeling of the LOCAL positions (relabel.hip): |0..0> stays |0..0>
            // under any relabeling, so the map is free to choose now.  Decided from rank 0's plan,
            // which every rank can compute, so all ranks pick the same map (the exchanges need
            // identical positions everywhere).  Global positions are untouched.
            std::vector<int> p0 = d->perm;
            const std::vector<DStep> st0 = plan_dist(gates, count, d->n, d->g, 0, p0);
            std::vector<uint64_t> tiles;
            for (const DStep& st : st0)
                if (st.kind == 0 && !st.ops.empty())
                    for (uint64_t t : plan_tiles(plan_fused(st.ops, d->L))) tiles.push_back(t);
            double before = 0.0, after = 0.0;
            const std::vector<int> pi = choose_relabel(tiles, d->L, &before, &after);
            if (!pi.empty())
                for (int q = 0; q < d->n; ++q)
                    if (d->perm[q] < d->L) d->perm[q] = pi[d->perm[q]];
        }
        d->fresh = false;
        d->sent_bytes = 0.0;
        const bool carry_on = carry_enabled();
        if (!(flags & QSIM_RUN_FUSED) || !carry_on) flush_carry(d);
        const uint64_t carry_in = d->carry.active ? d->carry.pmask : 0ull;
        qsim_dist::RunPlan& rp = run_plan(d, gates, count, carry_in);
        const auto& plans = rp.steps;
        const size_t S = d->shards.size();
        for (size_t i = 1; i < S; ++i)
            if (plans[i].size() != plans[0].size()) fail(QSIM_ERR_RUNTIME, "exchange skeleton mismatch");
        // merge the carried step into this run's first one (its leading passes per part too)
        const bool merge = d->carry.active && !plans[0].empty() && plans[0][0].kind == 0 && (plans[0][0].role & 2);
        if (!merge) flush_carry(d);
        d->overlapped = 0;
        d->fused_remaps = 0;
        decide_fused(d, rp, flags);
        std::vector<char> fused(S, 0);  // per shard: the first exchange runs fused
        for (size_t i = 0; i < S; ++i) fused[i] = fused_now(flags) && rp.fpack[i] && rp.fpack[i]->ok;
        const std::vector<char> unfused(S, 0);
        static const bool dbg = std::getenv("QSIM_DIST_DEBUG") != nullptr;
        if (dbg) {  // the exchange skeleton this run executes (kind, k, pivot mask, role)
            std::string line = "[dist] rank " + std::to_string(d->shards[0].rank) + " perm_in";
            for (int q = 0; q < d->n; ++q) line += " " + std::to_string(rp.perm_in[q]);
            line += " |";
            for (const DStep& st : plans[0])
                line += st.kind == 1 ? " X" + std::to_string(st.k) + ":" + std::to_string(st.pmask)
                                     : " O" + std::to_string(st.ops.size()) + "r" + std::to_string(st.role);
            std::fprintf(stderr, "%s\n", line.c_str());
        }
        int pending = merge ? d->carry.parts : 0;  // parts of an overlapped remap still to be waited for
        if (merge) ++d->carried;
        auto wait_pending = [&]() {
            if (pending > kMaxParts) fail(QSIM_ERR_RUNTIME, "pending remap with too many parts");
            for (int oi = 0; oi < pending; ++oi)
                QSIM_HIPCHK(hipStreamWaitEvent(d->stream, d->pev[3 * kMaxParts + d->order[oi]], 0));
            pending = 0;
        };
        // Every rank's plan has the same step skeleton (mark_overlap decides from
        // rank-independent data): walk the steps in lockstep.
        for (size_t k = 0; k < plans[0].size(); ++k) {
            const DStep& s0 = plans[0][k];
            for (size_t i = 1; i < S; ++i)
                if (plans[i][k].kind != s0.kind || plans[i][k].role != s0.role)
                    fail(QSIM_ERR_RUNTIME, "exchange skeleton mismatch");
            if (s0.kind == 1) {
                const std::vector<char>& fz = k == 1 ? fused : unfused;
                for (char f : fz) d->fused_remaps += f ? 1 : 0;
                if (s0.pmask) {
                    // the ops step before (role bit 1) recorded pev[j] after its tail part j;
                    // otherwise every part is ready now
                    const int K = part_count(s0.pmask);
                    wait_pending();
                    if (k == 0 || !(plans[0][k - 1].role & 1))
                        for (int h = 0; h < K; ++h) QSIM_HIPCHK(hipEventRecord(d->pev[h], d->stream));
                    exchange_parts(d, s0, fz);
                    pending = K;
                    ++d->overlapped;
                } else {
                    wait_pending();
                    exchange(d, s0, fz);
                }
                continue;
            }
            // ops step: head per half (after the exchange before), middle, tail per half
            const uint64_t pb = (s0.role & 2) ? (k == 0 ? carry_in : plans[0][k - 1].pmask) : 0ull;
            const uint64_t pa = (s0.role & 1) ? plans[0][k + 1].pmask : 0ull;
            std::vector<StepRun> runs(S);
            // fused first exchange: step 0 stores its last pass into the send buffer (slab
            // layout), step 2 reads the receive buffer in that layout (pivots at sigma's top
            // positions) and stores its last pass back to the state
            std::vector<uint64_t> pbs(S, pb);
            std::vector<double2*> homes(S, nullptr), alts(S, nullptr);
            for (size_t i = 0; i < S; ++i) {
                if (fused[i] && k == 0) {
                    runs[i] = prepare_variant(d, *rp.fpack[i], pb, pa);
                    alts[i] = d->shards[i].sendbuf;
                } else if (fused[i] && k == 2) {
                    const std::vector<int> sg = slab_sigma(d->L, plans[0][1]);
                    uint64_t ps = 0;
                    for (uint64_t m = pb; m; m &= m - 1) ps |= 1ull << sg[__builtin_ctzll(m)];
                    pbs[i] = ps;
                    runs[i] = prepare_variant(d, *rp.funpack[i], ps, 0);
                    homes[i] = d->shards[i].recvbuf;
                    alts[i] = d->shards[i].d;
                } else {
                    runs[i] = prepare_step(d, plans[i][k].ops, flags, *rp.fplans[i][k], pb, pa);
                }
            }
            const bool head = pb && pending;
            // the run's last step, the per-part head of the run's last remap: leave it pending (the
            // next run merges it into its first step's head; anything else flushes it).  Decided on
            // the step skeleton alone (roles, pivots: the same on every rank), never on this rank's
            // own passes — the next run plans its pivots with the carried ones (carry_in), so ranks
            // that decided differently would plan different part counts for the same exchange
            // (round 5 required every shard's step to lie wholly in the head; at world 8 / 20 qubits
            // some shards' lowerings differ from rank 0's — gates dropped by a global control — so
            // no run ever carried, and separate rank processes could have disagreed).  A shard whose
            // step has passes that touch the pivots runs them whole after the last part (flush_carry
            // and the merged head below).
            if (head && carry_on && k + 1 == plans[0].size() && !pa && (flags & QSIM_RUN_FUSED) && !(k == 0 && merge)) {
                {
                    qsim_dist::Carry& c = d->carry;
                    c.active = true;
                    c.pmask = pb;
                    c.parts = pending;
                    c.rp = &rp;
                    c.step = k;
                    c.runs = runs;
                    c.pbs = pbs;
                    c.homes = homes;
                    c.alts = alts;
                    rp.in_use = true;
                    pending = 0;
                    continue;
                }
            }
            if (head) {
                const bool carried = k == 0 && merge;
                const qsim_dist::Carry& c = d->carry;
                // a shard whose carried step is partial (see flush_carry) interleaves nothing: its
                // carried head per part, then after the last part the rest of that step whole and
                // this step's head whole
                auto partial = [&](size_t i) { return carried && c.runs[i].plan && c.runs[i].j1 < c.runs[i].np; };
                if (pending > kMaxParts) fail(QSIM_ERR_RUNTIME, "pending remap with too many parts");
                for (int oi = 0; oi < pending; ++oi) {
                    const int h = d->order[oi];
                    QSIM_HIPCHK(hipStreamWaitEvent(d->stream, d->pev[3 * kMaxParts + h], 0));
                    if (carried)  // part h of the previous run's last step, then part h of this one
                        for (size_t i = 0; i < S; ++i)
                            if (c.runs[i].plan)
                                run_part(d, d->shards[i], c.rp->steps[i][c.step].ops, c.runs[i], 0, c.runs[i].j1,
                                         c.pbs[i], h, c.homes[i], c.alts[i]);
                    for (size_t i = 0; i < S; ++i)
                        if (runs[i].plan && !partial(i))
                            run_part(d, d->shards[i], plans[i][k].ops, runs[i], 0, runs[i].j1, pbs[i], h, homes[i],
                                     alts[i]);
                }
                if (carried) {
                    for (size_t i = 0; i < S; ++i)
                        if (partial(i)) {
                            run_part(d, d->shards[i], c.rp->steps[i][c.step].ops, c.runs[i], c.runs[i].j1,
                                     c.runs[i].np, 0, -1, c.homes[i], c.alts[i]);
                            if (runs[i].plan)
                                run_part(d, d->shards[i], plans[i][k].ops, runs[i], 0, runs[i].j1, 0, -1, homes[i],
                                         alts[i]);
                        }
                    d->carry.active = false;
                    d->carry.rp->in_use = false;
                    d->carry.rp = nullptr;
                }
            }
            // coarse parts (DStep::coarse, rank-independent): this shard's passes just ahead of its
            // tail that avoid the coarse bits run per coarse part, each followed by the tails of its
            // fine parts, in the exchange's part order
            const uint64_t cb = pa ? (plans[0][k + 1].coarse & pa) : 0ull;
            std::vector<size_t> jc(S, 0);
            for (size_t i = 0; i < S; ++i) {
                if (!runs[i].plan) continue;
                jc[i] = runs[i].j2;
                const size_t lo = head ? runs[i].j1 : 0;
                if (cb)
                    while (jc[i] > lo && pass_avoids(runs[i].plan->passes[jc[i] - 1], cb)) --jc[i];
            }
            wait_pending();
            for (size_t i = 0; i < S; ++i) {
                if (runs[i].plan)
                    run_part(d, d->shards[i], plans[i][k].ops, runs[i], head ? runs[i].j1 : 0, jc[i], 0, -1,
                             homes[i], alts[i]);
                else run_part(d, d->shards[i], plans[i][k].ops, runs[i], 0, 1);  // per-gate: the whole list
            }
            if (pa) {  // the exchange after waits for pev[h]
                const int K = part_count(pa), Kc = 1 << __builtin_popcountll(cb), Kf = K / Kc;
                int ord[kMaxParts];
                part_order(pa, cb, ord);
                for (int cv = 0; cv < Kc; ++cv) {
                    if (cb)
                        for (size_t i = 0; i < S; ++i)
                            if (runs[i].plan)
                                run_part(d, d->shards[i], plans[i][k].ops, runs[i], jc[i], runs[i].j2, cb, cv, homes[i],
                                         alts[i]);
                    for (int f = 0; f < Kf; ++f) {
                        const int h = ord[cv * Kf + f];
                        for (size_t i = 0; i < S; ++i)
                            if (runs[i].plan)
                                run_part(d, d->shards[i], plans[i][k].ops, runs[i], runs[i].j2, runs[i].np, pa, h,
                                         homes[i], alts[i]);
                        QSIM_HIPCHK(hipEventRecord(d->pev[h], d->stream));
                    }
                }
            }
        }
        wait_pending();
        d->perm = rp.perm_out;
    });
}

int qsim_dist_remap_bytes(qsim_dist* d, double* sent) {
    return dguard([&] {
        need(d);
        if (sent) *sent = d->sent_bytes;
    });
}

int qsim_dist_fused_remaps(qsim_dist* d, int* remaps) {
    return dguard([&] {
        need(d);
        if (!remaps) fail(QSIM_ERR_INVALID_ARGUMENT, "null out");
        *remaps = d->fused_remaps;
    });
}

int qsim_dist_carried_runs(qsim_dist* d, int* runs) {
    return dguard([&] {
        need(d);
        if (!runs) fail(QSIM_ERR_INVALID_ARGUMENT, "null out");
        *runs = d->carried;
    });
}

int qsim_dist_overlapped(qsim_dist* d, int* remaps) {
    return dguard([&] {
        need(d);
        if (remaps) *remaps = d->overlapped;
    });
}

int qsim_dist_sync(qsim_dist* d) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        stream_wait(d, d->comm_stream);
        stream_wait(d, d->copy_stream);
        stream_wait(d, d->stream);
    });
}

// Every rank's engine idle, then a one-double all-reduce on the communicator: the ranks leave it
// within the collective's latency of one another (the timing barrier of bench.py's N > 1 steps —
// a host-file barrier releases its pollers milliseconds apart).
int qsim_dist_barrier(qsim_dist* d) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        stream_wait(d, d->comm_stream);
        stream_wait(d, d->copy_stream);
        stream_wait(d, d->stream);
        (void)allreduce_sum(d, 0.0);
    });
}

int qsim_dist_perm(qsim_dist* d, int32_t* perm) {
    return dguard([&] {
        need(d);
        for (int q = 0; q < d->n; ++q) perm[q] = d->perm[q];
    });
}

int qsim_dist_local_state(qsim_dist* d, double* dst) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        const size_t bytes = sizeof(double2) << d->L;
        for (size_t i = 0; i < d->shards.size(); ++i)  // virtual mode: all shards, rank order
            QSIM_HIPCHK(hipMemcpyAsync((char*)dst + i * bytes, d->shards[i].d, bytes,
                                       hipMemcpyDeviceToHost, d->stream));
        QSIM_HIPCHK(hipStreamSynchronize(d->stream));
    });
}

int qsim_dist_gather_state(qsim_dist* d, double* dst) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        const uint64_t shard = 1ull << d->L;
        const bool root = d->virt || d->shards[0].rank == 0;
        if (d->transport == qsim_dist::T_HOSTED) {  // host-staged: rank 0 receives every shard
            std::vector<double2> phys(root ? (1ull << d->n) : shard);
            QSIM_HIPCHK(hipMemcpyAsync(phys.data(), d->shards[0].d,
                                       sizeof(double2) * shard, hipMemcpyDeviceToHost, d->stream));
            QSIM_HIPCHK(hipStreamSynchronize(d->stream));
            std::vector<qsim_dist_post> hp;
            if (root)
                for (int r = 1; r < d->world; ++r)
                    hp.push_back({r, 0, sizeof(double2) * shard, nullptr, phys.data() + r * shard});
            else
                hp.push_back({0, 0, sizeof(double2) * shard, phys.data(), nullptr});
            host_call(d, hp, "gather");
            if (root && dst) unpermute(d, phys, dst);
            return;
        }
        double2* all = nullptr;
        if (root) QSIM_HIPCHK(hipMalloc((void**)&all, (sizeof(double2) << d->n)));
        if (d->virt) {
            for (const Shard& s : d->shards)
                QSIM_HIPCHK(hipMemcpyAsync(all + s.rank * shard, s.d, sizeof(double2) * shard,
                                           hipMemcpyDeviceToDevice, d->stream));
        } else {
            QSIM_NCCLCHK(ncclGroupStart());
            if (root) {
                QSIM_HIPCHK(hipMemcpyAsync(all, d->shards[0].d, sizeof(double2) * shard,
                                           hipMemcpyDeviceToDevice, d->stream));
                for (int r = 1; r < d->world; ++r)
                    QSIM_NCCLCHK(ncclRecv(all + r * shard, shard * 2, ncclDouble, r, d->comm, d->stream));
            } else {
                QSIM_NCCLCHK(ncclSend(d->shards[0].d, shard * 2, ncclDouble, 0, d->comm, d->stream));
            }
            QSIM_NCCLCHK(ncclGroupEnd());
            comm_settle(d, "gather");
        }
        stream_wait(d, d->stream);
        if (root) {
            std::vector<double2> phys(1ull << d->n);
            QSIM_HIPCHK(hipMemcpy(phys.data(), all, sizeof(double2) << d->n, hipMemcpyDeviceToHost));
            QSIM_HIPCHK(hipFree(all));
            if (dst) unpermute(d, phys, dst);
        }
    });
}

int qsim_dist_total_probability(qsim_dist* d, double* out) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        QSIM_HIPCHK(hipSetDevice(d->device));
        double local = 0.0;
        for (const Shard& s : d->shards)
            local += reduce_norm(s.d, d->L, -1, d->d_partials, d->d_result, d->stream);
        *out = allreduce_sum(d, local);
    });
}

int qsim_dist_prob_bit_zero(qsim_dist* d, int q, double* out) {
    return dguard_comm(d, [&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        flush_carry(d);  // (the previous run's last step, if it was left pending)
        if (q < 0 || q >= d->n) fail(QSIM_ERR_INVALID_ARGUMENT, "bit out of range");
        QSIM_HIPCHK(hipSetDevice(d->device));
        const int p = d->perm[q];
        double local = 0.0;
        for (const Shard& s : d->shards) {
            if (p < d->L) local += reduce_norm(s.d, d->L, p, d->d_partials, d->d_result, d->stream);
            else if (!((s.rank >> (p - d->L)) & 1))
                local += reduce_norm(s.d, d->L, -1, d->d_partials, d->d_result, d->stream);
        }
        *out = allreduce_sum(d, local);
    });
}

int qsim_dist_profile(qsim_dist* d, int enable) {
    return dguard([&] {
        need(d);
        d->timer.enabled = enable != 0;
    });
}

int qsim_dist_profile_count(qsim_dist* d, int* n) {
    return dguard([&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        d->timer.resolve();
        *n = (int)d->timer.stats.size();
    });
}

int qsim_dist_profile_get(qsim_dist* d, int i, char* name, size_t name_len, double* total_ms,
                          int64_t* launches, double* alg_bytes) {
    return dguard([&] {
        need(d);
        QSIM_HIPCHK(hipSetDevice(d->device));
        d->timer.resolve();
        if (i < 0 || i >= (int)d->timer.stats.size()) fail(QSIM_ERR_OUT_OF_RANGE, "bad index");
        const auto& st = d->timer.stats[i];
        if (name && name_len) {
            std::strncpy(name, st.name.c_str(), name_len - 1);
            name[name_len - 1] = 0;
        }
        if (total_ms) *total_ms = st.ms;
        if (launches) *launches = st.launches;
        if (alg_bytes) *alg_bytes = st.bytes;
    });
}

int qsim_dist_plan(int n, int world, int rank, const qsim_gate* gates, size_t count,
                   int32_t* perm_inout, qsim_dist_step* steps, size_t step_cap, size_t* n_steps,
                   qsim_op* ops, size_t op_cap, size_t* n_ops) {
    return dguard([&] {
        const int g = log2_exact(world);
        check_sizes(n, g);
        if (rank < 0 || rank >= world) fail(QSIM_ERR_INVALID_ARGUMENT, "rank out of range");
        std::vector<int> perm(n);
        for (int q = 0; q < n; ++q) perm[q] = perm_inout ? perm_inout[q] : q;
        const std::vector<DStep> st = plan_dist(gates, count, n, g, rank, perm);
        size_t si = 0, oi = 0;
        for (const DStep& s : st) {
            if (si < step_cap) {
                qsim_dist_step& o = steps[si];
                std::memset(&o, 0, sizeof(o));
                o.kind = s.kind;
                o.k = s.k;
                o.op_begin = (int32_t)oi;
                o.op_end = (int32_t)(oi + s.ops.size());
                for (int j = 0; j < 8; ++j) {
                    o.gpos[j] = s.gpos[j];
                    o.lpos[j] = s.lpos[j];
                }
                o.pivot = s.pivot;
                o.pmask = s.pmask;
                o.coarse = s.coarse;
                o.role = s.role;
            }
            for (const Op& op : s.ops) {
                if (oi < op_cap) {
                    qsim_op& r = ops[oi];
                    r.kind = op.kind;
                    r.sub = op.sub;
                    r.t0 = op.t0;
                    r.t1 = op.t1;
                    r.cmask = op.cmask;
                    r.d0_one = op.d0_one ? 1 : 0;
                    r.src = op.src;
                    for (int j = 0; j < 8; ++j) r.m[j] = op.m[j];
                }
                ++oi;
            }
            ++si;
        }
        if (n_steps) *n_steps = si;
        if (n_ops) *n_ops = oi;
        if (perm_inout)
            for (int q = 0; q < n; ++q) perm_inout[q] = perm[q];
    });
}

static int plan_passes_impl(int n, int world, int rank, const qsim_gate* gates, size_t count, int32_t* perm_inout,
                            uint64_t* carry_inout, int32_t* passes, size_t cap, size_t* n_steps, int width) {
    return dguard([&] {
        const int g = log2_exact(world);
        check_sizes(n, g);
        if (rank < 0 || rank >= world) fail(QSIM_ERR_INVALID_ARGUMENT, "rank out of range");
        std::vector<int> perm(n);
        for (int q = 0; q < n; ++q) perm[q] = perm_inout ? perm_inout[q] : q;
        const uint64_t carry = carry_inout ? *carry_inout : 0ull;
        const std::vector<DStep> st = plan_dist(gates, count, n, g, rank, perm, carry);
        const int L = n - g;
        uint64_t carry_out = 0;
        for (size_t k = 0; k < st.size(); ++k) {
            int np = 0, head = 0, tail = 0, coarse = 0, coarse_bits = 0;
            if (st[k].kind == 0 && !st[k].ops.empty()) {  // as prepare_step plans it
                const uint64_t pb = (st[k].role & 2) ? (k == 0 ? carry : st[k - 1].pmask) : 0ull;
                const uint64_t pa = (st[k].role & 1) ? st[k + 1].pmask : 0ull;
                const Plan pl = plan_fused(st[k].ops, L, -1, pa, pb);
                np = (int)pl.passes.size();
                if (pb)
                    while (head < np && pass_avoids(pl.passes[head], pb)) ++head;
                if (pa)
                    while (tail < np - head && pass_avoids(pl.passes[np - 1 - tail], pa)) ++tail;
                const uint64_t cb = pa ? (st[k + 1].coarse & pa) : 0ull;
                if (cb) {  // as qsim_dist_run splits the step
                    int jc = np - tail;
                    while (jc > head && pass_avoids(pl.passes[jc - 1], cb)) --jc;
                    coarse = np - tail - jc;
                    coarse_bits = __builtin_popcountll(cb);
                }
                static const bool dbg = std::getenv("QSIM_DIST_DEBUG_PASSES") != nullptr;
                if (dbg && pa) {  // the exchange-after pivots each pass touches
                    std::string line = "[passes] step " + std::to_string(k) + " pa " + std::to_string(pa) + ":";
                    for (int j = 0; j < np; ++j) {
                        uint64_t tm = 0;
                        const FusedPass& fp = pl.passes[j];
                        if (fp.single >= 0 || fp.h < 4) tm = pa;
                        else
                            for (int i = 0; i < 6 + fp.h - fp.r0; ++i) tm |= pa & (1ull << fp.hpos[i]);
                        line += " " + std::to_string(__builtin_popcountll(tm));
                    }
                    std::fprintf(stderr, "%s\n", line.c_str());
                }
            }
            if (k < cap && passes) {
                passes[width * k] = st[k].kind == 1 ? -1 : np;
                passes[width * k + 1] = head;
                passes[width * k + 2] = tail;
                if (width >= 5) {
                    passes[width * k + 3] = coarse;
                    passes[width * k + 4] = coarse_bits;
                }
            }
            // the per-part head of the run's last remap is carried into the next run (qsim_dist_run:
            // decided on the skeleton alone, the same on every rank)
            if (k + 1 == st.size() && k > 0 && st[k].kind == 0 && (st[k].role & 2) && !(st[k].role & 1) &&
                st[k - 1].pmask)
                carry_out = st[k - 1].pmask;
        }
        if (n_steps) *n_steps = st.size();
        if (perm_inout)
            for (int q = 0; q < n; ++q) perm_inout[q] = perm[q];
        if (carry_inout) *carry_inout = carry_out;
    });
}

int qsim_dist_plan_passes_carry(int n, int world, int rank, const qsim_gate* gates, size_t count,
                                int32_t* perm_inout, uint64_t* carry_inout, int32_t* passes, size_t cap,
                                size_t* n_steps) {
    return plan_passes_impl(n, world, rank, gates, count, perm_inout, carry_inout, passes, cap, n_steps, 3);
}

int qsim_dist_plan_passes_coarse(int n, int world, int rank, const qsim_gate* gates, size_t count,
                                 int32_t* perm_inout, uint64_t* carry_inout, int32_t* passes, size_t cap,
                                 size_t* n_steps) {
    return plan_passes_impl(n, world, rank, gates, count, perm_inout, carry_inout, passes, cap, n_steps, 5);
}

int qsim_dist_plan_passes(int n, int world, int rank, const qsim_gate* gates, size_t count,
                          int32_t* perm_inout, int32_t* passes, size_t cap, size_t* n_steps) {
    return qsim_dist_plan_passes_carry(n, world, rank, gates, count, perm_inout, nullptr, passes, cap, n_steps);
}

int qsim_dist_plan_memo_clear(void) {
    return dguard([&] {
        std::lock_guard<std::mutex> l(g_pivot_mu);
        g_pivots.clear();
        g_cycles.clear();
    });
}

int qsim_dist_slab_map(int n, int world, int rank, const qsim_dist_step* step, int part,
                       int32_t* my_c, int32_t* peer_of, uint64_t* index, size_t index_cap) {
    return dguard([&] {
        const int g = log2_exact(world);
        check_sizes(n, g);
        if (rank < 0 || rank >= world) fail(QSIM_ERR_INVALID_ARGUMENT, "rank out of range");
        if (!step || step->kind != 1 || step->k < 1 || step->k > g)
            fail(QSIM_ERR_INVALID_ARGUMENT, "not an exchange step");
        const int L = n - g;
        DStep ex;
        ex.kind = 1;
        ex.k = step->k;
        uint64_t used = 0;
        for (int j = 0; j < ex.k; ++j) {
            ex.gpos[j] = step->gpos[j];
            ex.lpos[j] = step->lpos[j];
            if (ex.gpos[j] < L || ex.gpos[j] >= n || ex.lpos[j] < 0 || ex.lpos[j] >= L ||
                ((used >> ex.lpos[j]) & 1ull))
                fail(QSIM_ERR_INVALID_ARGUMENT, "bad exchange positions");
            used |= 1ull << ex.lpos[j];
        }
        ex.pmask = step->pmask;
        if (ex.pmask & (used | ~((1ull << L) - 1)))
            fail(QSIM_ERR_INVALID_ARGUMENT, "bad pivot mask");
        const int m = __builtin_popcountll(ex.pmask);
        if (part >= (1 << m)) fail(QSIM_ERR_INVALID_ARGUMENT, "part out of range");
        const XPlan x = xplan(L, rank, ex, part < 0 ? -1 : part);
        if (my_c) *my_c = x.a.my_c;
        if (peer_of)
            for (int c = 0; c < (1 << ex.k); ++c) peer_of[c] = x.peer_of[c];
        const uint64_t count = (uint64_t)x.a.chunk << ex.k;
        if (index) {
            if (index_cap < count) fail(QSIM_ERR_INVALID_ARGUMENT, "index buffer too small");
            for (uint64_t e = 0; e < count; ++e) index[e] = xlocal(x.a, e);
        }
    });
}

}  // extern "C"
