// relayout.hip — relayout plans: every tile pass stores its tile under the NEXT pass's layout.
//
// A staged pass's tile always spans the physical run positions 0..r0-1 (the contiguous HBM run
// each wave instruction moves), so under one fixed layout every pass of a plan shares the same
// r0 >= 4 qubits and only 12 - r0 tile slots are free (fused.hip: plan_fused).  But a pass reads
// and writes every amplitude exactly once, and it may write them anywhere: storing tile bit x at
// physical position st_pos[x] and the tile-id bits at st_tid[] instead of where they were loaded
// from is a qubit relabeling at no extra HBM traffic.  The only constraint is coalescing: the
// store's run positions 0..3 must receive qubits of the storing pass's own tile.  So a plan is a
// sequence of 12-qubit tiles T_1..T_K in which consecutive tiles (and T_K, T_1: the last pass
// restores the first layout, so a re-run of the circuit starts where the first run did and
// readers' restore logic is unchanged) share at least four qubits — the next pass's run — and
// every other tile qubit, and its physical position, is free.  W-HC 30q: 5 passes with a fixed
// run, 4 as relayout passes (seed 42); 6 -> 5 for seeds 1, 2, 4.
//
// Search: a beam over tile sequences (like fused.hip's beam_passes; a state is the set of gates
// not yet run) where a tile grows one qubit at a time from the first remaining gate, keeping
// enough slots for four qubits of the previous tile.  Layouts: the run of pass k+1 goes to
// positions 0..3, the other qubits of T_k and T_k+1 to the positions the layout cost model
// (layout_cost.hpp, one-pass probes) prices lowest for T_k's store plus T_k+1's load.  The
// reference has one kernel launch per gate (src/Simulator.cu:28-154); none of this exists there.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <random>
#include <unordered_set>

#include "engine.hpp"

namespace qsim_hip {

namespace {

constexpr int kTile = 12;  // 12-qubit tiles (h = 6): two 64 KiB workgroups per CU
constexpr int kRun = 4;    // qubits shared by consecutive tiles (the next pass's 256 B run)

int env_int(const char* k, int d) {
    const char* e = std::getenv(k);
    return e ? std::atoi(e) : d;
}

uint64_t op_mask(const Op& op) {
    uint64_t m = op.cmask | (1ull << op.t0);
    if (op.kind == K_SWAP) m |= 1ull << op.t1;
    return m;
}

// Qubits an op needs inside the tile: its targets; with tile-id controls (QSIM_TILE_CTRL_OUT) a
// control outside the tile is a tile constant (the op runs on the tiles where it reads 1).
uint64_t op_need(const Op& op, bool ctrl_out) {
    if (!ctrl_out) return op_mask(op);
    uint64_t m = 1ull << op.t0;
    if (op.kind == K_SWAP) m |= 1ull << op.t1;
    return m;
}

struct Search {
    const std::vector<uint64_t>& qm;   // every qubit of the op (ordering: ops on disjoint qubits commute)
    int n;
    const std::vector<uint64_t>& need;  // the qubits the tile must hold
    size_t window = 512;

    // (gates admitted, gates partly covered) over the first `window` remaining gates
    int score(const std::vector<int>& rem, uint64_t allowed) const {
        uint64_t blocked = 0;
        int full = 0, part = 0;
        const size_t m = std::min(rem.size(), window);
        for (size_t i = 0; i < m; ++i) {
            const uint64_t q = qm[rem[i]], nd = need[rem[i]];
            if (q & blocked) {
                blocked |= q;
            } else if ((nd & ~allowed) == 0) {
                ++full;
            } else {
                if (nd & allowed) ++part;
                blocked |= q;
            }
        }
        return full * 4096 + part;
    }
    // the gates a pass over `allowed` leaves (a gate runs unless it needs another qubit or shares
    // one with a gate left behind: gates on disjoint qubits commute exactly)
    std::vector<int> apply(const std::vector<int>& rem, uint64_t allowed, std::vector<int>* ran = nullptr) const {
        std::vector<int> out;
        uint64_t blocked = 0;
        for (int i : rem) {
            const uint64_t q = qm[i];
            if ((q & blocked) == 0 && (need[i] & ~allowed) == 0) {
                if (ran) ran->push_back(i);
                continue;
            }
            out.push_back(i);
            blocked |= q;
        }
        return out;
    }
};

struct St {
    std::vector<int> rem;
    std::vector<uint64_t> tiles;
};

struct VecHash {
    size_t operator()(const std::vector<int>& v) const {
        uint64_t h = 0x9e3779b97f4a7c15ull ^ v.size();
        for (int x : v) h = (h ^ (uint64_t)x) * 0x100000001b3ull;
        return (size_t)h;
    }
};

// Last tile rebuilt so that it shares kRun qubits with the first (the cycle closes): its gates'
// qubits, a run from the tile before it, qubits of the first tile, then its old padding.
bool close_cycle(std::vector<uint64_t>& T, const std::vector<uint64_t>& U) {
    const size_t K = T.size();
    if (K == 1 || __builtin_popcountll(T[K - 1] & T[0]) >= kRun) return true;
    uint64_t t = U[K - 1];
    const uint64_t ov = T[K - 2] & T[K - 1];
    // the run the last pass loads: from T[K-2] & T[K-1], preferring qubits it needs anyway and
    // qubits of the first tile
    int have = __builtin_popcountll(t & ov);
    for (int pref = 0; pref < 2 && have < kRun; ++pref)
        for (uint64_t m = ov & ~t; m && have < kRun; m &= m - 1) {
            const uint64_t b = m & (~m + 1);
            if (pref == 0 && !(b & T[0])) continue;
            t |= b;
            ++have;
        }
    if (have < kRun) return false;
    for (uint64_t m = T[0] & ~t; m && __builtin_popcountll(t & T[0]) < kRun; m &= m - 1) t |= m & (~m + 1);
    if (__builtin_popcountll(t & T[0]) < kRun || __builtin_popcountll(t) > kTile) return false;
    for (uint64_t m = T[K - 1] & ~t; m && __builtin_popcountll(t) < kTile; m &= m - 1) t |= m & (~m + 1);
    T[K - 1] = t;
    return true;
}

std::vector<std::vector<uint64_t>> search_tiles(const Search& S, size_t nops, int width, size_t max_passes,
                                               int nvar) {
    const int n = S.n;
    std::vector<St> states(1);
    states[0].rem.resize(nops);
    for (size_t i = 0; i < nops; ++i) states[0].rem[i] = (int)i;
    const uint64_t all = n >= 64 ? ~0ull : (1ull << n) - 1ull;
    for (size_t step = 0; step < max_passes; ++step) {
        std::vector<St> next;
        std::unordered_set<std::vector<int>, VecHash> seen;
        for (const St& s : states) {
            const uint64_t prev = s.tiles.empty() ? 0ull : s.tiles.back();
            const uint64_t seed = S.need[s.rem.front()];
            std::vector<std::pair<int, uint64_t>> part = {{S.score(s.rem, seed), seed}};
            for (;;) {
                bool grew = false;
                std::vector<std::pair<int, uint64_t>> grown;
                std::unordered_set<uint64_t> dup;
                for (const auto& pp : part) {
                    const uint64_t h = pp.second;
                    const int sz = __builtin_popcountll(h);
                    if (sz >= kTile) {
                        if (dup.insert(h).second) grown.push_back(pp);
                        continue;
                    }
                    grew = true;
                    const int need = prev ? std::max(0, kRun - __builtin_popcountll(h & prev)) : 0;
                    const uint64_t cand = (sz + need < kTile ? all : prev) & ~h;
                    for (uint64_t m = cand; m; m &= m - 1) {
                        const uint64_t hh = h | (m & (~m + 1));
                        if (dup.insert(hh).second) grown.push_back({S.score(s.rem, hh), hh});
                    }
                }
                if (!grew) break;
                std::stable_sort(grown.begin(), grown.end(),
                                 [](const auto& a, const auto& b) { return a.first > b.first; });
                if ((int)grown.size() > width) grown.resize(width);
                part.swap(grown);
            }
            for (const auto& pp : part) {
                St t;
                t.rem = S.apply(s.rem, pp.second);
                // (finished sequences are all kept: they are the variants a timed first run compares)
                if (t.rem.size() == s.rem.size() || (!t.rem.empty() && !seen.insert(t.rem).second)) continue;
                t.tiles = s.tiles;
                t.tiles.push_back(pp.second);
                next.push_back(std::move(t));
            }
        }
        if (next.empty()) return {};
        std::stable_sort(next.begin(), next.end(), [](const St& a, const St& b) { return a.rem.size() < b.rem.size(); });
        std::vector<std::vector<uint64_t>> done;  // closed sequences of this (the fewest-pass) step
        for (St& s : next) {
            if (!s.rem.empty()) break;
            // a finished sequence: close the cycle (its gates per pass first)
            std::vector<uint64_t> U;
            std::vector<int> rem(nops);
            for (size_t i = 0; i < nops; ++i) rem[i] = (int)i;
            for (uint64_t t : s.tiles) {
                std::vector<int> ran;
                rem = S.apply(rem, t, &ran);
                uint64_t u = 0;
                for (int i : ran) u |= S.need[i];
                U.push_back(u);
            }
            if (close_cycle(s.tiles, U)) {
                done.push_back(s.tiles);
                if ((int)done.size() >= nvar) break;
            }
        }
        if (!done.empty()) return done;
        next.erase(std::remove_if(next.begin(), next.end(), [](const St& s) { return s.rem.empty(); }), next.end());
        if (next.empty()) return {};
        if ((int)next.size() > width) next.resize(width);
        states.swap(next);
    }
    return {};
}

// A layout (logical -> physical) with `run` at positions 0..3 and the other qubits of x (the
// tile stored into this layout) and y (the tile loaded from it) where the layout model prices
// store + load lowest; the remaining qubits fill the remaining positions in order.
// seed: the hill climbing's restarts (layout variants of one tile sequence differ by it)
std::vector<int> assign_layout(int n, uint64_t run, uint64_t x, uint64_t y, unsigned seed = 0) {
    std::vector<int> L(n, -1);
    int k = 0;
    for (uint64_t m = run; m; m &= m - 1) L[__builtin_ctzll(m)] = k++;
    std::vector<int> sq;
    // QSIM_RELAYOUT_RUN6=1: positions 4 and 5 go to tile qubits first (shared ones, then the
    // loading tile's), so loads and stores move whole 1 KiB runs where the tiles allow
    // (2: the storing tile's qubits instead, so the stores move whole runs)
    static const int run6 = env_int("QSIM_RELAYOUT_RUN6", 0);
    int first = kRun;
    if (run6) {
        const uint64_t pref[2] = {x & y & ~run, (run6 == 2 ? x : y) & ~run};
        for (int p = kRun; p < 6; ++p)
            for (uint64_t c : pref) {
                uint64_t m = c;
                for (int q = 0; q < n; ++q)
                    if (L[q] >= 0) m &= ~(1ull << q);
                if (!m) continue;
                L[__builtin_ctzll(m)] = p;
                first = p + 1;
                break;
            }
    }
    uint64_t placed = run;  // qubits with a position already
    for (int q = 0; q < n; ++q)
        if (L[q] >= 0) placed |= 1ull << q;
    const int npos = n - first;  // positions first..n-1
    for (uint64_t m = (x | y) & ~placed; m; m &= m - 1) sq.push_back(__builtin_ctzll(m));
    uint64_t fixed_x = 0, fixed_y = 0;  // positions already taken by x / y qubits
    for (int q = 0; q < n; ++q)
        if (L[q] >= 0) {
            if ((x >> q) & 1ull) fixed_x |= 1ull << L[q];
            if ((y >> q) & 1ull) fixed_y |= 1ull << L[q];
        }
    auto cost = [&](const std::vector<int>& pos_of) {
        uint64_t mx = fixed_x, my = fixed_y;
        for (size_t i = 0; i < sq.size(); ++i) {
            const uint64_t b = 1ull << sq[i];
            if (x & b) mx |= 1ull << pos_of[i];
            if (y & b) my |= 1ull << pos_of[i];
        }
        return layout_cost_us(mx) + layout_cost_us(my);
    };
    std::vector<int> best_pos;
    double best = 1e300;
    for (int restart = 0; restart < 4; ++restart) {
        std::mt19937 rng(0x7e1a0u + (unsigned)restart + 0x1000u * seed);
        std::vector<int> slots(npos);
        for (int i = 0; i < npos; ++i) slots[i] = first + i;
        if (restart > 0) std::shuffle(slots.begin(), slots.end(), rng);
        // sq[i] at slots[i]; slots beyond sq.size() are free
        std::vector<int> pos_of(slots.begin(), slots.begin() + sq.size());
        double cur = cost(pos_of);
        std::uniform_int_distribution<int> pick_q(0, (int)sq.size() - 1), pick_p(0, npos - 1);
        for (int it = 0; it < 3000; ++it) {
            const int a = pick_q(rng), pb = first + pick_p(rng);
            int b = -1;  // the qubit of sq at position pb, if any
            for (size_t i = 0; i < sq.size(); ++i)
                if (pos_of[i] == pb) b = (int)i;
            if (b == a) continue;
            const int pa = pos_of[a];
            pos_of[a] = pb;
            if (b >= 0) pos_of[b] = pa;
            const double c = cost(pos_of);
            if (c <= cur) {
                cur = c;
            } else {
                pos_of[a] = pa;
                if (b >= 0) pos_of[b] = pb;
            }
        }
        if (cur < best) {
            best = cur;
            best_pos = pos_of;
        }
    }
    std::vector<char> used(n, 0);
    for (int q = 0; q < n; ++q)
        if (L[q] >= 0) used[L[q]] = 1;
    for (size_t i = 0; i < sq.size(); ++i) {
        L[sq[i]] = best_pos[i];
        used[best_pos[i]] = 1;
    }
    int p = 0;
    for (int q = 0; q < n; ++q) {
        if (L[q] >= 0) continue;
        while (used[p]) ++p;
        L[q] = p;
        used[p] = 1;
    }
    return L;
}

// kRun qubits of `pool` for a run, the least used as gate targets by the two passes whose lanes
// they become (lane bits can only be register bits in a middle stage)
uint64_t choose_run(uint64_t pool, const int* uses) {
    std::vector<int> q;
    for (uint64_t m = pool; m; m &= m - 1) q.push_back(__builtin_ctzll(m));
    std::stable_sort(q.begin(), q.end(), [&](int a, int b) { return uses[a] < uses[b]; });
    uint64_t r = 0;
    for (int i = 0; i < kRun && i < (int)q.size(); ++i) r |= 1ull << q[i];
    return r;
}

}  // namespace

static std::atomic<int> g_relayout{-1}, g_relayout_min{-1};
bool relayout_enabled(int n) {
    if (g_relayout.load() < 0) g_relayout.store(env_int("QSIM_RELAYOUT", 1));
    if (g_relayout_min.load() < 0) g_relayout_min.store(env_int("QSIM_RELAYOUT_MIN_QUBITS", 20));
    return g_relayout.load() != 0 && n >= g_relayout_min.load() && n - kTile <= 32;
}
bool relayout_forced() { return g_relayout.load() == 2; }
void relayout_configure(int mode, int min_qubits) {
    relayout_enabled(0);  // defaults first
    if (mode >= 0) g_relayout.store(mode);
    if (min_qubits >= 0) g_relayout_min.store(min_qubits);
}

namespace {
// One relayout choice from a closed tile sequence T: runs, layouts, the plan.
bool build_choice(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                  const std::vector<Op>& logical, const Search& S, const std::vector<uint64_t>& T,
                  size_t max_passes, RelayoutChoice& out, unsigned seed = 0) {
    const size_t K = T.size();
    if (K < 2 || K >= max_passes) return false;
    // gates of every pass
    std::vector<std::vector<int>> ran(K);
    {
        std::vector<int> rem(logical.size());
        for (size_t i = 0; i < rem.size(); ++i) rem[i] = (int)i;
        for (size_t k = 0; k < K; ++k) rem = S.apply(rem, T[k], &ran[k]);
        if (!rem.empty()) return false;
    }
    // runs: R[k] (loaded by pass k) from T[k-1] & T[k], R[0] from T[K-1] & T[0]
    std::vector<uint64_t> R(K);
    for (size_t k = 0; k < K; ++k) {
        const size_t pk = (k + K - 1) % K;
        int uses[64] = {0};
        for (size_t j : {pk, k})
            for (int i : ran[j]) ++uses[logical[i].t0];
        R[k] = choose_run(T[pk] & T[k], uses);
        if (__builtin_popcountll(R[k]) != kRun) return false;
    }
    // layouts: L[k] is loaded by pass k and stored by pass k-1 (L[0] also by the last pass)
    std::vector<std::vector<int>> L(K + 1);
    for (size_t k = 0; k < K; ++k) L[k] = assign_layout(n, R[k], T[(k + K - 1) % K], T[k], seed);
    L[K] = L[0];
    out.perm = L[0];
    out.ops = lower(out.perm);
    if (out.ops.size() != logical.size()) return false;
    std::vector<int> inv0(n);
    for (int q = 0; q < n; ++q) inv0[L[0][q]] = q;
    Plan plan;
    double cost = 0.0;
    for (size_t k = 0; k < K; ++k) {
        const std::vector<int>& ld = L[k];
        const std::vector<int>& sl = L[k + 1];
        std::vector<int> tq, nt;  // tile / non-tile logical qubits by load position
        std::vector<int> by_pos(n);
        for (int q = 0; q < n; ++q) by_pos[ld[q]] = q;
        for (int p = 0; p < n; ++p) ((T[k] >> by_pos[p]) & 1ull ? tq : nt).push_back(by_pos[p]);
        if ((int)tq.size() != kTile) return false;
        int r0 = 0;
        while (r0 < kTile && ld[tq[r0]] == r0) ++r0;
        if (r0 < kRun) return false;
        int hpos[kHposMax] = {0}, bit_of[64], st_pos[13] = {0}, st_tid[32] = {0}, phys_of[64] = {0};
        for (int q = 0; q < 64; ++q) bit_of[q] = -1;
        for (int q = 0; q < n; ++q) phys_of[out.perm[q]] = ld[q];  // plan qubit -> load position
        for (int x = r0; x < kTile; ++x) hpos[x - r0] = ld[tq[x]];
        bool moved = false;
        for (int x = 0; x < kTile; ++x) {
            bit_of[out.perm[tq[x]]] = x;  // the ops name plan qubits = positions under L[0]
            st_pos[x] = sl[tq[x]];
            moved = moved || st_pos[x] != ld[tq[x]];
        }
        for (size_t i = 0; i < nt.size(); ++i) {
            st_tid[i] = sl[nt[i]];
            moved = moved || st_tid[i] != ld[nt[i]];
        }
        std::vector<Op> pops;
        for (int i : ran[k]) pops.push_back(out.ops[i]);
        {
            const TileHeightScope scope(6);
            append_tile_pass(plan, pops, n, 6, r0, hpos, bit_of, moved ? st_pos : nullptr, st_tid, phys_of);
        }
        uint64_t mld = 0, mst = 0;
        for (int q : tq) {
            mld |= 1ull << ld[q];
            mst |= 1ull << sl[q];
        }
        cost += 0.5 * (layout_cost_us(mld) + layout_cost_us(mst));
        static const bool dbg = std::getenv("QSIM_RELAYOUT_DEBUG") != nullptr;
        if (dbg) {
            std::fprintf(stderr, "[relayout] pass %zu: %zu gates, r0 %d, load", k, ran[k].size(), r0);
            for (int b = 0; b < n; ++b)
                if ((mld >> b) & 1ull) std::fprintf(stderr, " %d", b);
            std::fprintf(stderr, " | store");
            for (int b = 0; b < n; ++b)
                if ((mst >> b) & 1ull) std::fprintf(stderr, " %d", b);
            std::fprintf(stderr, " | model %.0f / %.0f us\n", layout_cost_us(mld), layout_cost_us(mst));
        }
    }
    out.plan = std::move(plan);
    out.cost_us = cost;
    return true;
}

// Process-wide memo of relayout choices by circuit (its identity-lowered ops): a state reset and
// re-run, or another state running the same circuit, does not search again.
struct RelayoutMemo {
    int n;
    bool ctrl_out;  // planned with tile-constant controls
    size_t max_passes;
    std::vector<unsigned char> key;
    std::vector<RelayoutChoice> v;
    uint64_t used;
};
std::mutex g_rl_mu;
std::vector<RelayoutMemo> g_rl_memo;
uint64_t g_rl_clock = 0;
std::vector<unsigned char> ops_key(const std::vector<Op>& ops) {
    std::vector<unsigned char> k;
    for (const Op& o : ops) {
        const int64_t ints[7] = {o.kind, o.sub, o.t0, o.t1, (int64_t)o.cmask, o.d0_one ? 1 : 0, o.src};
        const unsigned char* a = reinterpret_cast<const unsigned char*>(ints);
        k.insert(k.end(), a, a + sizeof ints);
        const unsigned char* m = reinterpret_cast<const unsigned char*>(o.m);
        k.insert(k.end(), m, m + sizeof o.m);
    }
    return k;
}
}  // namespace

size_t plan_relayout_variants(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                              size_t max_passes, std::vector<RelayoutChoice>& out) {
    out.clear();
    if (n < kTile + kRun || n - kTile > 32) return 0;
    std::vector<int> id(n);
    for (int q = 0; q < n; ++q) id[q] = q;
    const std::vector<Op> logical = lower(id);
    if (logical.empty()) return 0;
    const std::vector<unsigned char> key = ops_key(logical);
    {
        std::lock_guard<std::mutex> l(g_rl_mu);
        for (RelayoutMemo& m : g_rl_memo)
            if (m.n == n && m.ctrl_out == tile_ctrl_out() && m.max_passes == max_passes && m.key == key) {
                m.used = ++g_rl_clock;
                out = m.v;
                return out.size();
            }
    }
    std::vector<uint64_t> qm(logical.size()), nd(logical.size());
    bool fits = true;
    for (size_t i = 0; i < logical.size(); ++i) {
        qm[i] = op_mask(logical[i]);
        nd[i] = op_need(logical[i], tile_ctrl_out());
        fits = fits && __builtin_popcountll(nd[i]) <= kTile - kRun;
    }
    if (fits) {
        const Search S{qm, n, nd};
        static const int width = env_int("QSIM_RELAYOUT_BEAM", 96);
        static const int nvar = std::max(1, env_int("QSIM_RELAYOUT_VARIANTS", 3));
        static const int nlay = std::max(1, env_int("QSIM_RELAYOUT_LAYOUT_VARIANTS", 2));
        const int w = std::max(2, (int)(width * 256.0 / std::max<size_t>(256, logical.size())));
        for (const std::vector<uint64_t>& T : search_tiles(S, logical.size(), w, std::min<size_t>(max_passes, 64), nvar)) {
            for (int ls = 0; ls < nlay; ++ls) {  // layout variants of the sequence (unique first layouts:
                                                 // a memoised choice is found again by it)
                RelayoutChoice rc;
                if (!build_choice(n, lower, logical, S, T, max_passes, rc, (unsigned)ls)) continue;
                bool dup = false;
                for (const RelayoutChoice& o : out) dup = dup || o.perm == rc.perm;
                if (!dup) out.push_back(std::move(rc));
            }
        }
        std::stable_sort(out.begin(), out.end(), [](const RelayoutChoice& x, const RelayoutChoice& y) {
            return x.plan.passes.size() != y.plan.passes.size() ? x.plan.passes.size() < y.plan.passes.size()
                                                                : x.cost_us < y.cost_us;
        });
    }
    std::lock_guard<std::mutex> l(g_rl_mu);
    if (g_rl_memo.size() >= 8)
        g_rl_memo.erase(std::min_element(g_rl_memo.begin(), g_rl_memo.end(),
                                         [](const RelayoutMemo& x, const RelayoutMemo& y) { return x.used < y.used; }));
    g_rl_memo.push_back(RelayoutMemo{n, tile_ctrl_out(), max_passes, key, out, ++g_rl_clock});
    return out.size();
}

bool plan_relayout(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                   size_t max_passes, RelayoutChoice& out) {
    std::vector<RelayoutChoice> v;
    if (!plan_relayout_variants(n, lower, max_passes, v)) return false;
    out = std::move(v.front());
    return true;
}

// One gate-free relayout pass that moves logical qubit q from physical position perm[q] to q
// (the identity-layout restore before index-based readers: one pass instead of a SWAP network of
// several).  Tile: physical 0..5 (the load runs) and the positions of logical 0..5 (the store
// runs), padded; every tile bit and tile-id bit is stored at its logical position.
Plan plan_permutation_pass(int n, const std::vector<int>& perm) {
    if (n < kTile || n - kTile > 32 || (int)perm.size() != n) fail(QSIM_ERR_RUNTIME, "permutation pass out of range");
    std::vector<int> inv(n);
    for (int q = 0; q < n; ++q) inv[perm[q]] = q;
    uint64_t tile = 0;  // physical positions
    for (int q = 0; q < 6; ++q) tile |= (1ull << q) | (1ull << perm[q]);
    for (int p = 6; p < n && __builtin_popcountll(tile) < kTile; ++p) tile |= 1ull << p;
    const int r0 = 6;  // (physical 0..5 are tile positions)
    int hpos[kHposMax] = {0}, bit_of[64], st_pos[13] = {0}, st_tid[32] = {0};
    for (int q = 0; q < 64; ++q) bit_of[q] = -1;
    int x = 0, i = 0;
    for (int p = 0; p < n; ++p) {
        if ((tile >> p) & 1ull) {
            if (x >= r0) hpos[x - r0] = p;
            bit_of[p] = x;
            st_pos[x++] = inv[p];
        } else {
            st_tid[i++] = inv[p];
        }
    }
    Plan plan;
    const TileHeightScope scope(6);
    append_tile_pass(plan, {}, n, 6, r0, hpos, bit_of, st_pos, st_tid);
    return plan;
}

// ---------------------------------------------------------------------------------------
// Host execution of a plan (tests: qsim_plan_exec_host).  Every staged pass is run tile by
// tile exactly as k_fused_staged / the generated kernels address it — first-stage HBM offsets,
// per-stage thread index (zero insertion or the store-ordered tmap), LDS slots through the
// stage layouts' sigma, the store under the pass's (or the next layout's) positions — so the
// planners' index math is pinned on the CPU.  Op arithmetic is the interpreter's (the
// unnormalised H butterfly with the pass scale at the store).
// ---------------------------------------------------------------------------------------
namespace {
using cd = std::complex<double>;

uint32_t ins0h(uint32_t p, int b) {
    const uint32_t lo = p & ((1u << b) - 1u);
    return ((p ^ lo) << 1) | lo;
}

void exec_stage_op(const TileOp& op, cd* v, int R, uint32_t jb) {
    const uint32_t cr = op.cm_reg, ct = op.cm_thr;
    const bool thr_ok = (jb & ct) == ct;
    if (op.kind == K_DIAG) {
        const cd d0(op.m[0], op.m[1]), d1(op.m[2], op.m[3]);
        const bool tbit = ((jb >> op.b0) & 1u) != 0;
        for (int r = 0; r < R; ++r) {
            const bool bit = op.p0 >= 0 ? (((r >> op.p0) & 1) != 0) : tbit;
            const bool ok = (((uint32_t)r & cr) == cr) && thr_ok && (bit || !op.d0_one);
            if (!ok) continue;
            if (op.sub == S_NEG) v[r] = -v[r];
            else v[r] = (bit ? d1 : d0) * v[r];
        }
        return;
    }
    if (op.p0 < 0) fail(QSIM_ERR_RUNTIME, "stage op target is not a register bit");
    const int P = op.p0;
    const cd m0(op.m[0], op.m[1]), m1(op.m[2], op.m[3]), m2(op.m[4], op.m[5]), m3(op.m[6], op.m[7]);
    for (int r = 0; r < R; ++r) {
        if (r & (1 << P)) continue;
        const bool ok = (((uint32_t)r & cr) == cr) && thr_ok;
        if (!ok) continue;
        const cd a0 = v[r], a1 = v[r | (1 << P)];
        cd x0, x1;
        if (op.sub == S_X) {
            x0 = a1;
            x1 = a0;
        } else if (op.sub == S_H) {
            x0 = a0 + a1;
            x1 = a0 - a1;
        } else {
            x0 = m0 * a0 + m1 * a1;
            x1 = m2 * a0 + m3 * a1;
        }
        v[r] = x0;
        v[r | (1 << P)] = x1;
    }
}

void exec_plan_host(const Plan& plan, int n, std::vector<cd>& st) {
    for (const FusedPass& p : plan.passes) {
        if (p.single >= 0 || p.h < 4) fail(QSIM_ERR_RUNTIME, "host execution covers staged passes only");
        const int tb = 6 + p.h, RB = p.rb, R = 1 << RB, nthr = (1 << tb) >> RB;
        const int r0 = p.r0, nh = tb - r0, lt = n - tb;
        const double scale = std::ldexp(1.0, -(p.hu_count / 2)) * ((p.hu_count & 1) ? kInvSqrt2 : 1.0);
        std::vector<cd> lds(1u << tb), v((size_t)nthr * R);
        std::vector<cd> out = p.relayout ? std::vector<cd>(st.size()) : std::vector<cd>();
        std::vector<cd>& dst = p.relayout ? out : st;
        for (uint64_t tile = 0; tile < (1ull << lt); ++tile) {
            uint64_t kt = tile << r0;
            for (int i = 0; i < nh; ++i) {
                const uint64_t lo = kt & ((1ull << p.hpos[i]) - 1ull);
                kt = ((kt ^ lo) << 1) | lo;
            }
            uint64_t base_st = 0;
            if (p.relayout) {  // (as the kernels: the non-tile load positions' bits, moved)
                uint64_t hm = 0;
                for (int i = 0; i < nh; ++i) hm |= 1ull << p.hpos[i];
                for (int q = r0, i = 0; q < n && i < p.n_tid; ++q)
                    if (!((hm >> q) & 1ull)) base_st |= ((kt >> q) & 1ull) << p.st_tid[i++];
            }
            for (int s = p.stage_begin; s < p.stage_end; ++s) {
                const Stage& sg = plan.stages[s];
                const bool first = s == p.stage_begin, last = s == p.stage_end - 1;
                std::vector<uint32_t> jbs(nthr);
                for (int t = 0; t < nthr; ++t) {
                    uint32_t jb = 0;
                    if (sg.tscatter) {
                        for (int i = 0; i < tb - RB; ++i) jb |= (uint32_t)((t >> i) & 1) << sg.tmap[i];
                    } else {
                        jb = (uint32_t)t;
                        for (int i = 0; i < RB; ++i) jb = ins0h(jb, sg.fix[i]);
                    }
                    jbs[t] = jb;
                    cd* vt = &v[(size_t)t * R];
                    if (first) {
                        uint64_t g = kt | (jb & ((1u << r0) - 1u));
                        for (int i = 0; i < nh; ++i) g |= (uint64_t)((jb >> (r0 + i)) & 1u) << p.hpos[i];
                        for (int r = 0; r < R; ++r) vt[r] = st[g | sg.goff[r]];
                    } else {
                        const uint32_t lb = 16u * lds_sigma(jb, sg.trow_in);
                        for (int r = 0; r < R; ++r) vt[r] = lds[(lb ^ sg.lds[r]) / 16u];
                    }
                }
                for (int t = 0; t < nthr; ++t)
                    for (int o = sg.op_begin; o < sg.op_end; ++o) {
                        const TileOp& op = plan.ops[o];
                        if ((kt & op.cm_out) != op.cm_out) continue;  // tile-constant control reads 0
                        exec_stage_op(op, &v[(size_t)t * R], R, jbs[t]);
                    }
                for (int t = 0; t < nthr; ++t) {
                    const uint32_t jb = jbs[t];
                    const cd* vt = &v[(size_t)t * R];
                    if (last) {
                        uint64_t g;
                        if (p.relayout) {
                            g = base_st;
                            for (int x = 0; x < tb; ++x) g |= (uint64_t)((jb >> x) & 1u) << p.st_pos[x];
                        } else {
                            g = kt | (jb & ((1u << r0) - 1u));
                            for (int i = 0; i < nh; ++i) g |= (uint64_t)((jb >> (r0 + i)) & 1u) << p.hpos[i];
                        }
                        for (int r = 0; r < R; ++r) dst[g | sg.goff[r]] = vt[r] * scale;
                    } else {
                        const uint32_t lbw = 16u * lds_sigma(jb, sg.trow_out);
                        for (int r = 0; r < R; ++r) lds[(lbw ^ sg.lds_w[r]) / 16u] = vt[r];
                    }
                }
            }
        }
        if (p.relayout) st.swap(out);
    }
}
}  // namespace

}  // namespace qsim_hip

extern "C" int qsim_plan_exec_host(int n_qubits, const qsim_gate* gates, size_t count, int mode, double* amps,
                                   int32_t* perm, int* passes) {
    using namespace qsim_hip;
    try {
        if (n_qubits < 10 || n_qubits > 26) fail(QSIM_ERR_INVALID_ARGUMENT, "host execution: 10..26 qubits");
        if (!amps || (!gates && count)) fail(QSIM_ERR_INVALID_ARGUMENT, "null argument");
        const int n = n_qubits;
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], n);
        auto lower = [&](const std::vector<int>& pi) {
            std::vector<Op> ops;
            for (size_t i = 0; i < count; ++i) {
                qsim_gate m = gates[i];
                for (int j = 0; j < m.nqubits && j < 3; ++j) m.qubits[j] = pi[m.qubits[j]];
                ops.push_back(lower_gate(m, n));
                ops.back().src = (int)i;
            }
            return ops;
        };
        std::vector<int> pi(n);
        for (int q = 0; q < n; ++q) pi[q] = q;
        Plan plan;
        if (mode == 2) {  // the one-pass identity restore from layout `perm` (amps: physical order)
            if (!perm) fail(QSIM_ERR_INVALID_ARGUMENT, "null perm");
            std::vector<int> from(perm, perm + n), chk(from);
            std::sort(chk.begin(), chk.end());
            for (int q = 0; q < n; ++q)
                if (chk[q] != q) fail(QSIM_ERR_INVALID_ARGUMENT, "perm is not a permutation");
            plan = plan_permutation_pass(n, from);
            const uint64_t N = 1ull << n;
            std::vector<std::complex<double>> st(N);
            for (uint64_t i = 0; i < N; ++i) st[i] = std::complex<double>(amps[2 * i], amps[2 * i + 1]);
            exec_plan_host(plan, n, st);
            for (uint64_t i = 0; i < N; ++i) {
                amps[2 * i] = st[i].real();
                amps[2 * i + 1] = st[i].imag();
            }
            if (passes) *passes = (int)plan.passes.size();
            return QSIM_OK;
        }
        if (mode == 1) {
            RelayoutChoice rc;
            if (!plan_relayout(n, lower, SIZE_MAX, rc)) fail(QSIM_ERR_RUNTIME, "no relayout plan");
            pi = rc.perm;
            plan = std::move(rc.plan);
        } else {
            const TileHeightScope scope(6);
            plan = plan_fused(lower(pi), n, 6);
        }
        const uint64_t N = 1ull << n;
        std::vector<std::complex<double>> st(N);
        for (uint64_t i = 0; i < N; ++i) {  // logical index -> physical under pi
            uint64_t k = 0;
            for (int q = 0; q < n; ++q)
                if ((i >> q) & 1ull) k |= 1ull << pi[q];
            st[k] = std::complex<double>(amps[2 * i], amps[2 * i + 1]);
        }
        exec_plan_host(plan, n, st);
        for (uint64_t i = 0; i < N; ++i) {
            uint64_t k = 0;
            for (int q = 0; q < n; ++q)
                if ((i >> q) & 1ull) k |= 1ull << pi[q];
            amps[2 * i] = st[k].real();
            amps[2 * i + 1] = st[k].imag();
        }
        if (perm)
            for (int q = 0; q < n; ++q) perm[q] = pi[q];
        if (passes) *passes = (int)plan.passes.size();
        return QSIM_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return QSIM_ERR_RUNTIME;
    }
}

extern "C" int qsim_plan_relayout(int n_qubits, const qsim_gate* gates, size_t count, int32_t* perm, int* passes,
                                  double* predicted_us) {
    using namespace qsim_hip;
    try {
        if (n_qubits < 1 || n_qubits > 40) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        if (!gates && count) fail(QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        const int n = n_qubits;
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], n);
        auto lower = [&](const std::vector<int>& pi) {
            std::vector<Op> ops;
            for (size_t i = 0; i < count; ++i) {
                qsim_gate m = gates[i];
                for (int j = 0; j < m.nqubits && j < 3; ++j) m.qubits[j] = pi[m.qubits[j]];
                ops.push_back(lower_gate(m, n));
                ops.back().src = (int)i;
            }
            return ops;
        };
        RelayoutChoice rc;
        const bool ok = plan_relayout(n, lower, SIZE_MAX, rc);
        if (passes) *passes = ok ? (int)rc.plan.passes.size() : 0;
        if (predicted_us) *predicted_us = ok ? rc.cost_us : 0.0;
        if (perm)
            for (int q = 0; q < n; ++q) perm[q] = ok ? rc.perm[q] : q;
        return QSIM_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return QSIM_ERR_RUNTIME;
    }
}

extern "C" int qsim_set_relayout(int mode, int min_qubits) {
    qsim_hip::relayout_configure(mode, min_qubits);
    return QSIM_OK;
}
