// fused.hip — LDS-tiled multi-gate passes (the gates/s lever) and their host planner.
//
// The reference applies one kernel per gate (src/Simulator.cu:28-154), so every gate is a full
// HBM round trip of the state.  Here a pass streams the state once: each 256-thread workgroup
// owns a tile of 64 << h amplitudes spanning qubits {0..5} (the 64 lanes, 1 KiB contiguous
// runs) plus h chosen high qubits, stages it in LDS (64 KiB at h = 6, two workgroups per CU),
// applies every planned gate whose qubits lie inside the tile, and writes it back.  HBM traffic
// per pass is 32 B x 2^n, independent of how many gates the pass absorbs.
//
// Inside a pass the gates are grouped into register stages (h >= 4): each thread pulls the
// 2^(h-2) amplitudes spanned by the stage's target bits from LDS into registers, applies every
// gate of the stage there (diagonal gates need no target bit at all), and writes them back — one
// LDS round trip and one barrier per stage instead of per gate.
//
// Planner rule (both levels): a gate moves into the current pass/stage when its qubits fit and
// it shares no qubit with an earlier gate that was deferred (gates on disjoint qubits commute
// exactly).  Gate semantics are the per-gate kernels' (device_ops.hpp), i.e. src/Gates.cu.
#include <atomic>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>

#include "device_ops.hpp"
#include "engine.hpp"

namespace qsim_hip {

static inline uint32_t ins0_host(uint32_t p, int b) {
    const uint32_t lo = p & ((1u << b) - 1u);
    return ((p ^ lo) << 1) | lo;
}


// ---------------------------------------------------------------------------------------
// Host planner
// ---------------------------------------------------------------------------------------
static uint64_t op_qubits(const Op& op) {
    uint64_t m = op.cmask | (1ull << op.t0);
    if (op.kind == K_SWAP) m |= 1ull << op.t1;
    return m;
}
// The qubits a tile must hold for `op` (its targets with tile-constant controls, else all).
static uint64_t op_need(const Op& op, bool ctrl_out) {
    if (!ctrl_out) return op_qubits(op);
    uint64_t m = 1ull << op.t0;
    if (op.kind == K_SWAP) m |= 1ull << op.t1;
    return m;
}

static TileOp make_tile_op(int kind, int sub, int b0, int b1, uint32_t cm, int d0_one,
                           const double* m) {
    TileOp t{};
    t.kind = kind;
    t.sub = sub;
    t.b0 = b0;
    t.b1 = b1;
    t.cmask = cm;
    t.d0_one = d0_one;
    t.p0 = -1;
    for (int i = 0; i < 8; ++i) t.m[i] = m ? m[i] : 0.0;
    return t;
}

static constexpr int kMaxUnnormH = 512;

// Extra LDS cycles (bank conflicts) of one wave's 16 register accesses with stage register bits
// `sbits` (lanes = the stage's thread bits: tid spread over the other tile bits) under layout
// `trow`: ds_write_b128 banks by slot mod 8 in 8 groups of 8 contiguous lanes, ds_read_b128 by
// slot mod 16 in 4 groups of 16 lanes (MI355X_MICROARCH.md §LDS).
// tmap (null: ascending) orders the lanes over the non-register tile bits (Stage::tmap).
static int lds_conflicts(uint32_t sbits, const uint32_t* trow, bool write, int tile_bits,
                         const int* tmap = nullptr) {
    static const int kReadGroups[4][16] = {
        {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
        {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
        {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
        {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    int fix[4], nf = 0;
    for (int b = 0; b < tile_bits && nf < 4; ++b)
        if ((sbits >> b) & 1u) fix[nf++] = b;
    uint32_t lane_j[64];
    for (int l = 0; l < 64; ++l) {
        uint32_t j = (uint32_t)l;
        if (tmap) {
            j = 0;
            for (int i = 0; i < 6; ++i) j |= (uint32_t)((l >> i) & 1) << tmap[i];
        } else {
            for (int i = 0; i < nf; ++i) j = ins0_host(j, fix[i]);
        }
        lane_j[l] = j;
    }
    int extra = 0;
    for (int r = 0; r < (1 << nf); ++r) {
        uint32_t o = 0;
        for (int i = 0; i < nf; ++i)
            if ((r >> i) & 1) o |= 1u << fix[i];
        uint32_t addr[64];
        for (int l = 0; l < 64; ++l) addr[l] = lds_sigma(lane_j[l] | o, trow);
        const int groups = write ? 8 : 4, per = write ? 8 : 16, mod = write ? 8 : 16;
        for (int g = 0; g < groups; ++g) {
            uint32_t seen[16][16];
            int cnt[16] = {0}, worst = 1;
            for (int k = 0; k < per; ++k) {
                const int l = write ? g * 8 + k : kReadGroups[g][k];
                const uint32_t slot = addr[l] % (uint32_t)mod;
                bool dup = false;
                for (int t = 0; t < cnt[slot]; ++t) dup |= seen[slot][t] == addr[l];
                if (!dup) seen[slot][cnt[slot]++] = addr[l];
                worst = std::max(worst, cnt[slot]);
            }
            extra += worst - 1;
        }
    }
    return extra;
}

// A layout for the LDS round trip between a stage with register bits `wbits` (writes) and one
// with `rbits` (reads): the fixed j ^ ((j >> 4) & 15) when it is conflict-free, else the best
// triangular swizzle found by a deterministic random search with local moves.
static std::array<uint32_t, 4> choose_swizzle(uint32_t wbits, uint32_t rbits, int tile_bits,
                                              const int* rtmap = nullptr) {
    std::array<uint32_t, 4> best = {0x10u, 0x20u, 0x40u, 0x80u};
    const uint32_t all = (1u << tile_bits) - 1u;
    auto cost = [&](const std::array<uint32_t, 4>& t) {
        return lds_conflicts(wbits, t.data(), true, tile_bits) +
               lds_conflicts(rbits, t.data(), false, tile_bits, rtmap);
    };
    int bc = cost(best);
    uint64_t rng = 0x9e3779b97f4a7c15ull ^ ((uint64_t)wbits << 20) ^ rbits;
    auto next = [&]() {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    for (int it = 0; it < 4000 && bc > 0; ++it) {
        std::array<uint32_t, 4> c = best;
        if (it < 2000) {
            for (int i = 0; i < 4; ++i) c[i] = (uint32_t)next() & all & ~((2u << i) - 1u);
        } else {
            const int i = (int)(next() % 4);
            const int b = i + 1 + (int)(next() % (uint64_t)(tile_bits - i - 1));
            c[i] ^= 1u << b;
        }
        const int cc = cost(c);
        if (cc < bc) {
            bc = cc;
            best = c;
        }
    }
    return best;
}

// Group one pass's ops (tile bits) into register stages of at most `rb` target bits.
// st_pos (relayout passes, else null): store position of every tile bit; the last stage's lanes
// are then the six tile bits with the lowest store positions (its register bits avoid them) and
// its HBM offsets are store positions — a relayout pass always has an LDS round trip before it.
static void plan_stages(std::vector<TileOp>& pass_ops, std::vector<int>& pass_src, int tile_bits,
                        int rb, Plan& plan, FusedPass& p, const int* st_pos = nullptr) {
    // SWAP -> three controlled-X on the register bits (exact data movement).
    std::vector<TileOp> ops;
    std::vector<int> src;
    static const double xm[8] = {0, 0, 1, 0, 1, 0, 0, 0};
    for (size_t i = 0; i < pass_ops.size(); ++i) {
        const TileOp& t = pass_ops[i];
        if (t.kind == K_SWAP) {
            const uint32_t a = 1u << t.b0, b = 1u << t.b1;
            ops.push_back(make_tile_op(K_M1, S_X, t.b1, -1, t.cmask | a, 0, xm));
            ops.push_back(make_tile_op(K_M1, S_X, t.b0, -1, t.cmask | b, 0, xm));
            ops.push_back(make_tile_op(K_M1, S_X, t.b1, -1, t.cmask | a, 0, xm));
            for (int k = 1; k <= 3; ++k) {
                ops[ops.size() - k].step = t.step;
                ops[ops.size() - k].cm_out = t.cm_out;
            }
            src.push_back(pass_src[i]);  // the gate is reported once (introspection skips -1)
            src.push_back(-1);
            src.push_back(-1);
        } else {
            ops.push_back(t);
            src.push_back(pass_src[i]);
        }
    }
    p.stage_begin = (int)plan.stages.size();
    p.hu_count = 0;
    for (TileOp& t : ops) {
        if (t.kind == K_M1 && t.sub == S_H) {
            // unnormalized butterfly in the staged kernel: each one scales the tile's 2-norm by
            // exactly sqrt2, so at most kMaxUnnormH per pass bounds the growth to 2^(kMaxUnnormH/2)
            // (no overflow for any state of norm < 2^700); further H run as the normalised matrix
            if (t.cmask == 0 && t.cm_out == 0 && p.hu_count < kMaxUnnormH) ++p.hu_count;
            else t.sub = S_GEN;  // (also controlled H, not in the gate set; keep it exact)
        }
    }
    // The first stage is applied in registers straight after the HBM load and the last one
    // right before the HBM store, so both may only use high tile bits (>= 6) as register bits:
    // the 64 lanes must keep the 64 consecutive amplitudes of tile bits 0..5 (1 KiB runs).
    const uint32_t all_bits = (1u << tile_bits) - 1u, high_bits = all_bits & ~0x3fu;
    struct Taken {
        std::vector<int> in, deferred;
        uint32_t sbits = 0;
    };
    auto take = [&](const std::vector<int>& from, uint32_t allowed) {
        Taken t;
        uint32_t blocked = 0;
        for (int i : from) {
            const TileOp& o = ops[i];
            const uint32_t need = o.kind == K_M1 ? (1u << o.b0) : 0u;
            const uint32_t touch = o.cmask | (1u << o.b0);
            if ((touch & blocked) == 0 && (need & ~allowed) == 0 &&
                __builtin_popcount(t.sbits | need) <= rb) {
                t.sbits |= need;
                t.in.push_back(i);
            } else {
                t.deferred.push_back(i);
                blocked |= touch;
            }
        }
        return t;
    };
    // Fill a stage's free register bits: first with the stage ops' control bits, most used first
    // (a control on a register bit is resolved per register pair — a rename or a skipped pair —
    // instead of a per-lane select), then with the highest unused allowed bits (threads then walk
    // consecutive LDS slots).
    auto pad = [&](uint32_t sbits, uint32_t allowed, const std::vector<int>& in) {
        int cnt[32] = {0};
        for (int i : in)
            for (int b = 0; b < tile_bits; ++b)
                if ((ops[i].cmask >> b) & 1u) ++cnt[b];
        while (__builtin_popcount(sbits) < rb) {
            int best = -1;
            for (int b = 0; b < tile_bits; ++b)
                if (((allowed & ~sbits) >> b) & 1u && cnt[b] > 0 && (best < 0 || cnt[b] > cnt[best]))
                    best = b;
            if (best < 0) break;
            sbits |= 1u << best;
        }
        for (int b = tile_bits - 1; b >= 0 && __builtin_popcount(sbits) < rb; --b)
            if ((allowed >> b) & 1u) sbits |= 1u << b;
        return sbits;
    };
    // The ops an in-order scan takes with register bits fixed to S (an op is taken when its target
    // bit is in S and no earlier deferred op touches its bits; diagonal ops need no register bit).
    auto take_fixed = [&](const std::vector<int>& from, uint32_t S) {
        Taken t;
        uint32_t blocked = 0;
        for (int i : from) {
            const TileOp& o = ops[i];
            const uint32_t need = o.kind == K_M1 ? (1u << o.b0) : 0u;
            const uint32_t touch = o.cmask | (1u << o.b0);
            if ((touch & blocked) == 0 && (need & ~S) == 0) {
                t.sbits |= need;
                t.in.push_back(i);
            } else {
                t.deferred.push_back(i);
                blocked |= touch;
            }
        }
        return t;
    };
    // One stage: the first-fit scan (register bits claimed in program order), or — when it takes
    // more ops — register bits grown greedily from the best PAIR of allowed bits, one bit at a time,
    // each time the bit that lets the scan take the most ops (QSIM_STAGE_SEARCH=0: first fit
    // only).  Fewer LDS round trips per pass: the density-matrix passes spend their time in their
    // stages, W-HC 14q DM 39-47 stages per 6-pass plan with first fit.
    static const bool search = [] {
        const char* e = std::getenv("QSIM_STAGE_SEARCH");
        return e == nullptr || std::atoi(e) != 0;
    }();
    auto stage = [&](const std::vector<int>& from, uint32_t allowed) {
        Taken ff = take(from, allowed);
        if (!search || ff.deferred.empty() || rb < 2) return ff;
        std::vector<int> bits;
        for (int b = 0; b < tile_bits; ++b)
            if ((allowed >> b) & 1u) bits.push_back(b);
        uint32_t S = 0;
        size_t got = 0;
        for (size_t i = 0; i < bits.size(); ++i)
            for (size_t j = i + 1; j < bits.size(); ++j) {
                const uint32_t s2 = (1u << bits[i]) | (1u << bits[j]);
                const size_t c = take_fixed(from, s2).in.size();
                if (c > got) {
                    got = c;
                    S = s2;
                }
            }
        while (__builtin_popcount(S) < rb) {
            int bb = -1;
            for (int b : bits) {
                if ((S >> b) & 1u) continue;
                const size_t c = take_fixed(from, S | (1u << b)).in.size();
                if (c > got) {
                    got = c;
                    bb = b;
                }
            }
            if (bb < 0) break;
            S |= 1u << bb;
        }
        if (got <= ff.in.size()) return ff;
        return take_fixed(from, S);
    };
    // Candidate register-bit sets of one stage for the beam below: first fit, and the best few
    // pairs of allowed bits each grown greedily to rb bits.
    auto stage_cands = [&](const std::vector<int>& from, uint32_t allowed) {
        std::vector<Taken> out;
        out.push_back(take(from, allowed));
        if (out[0].deferred.empty() || rb < 2) return out;
        std::vector<int> bits;
        for (int b = 0; b < tile_bits; ++b)
            if ((allowed >> b) & 1u) bits.push_back(b);
        std::vector<std::pair<size_t, uint32_t>> pairs;
        for (size_t i = 0; i < bits.size(); ++i)
            for (size_t j = i + 1; j < bits.size(); ++j) {
                const uint32_t s2 = (1u << bits[i]) | (1u << bits[j]);
                pairs.push_back({take_fixed(from, s2).in.size(), s2});
            }
        std::sort(pairs.begin(), pairs.end(), [](const auto& a, const auto& b) {
            return a.first != b.first ? a.first > b.first : a.second < b.second;
        });
        for (size_t k = 0; k < pairs.size() && k < 4; ++k) {
            uint32_t S = pairs[k].second;
            size_t got = pairs[k].first;
            while (__builtin_popcount(S) < rb) {
                int bb = -1;
                for (int b : bits) {
                    if ((S >> b) & 1u) continue;
                    const size_t c = take_fixed(from, S | (1u << b)).in.size();
                    if (c > got) {
                        got = c;
                        bb = b;
                    }
                }
                if (bb < 0) break;
                S |= 1u << bb;
            }
            Taken t = take_fixed(from, S);
            bool dup = false;
            for (const Taken& o : out) dup = dup || o.in == t.in;
            if (!dup) out.push_back(std::move(t));
        }
        return out;
    };
    std::vector<int> rem(ops.size());
    for (size_t i = 0; i < rem.size(); ++i) rem[i] = (int)i;
    std::vector<std::pair<uint32_t, std::vector<int>>> seq;  // (register bits, ops) per stage
    static const int beam_w = [] {  // QSIM_STAGE_BEAM: beam width over stage sequences (0: greedy)
        const char* e = std::getenv("QSIM_STAGE_BEAM");
        return e ? std::max(0, std::atoi(e)) : 0;
    }();
    if (search && beam_w > 0) {
        // Beam over stage sequences: states ranked by the ops still to place (then by stages so
        // far, equal at a level); the first state with none left wins (fewest stages found).
        struct St {
            std::vector<int> rem;
            std::vector<std::pair<uint32_t, std::vector<int>>> seq;
        };
        std::vector<St> beam(1);
        beam[0].rem = rem;
        for (int level = 0; !beam.empty(); ++level) {
            std::vector<St> next;
            for (const St& st : beam)
                for (Taken& t : stage_cands(st.rem, level == 0 ? high_bits : all_bits)) {
                    St ns;
                    ns.seq = st.seq;
                    ns.seq.push_back({level == 0 ? pad(t.sbits, high_bits, t.in) : t.sbits, t.in});
                    ns.rem = std::move(t.deferred);
                    next.push_back(std::move(ns));
                }
            std::stable_sort(next.begin(), next.end(), [](const St& a, const St& b) { return a.rem.size() < b.rem.size(); });
            if (next.empty()) break;
            if (next[0].rem.empty()) {
                seq = std::move(next[0].seq);
                rem.clear();
                break;
            }
            next.resize(std::min<size_t>(next.size(), (size_t)beam_w));
            beam.swap(next);
        }
    } else {
        Taken first = stage(rem, high_bits);
        seq.push_back({pad(first.sbits, high_bits, first.in), first.in});
        rem.swap(first.deferred);
    }
    while (!rem.empty()) {
        Taken t = stage(rem, all_bits);
        seq.push_back({t.sbits, t.in});
        rem.swap(t.deferred);
    }
    // tile bits by store position (relayout): the first six are the store's lanes
    int st_order[32];
    uint32_t st_high = high_bits;
    if (st_pos) {
        for (int b = 0; b < tile_bits; ++b) st_order[b] = b;
        std::sort(st_order, st_order + tile_bits, [&](int a, int b) { return st_pos[a] < st_pos[b]; });
        st_high = all_bits;
        for (int i = 0; i < 6; ++i) st_high &= ~(1u << st_order[i]);
    }
    if (st_pos && seq.size() == 1) {
        seq.push_back({pad(0u, st_high, {}), {}});
    } else if (seq.size() > 1) {  // the last stage must be storable straight from registers
        if ((seq.back().first & ~st_high) == 0)
            seq.back().first = pad(seq.back().first, st_high, seq.back().second);
        else
            seq.push_back({pad(0u, st_high, {}), {}});
    }
    // thread-bit -> tile-bit map of every stage (ascending non-register bits; the relayout
    // pass's last stage in store-position order)
    std::vector<std::array<int, 10>> tmaps(seq.size());
    for (size_t si = 0; si < seq.size(); ++si) {
        int k = 0;
        const bool sorted = st_pos && si + 1 == seq.size();
        for (int i = 0; i < tile_bits; ++i) {
            const int b = sorted ? st_order[i] : i;
            if (!((seq[si].first >> b) & 1u) && k < 10) tmaps[si][k++] = b;
        }
        for (; k < 10; ++k) tmaps[si][k] = 0;
    }
    for (size_t k = 1; k + 1 < seq.size(); ++k) seq[k].first = pad(seq[k].first, all_bits, seq[k].second);
    // LDS layouts of the transitions: transition k sits between stage k's writes and stage k+1's
    // reads; each gets a conflict-free swizzle (choose_swizzle)
    std::vector<std::array<uint32_t, 4>> layout(seq.size());
    for (size_t k = 0; k + 1 < seq.size(); ++k)
        layout[k] = choose_swizzle(seq[k].first, seq[k + 1].first, tile_bits,
                                   st_pos && k + 2 == seq.size() ? tmaps[k + 1].data() : nullptr);
    for (size_t si = 0; si < seq.size(); ++si) {
        auto& sq = seq[si];
        const uint32_t sbits = sq.first;
        const std::vector<int>& in = sq.second;
        Stage st{};
        static const std::array<uint32_t, 4> kDefault = {0x10u, 0x20u, 0x40u, 0x80u};
        const std::array<uint32_t, 4>& tin = si > 0 ? layout[si - 1] : kDefault;
        const std::array<uint32_t, 4>& tout = si + 1 < seq.size() ? layout[si] : kDefault;
        for (int i = 0; i < 4; ++i) {
            st.trow_in[i] = tin[i];
            st.trow_out[i] = tout[i];
        }
        int k = 0;
        int pos_of[32];
        for (int b = 0; b < tile_bits; ++b)
            if ((sbits >> b) & 1u) {
                st.fix[k] = b;
                pos_of[b] = k;
                ++k;
            }
        const bool store_map = st_pos && si + 1 == seq.size();
        for (int i = 0; i < 10; ++i) st.tmap[i] = tmaps[si][i];
        st.tscatter = store_map ? 1 : 0;
        for (int r = 0; r < (1 << rb); ++r) {
            uint32_t o = 0;
            for (int i = 0; i < rb; ++i)
                if ((r >> i) & 1) o |= 1u << st.fix[i];
            uint64_t g = 0;
            for (int b = 0; b < tile_bits; ++b)
                if ((o >> b) & 1u) g |= 1ull << (store_map ? st_pos[b] : b < p.r0 ? b : p.hpos[b - p.r0]);
            st.goff[r] = g;
            st.lds[r] = 16u * lds_sigma(o, st.trow_in);
            st.lds_w[r] = 16u * lds_sigma(o, st.trow_out);
        }
        st.op_begin = (int)plan.ops.size();
        for (int i : in) {
            TileOp t = ops[i];
            t.p0 = ((sbits >> t.b0) & 1u) ? pos_of[t.b0] : -1;  // M1 targets are always stage bits
            t.cm_reg = 0;
            for (int b = 0; b < tile_bits; ++b)
                if (((t.cmask & sbits) >> b) & 1u) t.cm_reg |= 1u << pos_of[b];
            t.cm_thr = t.cmask & ~sbits;
            auto qubit_of = [&](int b) { return b < p.r0 ? b : p.hpos[b - p.r0]; };
            t.tq = qubit_of(t.b0);
            int nc = 0;
            for (int b = 0; b < tile_bits; ++b) {
                if (!((t.cmask >> b) & 1u)) continue;
                if (nc == 2) fail(QSIM_ERR_RUNTIME, "tile op with more than two controls");
                t.cq[nc] = qubit_of(b);
                t.cb[nc] = b;
                t.cpos[nc] = ((sbits >> b) & 1u) ? pos_of[b] : -1;
                ++nc;
            }
            for (; nc < 2; ++nc) t.cq[nc] = t.cb[nc] = t.cpos[nc] = -1;
            plan.ops.push_back(t);
            plan.order.push_back(src[i]);
        }
        st.op_end = (int)plan.ops.size();
        plan.stages.push_back(st);
    }
    p.stage_end = (int)plan.stages.size();
}

// One planned step: a tile pass (chosen qubits `hi` above the run, ops in execution order) or a
// per-gate step for a gate wider than the tile.
struct PassChoice {
    bool single = false;
    int r0 = 6;         // run width of this pass
    uint64_t hi = 0;
    std::vector<Op> ops;
};

// Split `ops` into passes.  Both strategies keep the exact-reordering rule (a gate may move
// ahead only of gates on disjoint qubits).
//   greedy: first fit in program order — a gate joins when its qubits still fit the tile.
//   lookahead: grow the tile's qubit set one qubit (or, when no single qubit helps, one pair) at
//     a time, each time taking the choice that lets the most upcoming gates into the pass.
// avoid: qubits a tile should contain only when that lets more gates in (ties go to others).
static std::vector<PassChoice> choose_passes(const std::vector<Op>& ops, int n, int r0, int nfree,
                                             bool lookahead, uint64_t avoid_all, uint64_t avoid_first = 0) {
    const uint64_t low = (1ull << r0) - 1ull;
    const bool co = tile_ctrl_out() && nfree + r0 >= 10;  // (staged tiles only)
    std::vector<PassChoice> out;
    std::vector<Op> rem = ops;
    std::vector<uint64_t> qm, nm;
    const size_t window = 512;  // gates scored per candidate (later ones are almost always blocked)
    auto score = [&](uint64_t allowed) {
        uint64_t blocked = 0;
        int c = 0;
        const size_t m = std::min(qm.size(), window);
        for (size_t i = 0; i < m; ++i) {
            if ((qm[i] & blocked) == 0 && (nm[i] & ~allowed) == 0) ++c;
            else blocked |= qm[i];
        }
        return c;
    };
    while (!rem.empty()) {
        // The first remaining gate is never blocked; if it needs more qubits than the tile's free
        // slots it runs as a per-gate step (keeps program order, guarantees progress).
        if (__builtin_popcountll(op_need(rem.front(), co) & ~low) > nfree) {
            PassChoice c;
            c.single = true;
            c.ops.push_back(rem.front());
            out.push_back(std::move(c));
            rem.erase(rem.begin());
            continue;
        }
        uint64_t hi = 0;
        const uint64_t avoid = avoid_all | (out.empty() ? avoid_first : 0ull);
        if (lookahead) {
            qm.resize(rem.size());
            nm.resize(rem.size());
            for (size_t i = 0; i < rem.size(); ++i) {
                qm[i] = op_qubits(rem[i]);
                nm[i] = op_need(rem[i], co);
            }
            while (__builtin_popcountll(hi) < nfree) {
                const int base = score(low | hi);
                int best = 2 * base + 1, bq = -1;  // key 2 * score + (not avoided)
                for (int q = r0; q < n; ++q) {
                    if ((hi >> q) & 1ull) continue;
                    const int c = 2 * score(low | hi | (1ull << q)) + (((avoid >> q) & 1ull) ? 0 : 1);
                    if (c > best) best = c, bq = q;
                }
                if (bq >= 0) {
                    hi |= 1ull << bq;
                    continue;
                }
                if (__builtin_popcountll(hi) + 2 > nfree) break;
                int pa = -1, pb = -1;
                best = base;
                for (int qa = r0; qa < n; ++qa) {
                    if ((hi >> qa) & 1ull) continue;
                    for (int qb = qa + 1; qb < n; ++qb) {
                        if ((hi >> qb) & 1ull) continue;
                        const int c = score(low | hi | (1ull << qa) | (1ull << qb));
                        if (c > best) best = c, pa = qa, pb = qb;
                    }
                }
                if (pa < 0) break;
                hi |= (1ull << pa) | (1ull << pb);
            }
            if (score(low | hi) == 0) hi = op_need(rem.front(), co) & ~low;  // (3-qubit first gate)
        }
        PassChoice c;
        uint64_t blocked = 0;
        std::vector<Op> deferred;
        for (const Op& op : rem) {
            const uint64_t q = op_qubits(op), qh = op_need(op, co) & ~low;
            const bool fits = lookahead ? (qh & ~hi) == 0 : __builtin_popcountll(hi | qh) <= nfree;
            if ((q & blocked) == 0 && fits) {
                if (!lookahead) hi |= qh;
                c.ops.push_back(op);
            } else {
                deferred.push_back(op);
                blocked |= q;
            }
        }
        c.hi = hi;
        out.push_back(std::move(c));
        rem.swap(deferred);
    }
    return out;
}

// Beam search over pass sequences (n >= QSIM_PLAN_BEAM_MIN_QUBITS, staged tiles).  A search
// state is the list of gates not yet run; a step is one tile pass, described by its run width r0
// (4..6, chosen per pass) and its 12 - r0 free tile qubits.  Each state proposes its best
// `width` tiles per r0 — grown one qubit at a time from the first remaining gate's qubits, keeping
// the `width` best partial sets, scored by the gates the tile admits (then by the gates it
// partly covers, so a 2-qubit gate's first qubit already counts) — and the `width` states with
// the fewest remaining gates survive each step.  The first state to run out of gates gives the
// plan.  W-HC 30q: 7 passes (one-tile-at-a-time lookahead) -> 5.
static std::vector<PassChoice> beam_passes(const std::vector<Op>& ops, int n, int heff, int width,
                                           uint64_t avoid_all, uint64_t avoid_first = 0) {
    const size_t window = 512;
    const bool co = tile_ctrl_out();
    std::vector<uint64_t> qm(ops.size()), nm(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) {
        qm[i] = op_qubits(ops[i]);
        nm[i] = op_need(ops[i], co);
    }
    auto run_mask = [](int r0) { return (1ull << r0) - 1ull; };
    // (admitted, partly covered) over the first `window` remaining gates
    auto score = [&](const std::vector<int>& rem, uint64_t allowed, uint64_t low) {
        uint64_t blocked = 0;
        int full = 0, part = 0;
        const size_t m = std::min(rem.size(), window);
        for (size_t i = 0; i < m; ++i) {
            const uint64_t q = qm[rem[i]], nd = nm[rem[i]];
            if (q & blocked) {
                blocked |= q;
            } else if ((nd & ~allowed) == 0) {
                ++full;
            } else {
                if (nd & allowed & ~low) ++part;
                blocked |= q;
            }
        }
        return full * 4096 + part;
    };
    auto apply = [&](const std::vector<int>& rem, uint64_t allowed) {
        std::vector<int> out;
        uint64_t blocked = 0;
        for (int i : rem) {
            const uint64_t q = qm[i];
            if ((q & blocked) == 0 && (nm[i] & ~allowed) == 0) continue;
            out.push_back(i);
            blocked |= q;
        }
        return out;
    };
    // HBM cost of a pass layout beyond a 1 KiB-run pass (single-pass probes at 30q,
    // profiles/r01/layout): a wave instruction spans the 2^r0-amplitude run plus the tile bits
    // just above it (the lane bits); 256 B runs cost ~15 %, lane bits at qubit >= 12 (segments
    // >= 64 KiB apart within one instruction) ~30 %.  Ranks plans with equal pass counts.
    auto layout_cost = [](int r0, uint64_t hi) {
        if (r0 >= 6) return 0;
        uint64_t h = hi;
        int lane_hi = 0;
        for (int k = 0; k < 6 - r0 && h; ++k) {
            lane_hi = __builtin_ctzll(h);
            h &= h - 1;
        }
        return (r0 == 5 ? 1 : 2) + (lane_hi >= 12 ? 2 : 0);
    };
    struct St {
        std::vector<int> rem;
        std::vector<std::pair<int, uint64_t>> hist;  // (r0, free tile qubits) per pass
        int cost = 0;
    };
    std::vector<St> states(1);
    states[0].rem.resize(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) states[0].rem[i] = (int)i;
    for (int guard = 0; guard <= (int)ops.size(); ++guard) {
        const St* done = nullptr;
        for (const St& s : states)
            if (s.rem.empty() && (!done || s.cost < done->cost)) done = &s;
        if (done) {
            const St& s = *done;
            {
                std::vector<PassChoice> out;
                std::vector<Op> rest = ops;
                for (const auto& h : s.hist) {
                    PassChoice c;
                    c.r0 = h.first;
                    c.hi = h.second;
                    const uint64_t allowed = run_mask(h.first) | h.second;
                    std::vector<Op> deferred;
                    uint64_t blocked = 0;
                    for (const Op& op : rest) {
                        const uint64_t q = op_qubits(op);
                        if ((q & blocked) == 0 && (op_need(op, co) & ~allowed) == 0) {
                            c.ops.push_back(op);
                        } else {
                            deferred.push_back(op);
                            blocked |= q;
                        }
                    }
                    rest.swap(deferred);
                    out.push_back(std::move(c));
                }
                return out;
            }
        }
        std::vector<St> next;
        std::vector<std::vector<int>> seen;
        for (const St& s : states) {
            const uint64_t avoid = avoid_all | (s.hist.empty() ? avoid_first : 0ull);
            for (int r0 = 6; r0 >= 4; --r0) {
                const uint64_t low = run_mask(r0);
                const int nfree = 6 + heff - r0;
                const uint64_t seed = nm[s.rem.front()] & ~low;
                if (__builtin_popcountll(seed) > nfree) continue;
                std::vector<std::pair<int, uint64_t>> part = {{score(s.rem, low | seed, low), seed}};
                for (int k = __builtin_popcountll(seed); k < nfree; ++k) {
                    std::vector<std::pair<int, uint64_t>> grown;
                    for (const auto& pp : part)
                        for (int q = r0; q < n; ++q) {
                            if ((pp.second >> q) & 1ull) continue;
                            const uint64_t h = pp.second | (1ull << q);
                            bool dup = false;
                            for (const auto& g2 : grown) dup = dup || g2.second == h;
                            // key 2 * score + (not avoided): an avoided qubit only on merit
                            if (!dup) grown.push_back({2 * score(s.rem, low | h, low) + (((avoid >> q) & 1ull) ? 0 : 1), h});
                        }
                    if (grown.empty()) break;
                    std::stable_sort(grown.begin(), grown.end(),
                                     [](const auto& a, const auto& b) { return a.first > b.first; });
                    if ((int)grown.size() > width) grown.resize(width);
                    part.swap(grown);
                }
                for (const auto& pp : part) {
                    St t;
                    t.rem = apply(s.rem, low | pp.second);
                    if (t.rem.size() == s.rem.size()) continue;
                    bool dup = false;
                    for (const auto& v : seen) dup = dup || v == t.rem;
                    if (dup) continue;
                    seen.push_back(t.rem);
                    t.hist = s.hist;
                    t.hist.push_back({r0, pp.second});
                    t.cost = s.cost + layout_cost(r0, pp.second);
                    next.push_back(std::move(t));
                }
            }
        }
        if (next.empty()) break;
        std::stable_sort(next.begin(), next.end(), [](const St& a, const St& b) {
            return a.rem.size() != b.rem.size() ? a.rem.size() < b.rem.size() : a.cost < b.cost;
        });
        if ((int)next.size() > width) next.resize(width);
        states.swap(next);
    }
    return {};  // (no progress possible: the caller keeps its other candidates)
}

static bool same_op(const Op& a, const Op& b) {
    if (a.kind != b.kind || a.sub != b.sub || a.t0 != b.t0 || a.t1 != b.t1 || a.cmask != b.cmask ||
        a.d0_one != b.d0_one || a.src != b.src)
        return false;
    for (int i = 0; i < 8; ++i)
        if (a.m[i] != b.m[i]) return false;
    return true;
}

PlanCache::Entry& PlanCache::get(const std::vector<Op>& ops, int n_qubits, hipStream_t stream,
                                 uint64_t avoid, uint64_t avoid_first) {
    for (auto& e : entries) {
        bool hit = e->n == n_qubits && e->h == tile_height_default() && e->avoid == avoid &&
                   e->avoid_first == avoid_first && e->ctrl_out == (tile_ctrl_out() ? 1 : 0) &&
                   e->key.size() == ops.size();
        for (size_t i = 0; hit && i < ops.size(); ++i) hit = same_op(e->key[i], ops[i]);
        if (hit) {
            e->used = ++clock;
            return *e;
        }
    }
    if (entries.size() >= kEntries) {  // evict the least recently used plan (and its code object:
                                       // ~JitModule waits for the device before unloading it)
        auto lru = std::min_element(entries.begin(), entries.end(),
                                    [](const auto& a, const auto& b) { return a->used < b->used; });
        if ((*lru)->jit.mod) QSIM_HIPCHK(hipStreamSynchronize(stream));  // its kernels may be queued
        entries.erase(lru);
    }
    auto e = std::make_unique<Entry>();
    e->plan = plan_fused(ops, n_qubits, -1, avoid, avoid_first);
    e->avoid_first = avoid_first;
    e->key = ops;
    e->n = n_qubits;
    e->h = tile_height_default();
    e->ctrl_out = tile_ctrl_out() ? 1 : 0;
    e->avoid = avoid;
    e->used = ++clock;
    entries.push_back(std::move(e));
    return *entries.back();
}

void PlanCache::put(std::vector<Op> ops, int n_qubits, Plan plan, hipStream_t stream) {
    if (entries.size() >= kEntries) {
        auto lru = std::min_element(entries.begin(), entries.end(),
                                    [](const auto& a, const auto& b) { return a->used < b->used; });
        if ((*lru)->jit.mod) QSIM_HIPCHK(hipStreamSynchronize(stream));
        entries.erase(lru);
    }
    auto e = std::make_unique<Entry>();
    e->plan = std::move(plan);
    e->key = std::move(ops);
    e->n = n_qubits;
    e->h = tile_height_default();
    e->ctrl_out = tile_ctrl_out() ? 1 : 0;
    e->used = ++clock;
    entries.push_back(std::move(e));
}

static int env_int(const char* k, int d) {
    const char* e = std::getenv(k);
    return e ? std::atoi(e) : d;
}

static std::atomic<int> g_tile_h{-1};  // qsim_set_tile_height (-1: not set)
static thread_local int t_tile_h = -1;  // TileHeightScope of the calling thread
static int env_tile_h() {                // QSIM_TILE_HMAX (-1: not set)
    static const int v = std::getenv("QSIM_TILE_HMAX") ? std::min(kTileHMax, std::max(0, env_int("QSIM_TILE_HMAX", 6))) : -1;
    return v;
}
int tile_height_default() {
    if (t_tile_h >= 0) return t_tile_h;
    const int h = g_tile_h.load();
    if (h >= 0) return h;
    const int e = env_tile_h();
    return e >= 0 ? e : kTileHDefault;
}
bool tile_height_is_set() { return g_tile_h.load() >= 0 || env_tile_h() >= 0; }
// Single-GPU states without an explicit height: 13-qubit tiles from 26 to 28 qubits, where their
// fewer passes outrun the slower streaming (W-HC 26q +23 %, 27q +15 %, 28q +5 %; 29q -3 %, 30q
// -2 %: profiles/r02/h7s/).  QSIM_TILE_AUTO=0 keeps 12-qubit tiles everywhere.
int tile_height_for(int n) {
    const int h = g_tile_h.load();
    if (h >= 0) return h;
    if (env_tile_h() >= 0) return env_tile_h();
    static const bool on = env_int("QSIM_TILE_AUTO", 1) != 0;
    return on && n >= 26 && n <= 28 ? 7 : kTileHDefault;
}
static thread_local int t_tile_rb = -1;
// Small states (12-qubit tiles, n <= 20: at most 256 tiles, i.e. at most one 4-wave workgroup
// per CU): 8 amplitudes per thread (512 threads) doubles the waves for the same tile — W-HC 18q
// +14 %, 20q unchanged (profiles/r02/rb/).  QSIM_TILE_RB overrides (2..4).
int tile_rb_for(int n, int h) {
    if (h != 6) return -1;
    static const int env = env_int("QSIM_TILE_RB", 0);
    if (env >= 2 && env <= 4) return env;
    return n >= 12 && n <= 20 ? 3 : -1;
}
// 13-qubit tiles: QSIM_TILE_RB7 = 3 gives 8 amplitudes per thread (1024-thread workgroups, 16
// waves per CU, half the registers of the default 4) — for the tile-height calibration and tests.
static std::atomic<int> g_tile_rb7{-1};
int tile_rb7() {
    const int v = g_tile_rb7.load();
    if (v >= 0) return v;
    static const int env = env_int("QSIM_TILE_RB7", 4);
    return env == 3 ? 3 : 4;
}
void tile_rb7_configure(int rb) { g_tile_rb7.store(rb == 3 || rb == 4 ? rb : -1); }
int tile_rb_default(int heff) {
    if (heff == 7) return tile_rb7();
    return heff == 6 && t_tile_rb >= 2 ? t_tile_rb : stage_rb(heff);
}
TileHeightScope::TileHeightScope(int h, int rb) : prev_(t_tile_h), prev_rb_(t_tile_rb) {
    t_tile_h = h;
    t_tile_rb = rb;
}
TileHeightScope::~TileHeightScope() {
    t_tile_h = prev_;
    t_tile_rb = prev_rb_;
}
void tile_height_configure(int h) {
    if (h > kTileHMax) fail(QSIM_ERR_INVALID_ARGUMENT, "tile height out of range (0..7)");
    g_tile_h.store(h < 0 ? -1 : h);
}

// One staged (h >= 4) or unstaged tile pass appended to `plan`: tile bits 0..r0-1 are physical
// positions 0..r0-1, tile bits r0.. are hpos[] (ascending); bit_of[q] is the tile bit of qubit q
// as the ops name it.  st_pos / st_tid (relayout passes, relayout.hip; null otherwise): store
// positions of the tile bits and of the tile-id bits.
static std::atomic<int> g_ctrl_out{-1};
static thread_local bool t_ctrl_off = false;
bool tile_ctrl_out() {
    if (t_ctrl_off) return false;
    if (g_ctrl_out.load() < 0) {
        const char* e = std::getenv("QSIM_TILE_CTRL_OUT");
        g_ctrl_out.store(e ? (std::atoi(e) != 0 ? 1 : 0) : 1);
    }
    return g_ctrl_out.load() != 0;
}
void tile_ctrl_out_configure(int mode) {
    tile_ctrl_out();
    if (mode >= 0) g_ctrl_out.store(mode ? 1 : 0);
}
CtrlOutOff::CtrlOutOff() : prev_(t_ctrl_off) { t_ctrl_off = true; }
CtrlOutOff::~CtrlOutOff() { t_ctrl_off = prev_; }

void append_tile_pass(Plan& plan, const std::vector<Op>& ops, int n, int h, int r0, const int* hpos,
                      const int* bit_of, const int* st_pos, const int* st_tid, const int* phys_of) {
    FusedPass p;
    p.h = h;
    p.r0 = r0;
    double bpa = 0.0;
    for (const Op& op : ops) bpa += op_alg_bytes(op, 1.0);
    p.alg_bpa = std::min(32.0, bpa);
    for (int i = 0; i < 6 + h - r0; ++i) p.hpos[i] = hpos[i];
    if (st_pos) {
        p.relayout = 1;
        p.n_tid = n - 6 - h;
        if (p.n_tid > 32 || h < 4) fail(QSIM_ERR_RUNTIME, "relayout pass out of range");
        for (int x = 0; x < 6 + h; ++x) p.st_pos[x] = st_pos[x];
        for (int i = 0; i < p.n_tid; ++i) p.st_tid[i] = st_tid[i];
    }
    std::vector<TileOp> tops;
    std::vector<int> tsrc;
    for (const Op& op : ops) {
        uint32_t cm = 0;
        uint64_t cm_out = 0;
        for (int q = 0; q < n; ++q)
            if ((op.cmask >> q) & 1ull) {
                if (bit_of[q] >= 0) cm |= 1u << bit_of[q];
                else cm_out |= 1ull << (phys_of ? phys_of[q] : q);
            }
        int b0 = bit_of[op.t0], b1 = op.kind == K_SWAP ? bit_of[op.t1] : -1;
        if (b0 < 0 || (op.kind == K_SWAP && b1 < 0)) fail(QSIM_ERR_RUNTIME, "tile pass: target outside the tile");
        if (cm_out && h < 4) fail(QSIM_ERR_RUNTIME, "tile-constant controls need staged tiles");
        if (op.kind == K_SWAP && b0 > b1) std::swap(b0, b1);
        tops.push_back(make_tile_op(op.kind, op.sub, b0, b1, cm, op.d0_one ? 1 : 0, op.m));
        tops.back().cm_out = cm_out;
        tops.back().step = op.src;
        tsrc.push_back(op.src);
    }
    if (h >= 4) {
        p.rb = tile_rb_default(h);
        plan_stages(tops, tsrc, 6 + h, p.rb, plan, p, st_pos);
    } else {
        if (st_pos) fail(QSIM_ERR_RUNTIME, "relayout pass needs staged tiles");
        p.op_begin = (int)plan.ops.size();
        for (size_t i = 0; i < tops.size(); ++i) {
            plan.ops.push_back(tops[i]);
            plan.order.push_back(tsrc[i]);
        }
        p.op_end = (int)plan.ops.size();
    }
    plan.fused_gate_count += ops.size();
    plan.tile_passes += 1;
    plan.passes.push_back(p);
}

void relayout_last_pass(Plan& plan, int n, const int* tau) {
    if (plan.passes.empty()) fail(QSIM_ERR_RUNTIME, "relayout_last_pass: empty plan");
    FusedPass p = plan.passes.back();
    if (p.single >= 0 || p.h < 4) fail(QSIM_ERR_RUNTIME, "relayout_last_pass: not a staged pass");
    // the pass's ops in execution order (tile-bit space; SWAPs already lowered)
    std::vector<TileOp> ops;
    std::vector<int> src;
    for (int k = p.stage_begin; k < p.stage_end; ++k)
        for (int o = plan.stages[k].op_begin; o < plan.stages[k].op_end; ++o) {
            ops.push_back(plan.ops[o]);
            src.push_back(plan.order[o]);
        }
    const int tb = 6 + p.h;
    int st_pos[13] = {0}, st_tid[32] = {0};
    uint64_t hm = 0;
    for (int x = 0; x < tb; ++x) {
        const int pos = x < p.r0 ? x : p.hpos[x - p.r0];
        if (x >= p.r0) hm |= 1ull << pos;
        st_pos[x] = tau[pos];
    }
    int k = 0;
    for (int q = p.r0; q < n; ++q)
        if (!((hm >> q) & 1ull)) {
            if (k >= 32) fail(QSIM_ERR_RUNTIME, "relayout_last_pass: too many tile-id bits");
            st_tid[k++] = tau[q];
        }
    p.relayout = 1;
    p.n_tid = k;
    for (int x = 0; x < tb; ++x) p.st_pos[x] = st_pos[x];
    for (int i = 0; i < k; ++i) p.st_tid[i] = st_tid[i];
    plan_stages(ops, src, tb, p.rb, plan, p, st_pos);  // (appends its stages; the old ones idle)
    plan.passes.back() = p;
}

Plan plan_fused(const std::vector<Op>& ops, int n, int hmax, uint64_t avoid, uint64_t avoid_first) {
    if (hmax < 0) hmax = tile_height_default();
    Plan plan;
    auto add_single = [&](const Op& op) {
        FusedPass p;
        p.single = (int)plan.singles.size();
        plan.singles.push_back(op);
        plan.passes.push_back(p);
    };
    if (n < 6) {  // the state is smaller than one wavefront tile
        for (const Op& op : ops) add_single(op);
        return plan;
    }
    const int heff = std::min(hmax, n - 6);
    // Staged tiles (12 bits at h = 6) may shorten the contiguous HBM run to 2^r0 amplitudes
    // (r0 = 4: 256 B runs, four per wave instruction) to free 12 - r0 tile slots for the planner.
    // Every (r0, strategy) candidate is planned and the one with the fewest HBM passes wins
    // (ties: the longer run).  QSIM_TILE_R0 / QSIM_PLANNER (0 greedy, 1 lookahead) pin one.
    // The small unstaged tiles keep r0 = 6 and the greedy split.
    static const int r0_pin = env_int("QSIM_TILE_R0", 0);
    static const int strat_pin = env_int("QSIM_PLANNER", -1);
    std::vector<PassChoice> best;
    for (int r0 = 6; r0 >= (heff >= 4 ? 4 : 6); --r0) {
        if (r0_pin && heff >= 4 && r0 != std::min(6, std::max(4, r0_pin))) continue;
        for (int la = 0; la <= (heff >= 4 ? 1 : 0); ++la) {
            if (strat_pin >= 0 && heff >= 4 && la != (strat_pin ? 1 : 0)) continue;
            std::vector<PassChoice> c = choose_passes(ops, n, r0, 6 + heff - r0, la != 0, avoid, avoid_first);
            for (PassChoice& ch : c) ch.r0 = r0;
            if (best.empty() || c.size() < best.size()) best.swap(c);
        }
    }
    static const int beam = env_int("QSIM_PLAN_BEAM", 32);
    static const int beam_min_q = env_int("QSIM_PLAN_BEAM_MIN_QUBITS", 20);
    if (beam > 0 && heff >= 4 && n >= beam_min_q && !r0_pin && strat_pin < 0 && best.size() > 1) {
        // width shrinks with the circuit so the search stays ~O(10^8) simple steps
        const int w = std::max(2, (int)(beam * 256.0 / std::max<size_t>(256, ops.size())));
        std::vector<PassChoice> c = beam_passes(ops, n, heff, w, avoid, avoid_first);
        if (!c.empty() && c.size() < best.size()) best.swap(c);
    }
    for (size_t pi = 0; pi < best.size(); ++pi) {
        PassChoice& ch = best[pi];
        if (ch.single) {
            add_single(ch.ops.front());
            continue;
        }
        const uint64_t pav = avoid | (pi == 0 ? avoid_first : 0ull);  // (padding of this pass)
        int r0 = ch.r0, hp = heff;
        uint64_t hi = ch.hi;
        // Mixed heights: a pass of a 13-qubit plan whose gates fit a 12-qubit tile runs as one
        // (two workgroups per CU stream faster than one big one; the pass count is unchanged).
        // Longer runs first.  QSIM_TILE_MIX=0 keeps every pass at the plan's height.
        static const bool mix = env_int("QSIM_TILE_MIX", 1) != 0;
        if (heff == 7 && mix) {
            uint64_t need = 0;
            for (const Op& op : ch.ops) need |= op_need(op, tile_ctrl_out());
            for (int r = 6; r >= 4; --r) {
                const uint64_t above = need & ~((1ull << r) - 1ull);
                if (__builtin_popcountll(above) <= 12 - r) {
                    hp = 6;
                    r0 = r;
                    hi = above;
                    break;
                }
            }
        }
        const int nfree = 6 + hp - r0;
        // Pad the tile to nfree chosen qubits (uniform tile size / occupancy).
        for (int q = r0; q < n && __builtin_popcountll(hi) < nfree; ++q)
            if (!((pav >> q) & 1ull)) hi |= 1ull << q;
        // too few qubits outside `avoid` (small states): fill up anyway — such a tile contains
        // the avoided qubit, which the caller detects (the sharded engine then runs the step on
        // the whole shard)
        for (int q = r0; q < n && __builtin_popcountll(hi) < nfree; ++q) hi |= 1ull << q;
        int hpos[kHposMax] = {0}, bit_of[64];
        int k = 0;
        for (int q = 0; q < 64; ++q) bit_of[q] = -1;
        for (int q = 0; q < r0; ++q) bit_of[q] = q;
        for (int q = r0; q < n; ++q)
            if ((hi >> q) & 1ull) {
                hpos[k] = q;
                bit_of[q] = r0 + k;
                ++k;
            }
        append_tile_pass(plan, ch.ops, n, hp, r0, hpos, bit_of, nullptr, nullptr);
    }
    return plan;
}

// ---------------------------------------------------------------------------------------
// Device
// ---------------------------------------------------------------------------------------
struct FArgs {
    double2* st;
    const TileOp* ops;
    const Stage* stages;
    uint64_t stride;     // 2^n
    uint64_t tpt_mask;   // tiles per trajectory - 1
    int log_tpt;
    int op_begin, op_end;
    int stage_begin, stage_end;
    int hpos[kHposMax];
    int r0;              // run bits (tile bits 0..r0-1 = qubits 0..r0-1); hpos covers the rest
    double scale;        // applied at the store: (1/sqrt2)^(unnormalized H butterflies)
    // Pauli frames of a batched noisy run: frames[2 * (step * nbatch + traj)] = {F, G}, the
    // frame X^F Z^G (phase dropped) in force before circuit step `step` (batched.hip).
    const uint64_t* frames;
    int nbatch;
    // Sub-space launch (sharded engine's overlapped remaps): tiles skip the fix_mask positions,
    // which read fix_val; zmask = fix_mask | the tile's own positions above the run.
    uint64_t fix_mask, fix_val, zmask;
    // Relayout pass (FusedPass::relayout): the tile is stored to dst (out of place) at the store
    // positions of its tile bits and tile-id bits.
    double2* dst;
    int relayout, n_tid;
    int st_pos[13];
    int st_tid[32];
    int nt_pos[32];  // the non-tile load positions, ascending (tile-id bit i <-> nt_pos[i])
};

// Runtime-count forms for the staged kernel (count = tile bits above the run, < kHposMax).
__device__ __forceinline__ uint64_t spread_n(uint32_t x, const int* hpos, int cnt) {
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < kHposMax; ++i)
        if (i < cnt) r |= (uint64_t)((x >> i) & 1u) << hpos[i];
    return r;
}
__device__ __forceinline__ uint64_t deposit_n(uint64_t k, const int* hpos, int cnt) {
#pragma unroll
    for (int i = 0; i < kHposMax; ++i) {
        if (i < cnt) {
            const uint64_t lo = k & ((1ull << hpos[i]) - 1ull);
            k = ((k ^ lo) << 1) | lo;
        }
    }
    return k;
}

template <int H>
__device__ __forceinline__ uint64_t spread(uint32_t x, const int* hpos) {
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < H; ++i) r |= (uint64_t)((x >> i) & 1u) << hpos[i];
    return r;
}

template <int H>
__device__ __forceinline__ uint64_t deposit_h(uint64_t k, const int* hpos) {
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const uint64_t lo = k & ((1ull << hpos[i]) - 1ull);
        k = ((k ^ lo) << 1) | lo;
    }
    return k;
}

__device__ __forceinline__ uint32_t ins0(uint32_t p, int b) {
    const uint32_t lo = p & ((1u << b) - 1u);
    return ((p ^ lo) << 1) | lo;
}

// LDS slot of tile element j.  A ds_read/write_b128 bank row is 256 B = 16 amplitudes, so the
// bank of an access is its low 4 index bits.  XOR-ing them with bits 4..7 keeps both access
// families conflict-free: the coalesced HBM phases (consecutive threads = consecutive j) and
// register stages whose bits include tile bits 0..3 (consecutive threads then stride 2^k
// amplitudes, which without the swizzle all land in one 16-B bank slot).
__device__ __forceinline__ uint32_t sw(uint32_t j) { return j ^ ((j >> 4) & 15u); }

// HBM <-> LDS halves shared by both tile kernels: element j = r*256 + tid, low 6 bits are lanes.
template <int H, bool NT = false>
__device__ __forceinline__ void tile_load(const FArgs& a, uint64_t base, double2* tile) {
    constexpr int T = 64 << H;
    constexpr int R = T >= 256 ? T / 256 : 1;
    const int tid = threadIdx.x;
    if constexpr (T >= 256) {  // every thread owns R elements: no guards (keeps v[] in VGPRs)
        double2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t j = (uint32_t)(r * 256 + tid);
            v[r] = ld<NT>(a.st + (base | (j & 63u) | spread<H>(j >> 6, a.hpos)));
        }
#pragma unroll
        for (int r = 0; r < R; ++r) tile[sw(r * 256 + tid)] = v[r];
    } else if (tid < T) {
        const uint32_t j = (uint32_t)tid;
        tile[sw(j)] = a.st[base | (j & 63u) | spread<H>(j >> 6, a.hpos)];
    }
}

template <int H, bool NT = false>
__device__ __forceinline__ void tile_store(const FArgs& a, uint64_t base, const double2* tile) {
    constexpr int T = 64 << H;
    constexpr int R = T >= 256 ? T / 256 : 1;
    const int tid = threadIdx.x;
    if constexpr (T >= 256) {
        double2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = tile[sw(r * 256 + tid)];
        if (a.scale != 1.0) {  // uniform
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = make_double2(v[r].x * a.scale, v[r].y * a.scale);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t j = (uint32_t)(r * 256 + tid);
            st<NT>(a.st + (base | (j & 63u) | spread<H>(j >> 6, a.hpos)), v[r]);
        }
    } else if (tid < T) {
        const uint32_t j = (uint32_t)tid;
        a.st[base | (j & 63u) | spread<H>(j >> 6, a.hpos)] = tile[sw(j)];
    }
}

// Unstaged kernel (h < 4): one LDS sweep + barrier per gate.
template <int H>
__global__ __launch_bounds__(256) void k_fused_tile(FArgs a) {
    constexpr int T = 64 << H;
    __shared__ double2 tile[T];
    const int tid = threadIdx.x;
    const uint64_t tile_id = blockIdx.x;
    const uint64_t base =
        (tile_id >> a.log_tpt) * a.stride + deposit_h<H>((tile_id & a.tpt_mask) << 6, a.hpos);
    tile_load<H>(a, base, tile);
    __syncthreads();
    for (int o = a.op_begin; o < a.op_end; ++o) {
        const TileOp op = ldc(a.ops, o);
        const int kind = op.kind, sub = op.sub, b0 = op.b0;
        const uint32_t cm = op.cmask;
        if (kind == K_M1) {
            const double2 m0 = make_double2(op.m[0], op.m[1]), m1 = make_double2(op.m[2], op.m[3]);
            const double2 m2 = make_double2(op.m[4], op.m[5]), m3 = make_double2(op.m[6], op.m[7]);
            for (uint32_t p = tid; p < (uint32_t)T / 2; p += 256) {
                const uint32_t j0 = ins0(p, b0), j1 = j0 | (1u << b0);
                if ((j0 & cm) == cm) {
                    double2 x0 = tile[sw(j0)], x1 = tile[sw(j1)];
                    m1_pair(sub, m0, m1, m2, m3, x0, x1);
                    tile[sw(j0)] = x0;
                    tile[sw(j1)] = x1;
                }
            }
        } else if (kind == K_DIAG) {
            const double2 d0 = make_double2(op.m[0], op.m[1]), d1 = make_double2(op.m[2], op.m[3]);
            if (op.d0_one) {  // only the target==1 half, enumerated directly
                for (uint32_t p = tid; p < (uint32_t)T / 2; p += 256) {
                    const uint32_t j = ins0(p, b0) | (1u << b0);
                    if ((j & cm) == cm) tile[sw(j)] = diag1(sub, d1, tile[sw(j)]);
                }
            } else {
                for (uint32_t j = tid; j < (uint32_t)T; j += 256)
                    if ((j & cm) == cm)
                        tile[sw(j)] = diag_apply(sub, 0, d0, d1, (j >> b0) & 1u, tile[sw(j)]);
            }
        } else {  // K_SWAP, b0 < b1
            const int b1 = op.b1;
            for (uint32_t p = tid; p < (uint32_t)T / 4; p += 256) {
                const uint32_t j = ins0(ins0(p, b0), b1);
                const uint32_t ja = j | (1u << b1), jb = j | (1u << b0);
                if ((j & cm) == cm) {
                    const double2 xa = tile[sw(ja)], xb = tile[sw(jb)];
                    tile[sw(ja)] = xb;
                    tile[sw(jb)] = xa;
                }
            }
        }
        __syncthreads();
    }
    tile_store<H>(a, base, tile);
}

// Register-stage ops.  The target register bit P and the gate sub-kind are compile-time (one
// dispatch per op, none per pair); controls become per-pair selects, never branches.
template <int SUB>
__device__ __forceinline__ void pair_t(double2 m0, double2 m1, double2 m2, double2 m3,
                                       double2& a0, double2& a1) {
    m1_pair(SUB, m0, m1, m2, m3, a0, a1);  // SUB folds to one arm after inlining
}

__device__ __forceinline__ double2 sel(bool c, double2 a, double2 b) {
    return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

// Controls: register-bit controls (cm_reg) skip whole pairs by a scalar test on the
// compile-time register index; thread-bit controls (cm_thr) are one per-thread select.
// FP64 issue (16 lanes/clk/SIMD on gfx950) and instruction-cache footprint both matter here, so
// the interpreter has exactly three 2x2 arms per target register bit P — swap (X, CNOT, CCX, the
// SWAP lowering: selects only), the unnormalized Hadamard butterfly (a0+a1, a0-a1: 4 DP adds per
// pair; the (1/sqrt2)^k of a pass is applied once when the tile is stored) and the general
// complex 2x2 — and two diagonal arms (negate: Z/CZ; general phase).
enum StageArm : int { A_SWAP = 0, A_HU = 1, A_GEN = 2 };

// No per-pair branches: a branch around one pair makes the compiler merge two versions of the
// register array (v_mov copies of every live amplitude).  Controls are therefore either absent
// (PRED = false, pure arithmetic) or folded — register-bit part as a uniform scalar condition,
// thread-bit part as a per-lane one — into one select per dword.
template <int RB, int P, int ARM, bool PRED>
__device__ __forceinline__ void stage_m1(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op) {
    const uint32_t cr = op.cm_reg, ct = op.cm_thr;
    const double2 m0 = make_double2(op.m[0], op.m[1]), m1 = make_double2(op.m[2], op.m[3]);
    const double2 m2 = make_double2(op.m[4], op.m[5]), m3 = make_double2(op.m[6], op.m[7]);
    const bool thr_ok = (jb & ct) == ct;
#pragma unroll
    for (int r = 0; r < (1 << RB); ++r) {
        if (r & (1 << P)) continue;  // compile time
        const double2 a0 = v[r], a1 = v[r | (1 << P)];
        double2 x0, x1;
        if constexpr (ARM == A_SWAP) {
            x0 = a1;
            x1 = a0;
        } else if constexpr (ARM == A_HU) {
            x0 = make_double2(a0.x + a1.x, a0.y + a1.y);
            x1 = make_double2(a0.x - a1.x, a0.y - a1.y);
        } else {
            x0 = cadd(cmul(m0, a0), cmul(m1, a1));
            x1 = cadd(cmul(m2, a0), cmul(m3, a1));
        }
        if constexpr (PRED) {
            const bool ok = (((uint32_t)r & cr) == cr) && thr_ok;
            x0 = sel(ok, x0, a0);
            x1 = sel(ok, x1, a1);
        }
        v[r] = x0;
        v[r | (1 << P)] = x1;
    }
}

template <int RB, bool NEG>
__device__ __forceinline__ void stage_diag(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op) {
    const uint32_t cr = op.cm_reg, ct = op.cm_thr;
    const int p0 = op.p0, d0_one = op.d0_one;
    const double2 d0 = make_double2(op.m[0], op.m[1]), d1 = make_double2(op.m[2], op.m[3]);
    const bool thr_ok = (jb & ct) == ct;
    const bool tbit = ((jb >> op.b0) & 1u) != 0;  // target bit when it is a thread bit
#pragma unroll
    for (int r = 0; r < (1 << RB); ++r) {
        const bool bit = p0 >= 0 ? (((r >> p0) & 1) != 0) : tbit;
        const bool ok = (((uint32_t)r & cr) == cr) && thr_ok && (bit || !d0_one);
        if constexpr (NEG) {  // d1 = -1, d0 = 1
            v[r] = sel(ok, make_double2(-v[r].x, -v[r].y), v[r]);
        } else {
            const double2 f = make_double2(bit ? d1.x : d0.x, bit ? d1.y : d0.y);
            v[r] = sel(ok, cmul(f, v[r]), v[r]);
        }
    }
}

template <int RB, int P>
__device__ __forceinline__ void stage_m1_arm(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op) {
    const bool pred = (op.cm_reg | op.cm_thr) != 0;
    switch (op.sub) {
        case S_X:
            if (pred) stage_m1<RB, P, A_SWAP, true>(v, jb, op);
            else stage_m1<RB, P, A_SWAP, false>(v, jb, op);
            break;
        case S_H:  // never controlled (no CH in the gate set; the planner re-labels it S_GEN)
            stage_m1<RB, P, A_HU, false>(v, jb, op);
            break;
        default:
            if (pred) stage_m1<RB, P, A_GEN, true>(v, jb, op);
            else stage_m1<RB, P, A_GEN, false>(v, jb, op);
            break;
    }
}

template <int RB>
__device__ __forceinline__ void stage_op(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op) {
    if (op.kind == K_DIAG) {  // SWAPs were lowered to controlled-X by the planner
        if (op.sub == S_NEG) stage_diag<RB, true>(v, jb, op);
        else stage_diag<RB, false>(v, jb, op);
        return;
    }
    switch (op.p0) {
        case 0: stage_m1_arm<RB, 0>(v, jb, op); break;
        case 1: stage_m1_arm<RB, 1>(v, jb, op); break;
        case 2: if constexpr (RB > 2) stage_m1_arm<RB, 2>(v, jb, op); break;
        case 3: if constexpr (RB > 3) stage_m1_arm<RB, 3>(v, jb, op); break;
        default: break;
    }
}

// One op under a Pauli frame X^F Z^G (batched noisy runs).  The stored vector phi relates to the
// trajectory's state by psi = X^F Z^G phi (up to a phase), so a gate U on psi is applied to phi as
// Z^G X^F U X^F Z^G: for the target qubit t that is M -> X^f M X^f (rows and columns swapped
// when f = F_t) then the off-diagonal signs flipped when g = G_t; a control c is satisfied when
// the stored bit is 1 ^ F_c; a diagonal op applies d(stored bit ^ f).  Everything runs through
// the general arms (one select per dword); F and G are uniform over a tile (one trajectory).
// REAL: all four entries real (X, H, Ry, CX and their frame conjugates) — half the FP64 work;
// PRED: the op has controls (per-pair select), else pure arithmetic.
template <int RB, int P, bool REAL, bool PRED>
__device__ __forceinline__ void frame_m1(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op,
                                         double2 m0, double2 m1, double2 m2, double2 m3,
                                         uint32_t pol_reg, uint32_t pol_thr) {
    const uint32_t cr = op.cm_reg, ct = op.cm_thr;
    const bool thr_ok = ((jb ^ pol_thr) & ct) == ct;
#pragma unroll
    for (int r = 0; r < (1 << RB); ++r) {
        if (r & (1 << P)) continue;
        const double2 a0 = v[r], a1 = v[r | (1 << P)];
        double2 x0, x1;
        if constexpr (REAL) {
            x0 = make_double2(m0.x * a0.x + m1.x * a1.x, m0.x * a0.y + m1.x * a1.y);
            x1 = make_double2(m2.x * a0.x + m3.x * a1.x, m2.x * a0.y + m3.x * a1.y);
        } else {
            x0 = cadd(cmul(m0, a0), cmul(m1, a1));
            x1 = cadd(cmul(m2, a0), cmul(m3, a1));
        }
        if constexpr (PRED) {
            const bool ok = ((((uint32_t)r ^ pol_reg) & cr) == cr) && thr_ok;
            x0 = sel(ok, x0, a0);
            x1 = sel(ok, x1, a1);
        }
        v[r] = x0;
        v[r | (1 << P)] = x1;
    }
}

template <int RB, int P>
__device__ __forceinline__ void frame_m1_arm(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op,
                                             double2 m0, double2 m1, double2 m2, double2 m3,
                                             uint32_t pol_reg, uint32_t pol_thr) {
    const bool real = m0.y == 0.0 && m1.y == 0.0 && m2.y == 0.0 && m3.y == 0.0;  // uniform
    const bool pred = (op.cm_reg | op.cm_thr) != 0;
    if (real) {
        if (pred) frame_m1<RB, P, true, true>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr);
        else frame_m1<RB, P, true, false>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr);
    } else {
        if (pred) frame_m1<RB, P, false, true>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr);
        else frame_m1<RB, P, false, false>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr);
    }
}

template <int RB>
__device__ __forceinline__ void stage_op_frame(double2 (&v)[1 << RB], uint32_t jb, const TileOp& op,
                                               const uint64_t* frames, int nbatch, uint64_t traj) {
    const uint64_t* fr = frames + 2 * ((uint64_t)op.step * (uint64_t)nbatch + traj);
    const uint64_t F = fr[0], G = fr[1];  // uniform: scalar loads
    uint32_t pol_reg = 0, pol_thr = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (op.cq[k] < 0 || !((F >> op.cq[k]) & 1ull)) continue;
        if (op.cpos[k] >= 0) pol_reg |= 1u << op.cpos[k];
        else pol_thr |= 1u << op.cb[k];
    }
    const bool f = (F >> op.tq) & 1ull, g = (G >> op.tq) & 1ull;
    if (op.kind == K_DIAG) {
        const double2 d0 = make_double2(op.m[0], op.m[1]), d1 = make_double2(op.m[2], op.m[3]);
        const uint32_t cr = op.cm_reg, ct = op.cm_thr;
        const bool thr_ok = ((jb ^ pol_thr) & ct) == ct;
        const bool tbit = (((jb >> op.b0) & 1u) != 0) != f;
#pragma unroll
        for (int r = 0; r < (1 << RB); ++r) {
            const bool bit = op.p0 >= 0 ? ((((r >> op.p0) & 1) != 0) != f) : tbit;  // logical bit
            const bool ok = ((((uint32_t)r ^ pol_reg) & cr) == cr) && thr_ok && (bit || !op.d0_one);
            const double2 d = make_double2(bit ? d1.x : d0.x, bit ? d1.y : d0.y);
            v[r] = sel(ok, cmul(d, v[r]), v[r]);
        }
        return;
    }
    double2 m0 = make_double2(op.m[0], op.m[1]), m1 = make_double2(op.m[2], op.m[3]);
    double2 m2 = make_double2(op.m[4], op.m[5]), m3 = make_double2(op.m[6], op.m[7]);
    if (f) {  // X M X
        const double2 t0 = m0, t1 = m1;
        m0 = m3;
        m1 = m2;
        m2 = t1;
        m3 = t0;
    }
    if (g) {  // Z M Z
        m1 = make_double2(-m1.x, -m1.y);
        m2 = make_double2(-m2.x, -m2.y);
    }
    switch (op.p0) {
        case 0: frame_m1_arm<RB, 0>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr); break;
        case 1: frame_m1_arm<RB, 1>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr); break;
        case 2: if constexpr (RB > 2) frame_m1_arm<RB, 2>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr); break;
        case 3: if constexpr (RB > 3) frame_m1_arm<RB, 3>(v, jb, op, m0, m1, m2, m3, pol_reg, pol_thr); break;
        default: break;
    }
}

// Thread index spread over the tile bits that are not the stage's register bits.
template <int RB>
__device__ __forceinline__ uint32_t stage_jb(const Stage& st) {
    uint32_t jb = threadIdx.x;
#pragma unroll
    for (int i = 0; i < RB; ++i) jb = ins0(jb, st.fix[i]);
    return jb;
}

// Staged pass.  Stage `stage_begin` runs in registers straight from the HBM loads and stage
// `stage_end - 1` straight into the HBM stores (the planner gives both only high tile bits as
// register bits, so a wave still moves 64 consecutive amplitudes = one 1 KiB run per
// instruction); only the stages in between round-trip through LDS (read, ops, write, barrier).
// A pass whose ops fit one such stage never touches LDS.
template <int H, bool NT, bool FR = false, int RBT = stage_rb(H)>
__global__ __launch_bounds__((64 << H) >> RBT, H >= 7 ? 1 : 2) void k_fused_staged(FArgs a) {  // LDS-bound: 2 WGs/CU (h <= 6), 1 at h = 7
    constexpr int T = 64 << H;
    constexpr int RB = RBT;
    constexpr int R = 1 << RB;
    __shared__ double2 tile[T];
    const uint64_t tile_id = blockIdx.x;
    const int r0 = a.r0, nh = 6 + H - r0;  // run bits, tile bits above the run
    uint64_t kt = (tile_id & a.tpt_mask) << r0;
    if (a.fix_mask) {  // uniform: zero insertion at every skipped position, ascending
        for (uint64_t m = a.zmask; m; m &= m - 1ull) {
            const uint64_t lo = kt & ((1ull << __builtin_ctzll(m)) - 1ull);
            kt = ((kt ^ lo) << 1) | lo;
        }
        kt |= a.fix_val;
    } else {
        kt = deposit_n(kt, a.hpos, nh);
    }
    const uint64_t base = (tile_id >> a.log_tpt) * a.stride + kt;
    uint64_t base_st = 0;  // relayout: the tile's base under the store layout
    if (a.relayout) {
        // every non-tile load position's bit (tile-id bits, and a sub-space launch's fixed bits)
        // moved to its store position
        for (int i = 0; i < a.n_tid; ++i) base_st |= ((kt >> a.nt_pos[i]) & 1ull) << a.st_tid[i];
        base_st += (tile_id >> a.log_tpt) * a.stride;
    }
    const uint32_t run_mask = (1u << r0) - 1u;
    const int sb = a.stage_begin, se = a.stage_end;
    double2 v[R];
    char* const lds = reinterpret_cast<char*>(tile);
    for (int s = sb; s < se; ++s) {  // one copy of the op interpreter; phase branches are uniform
        const Stage sg = ldc(a.stages, s);
        uint32_t jb;
        if (sg.tscatter) {  // relayout pass, last stage: lanes over the store's run bits
            jb = 0;
#pragma unroll
            for (int i = 0; i < 6 + H - RB; ++i) jb |= ((threadIdx.x >> i) & 1u) << sg.tmap[i];
        } else {
            jb = stage_jb<RB>(sg);
        }
        const uint32_t lb = 16u * lds_sigma(jb, sg.trow_in);    // thread part: LDS reads
        const uint32_t lbw = 16u * lds_sigma(jb, sg.trow_out);  // and writes
        if (s == sb) {
            const uint64_t gb = base | (jb & run_mask) | spread_n(jb >> r0, a.hpos, nh);
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = ld<NT>(a.st + (gb | sg.goff[r]));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = *reinterpret_cast<const double2*>(lds + (lb ^ sg.lds[r]));
        }
        if constexpr (FR) {
            const uint64_t traj = tile_id >> a.log_tpt;
            for (int o = sg.op_begin; o < sg.op_end; ++o) {
                const TileOp op = ldc(a.ops, o);
                if (op.step < 0) stage_op<RB>(v, jb, op);  // Clifford: moved the frame instead
                else stage_op_frame<RB>(v, jb, op, a.frames, a.nbatch, traj);
            }
        } else {
            for (int o = sg.op_begin; o < sg.op_end; ++o) {
                const TileOp op = ldc(a.ops, o);
                // tile-constant controls: the tile's non-tile bits decide for the whole tile
                // (uniform: the load base holds them, incl. a sub-space launch's fixed bits)
                if ((base & op.cm_out) != op.cm_out) continue;
                stage_op<RB>(v, jb, op);
            }
        }
        if (s == se - 1) {
            uint64_t gb;
            if (a.relayout) {
                gb = base_st;
#pragma unroll
                for (int x = 0; x < 6 + H; ++x) gb |= (uint64_t)((jb >> x) & 1u) << a.st_pos[x];
            } else {
                gb = base | (jb & run_mask) | spread_n(jb >> r0, a.hpos, nh);
            }
            const double sc = a.scale;
            double2* const out = a.relayout ? a.dst : a.st;
#pragma unroll
            for (int r = 0; r < R; ++r)
                st<NT>(out + (gb | sg.goff[r]), make_double2(v[r].x * sc, v[r].y * sc));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) *reinterpret_cast<double2*>(lds + (lbw ^ sg.lds_w[r])) = v[r];
            __syncthreads();
        }
    }
}

// Staged passes use non-temporal HBM loads/stores (every amplitude is touched once per pass;
// +1.5 % on the 28q W-HC sweep); QSIM_FUSED_NT=0 restores the default cache policy.  Read once
// per process, like the per-gate knobs in gates.hip.
static bool fused_nt() {
    static const bool v = [] {
        const char* e = std::getenv("QSIM_FUSED_NT");
        return e == nullptr || std::atoi(e) != 0;
    }();
    return v;
}

// Workgroups of a persistent pass kernel: every CU's resident share (one 128 KiB-LDS workgroup per
// CU at h = 7, two 64 KiB ones below; QSIM_JIT_PIPE_WG overrides the per-CU count).
static uint64_t pipe_workgroups(int h) {
    static const int cus = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    static const int per = env_int("QSIM_JIT_PIPE_WG", 0);
    return (uint64_t)cus * (uint64_t)(per > 0 ? per : (h >= 7 ? 1 : 2));
}

double2* launch_fused(double2* st, int n, uint64_t batch, const Plan& plan, const TileOp* d_ops,
                      const Stage* d_stages, hipStream_t s, Timer* tm, const JitModule* jm,
                      const uint64_t* frames, const FusedRange& range) {
    double2* const home = st;
    const int nfix = __builtin_popcountll(range.fix_mask);
    const double pass_bytes = 32.0 * std::ldexp((double)(1ull << n), -nfix) * (double)batch;
    const bool nt = fused_nt();
    const size_t last = std::min(range.last, plan.passes.size());
    double2* next_st = st;  // where the next pass reads (a relayout pass's dst)
    for (size_t pidx = range.first; pidx < last; ++pidx) {
        st = next_st;
        const FusedPass& p = plan.passes[pidx];
        if (range.fix_mask && (p.single >= 0 || p.h < 4 || frames))
            fail(QSIM_ERR_RUNTIME, "sub-space launch needs staged tile passes");
        if (frames && (p.single >= 0 || p.h < 4))
            fail(QSIM_ERR_RUNTIME, "Pauli-frame passes need staged tiles (n >= 10)");
        if (p.single >= 0) {
            launch_op(st, n, batch, plan.singles[p.single], s, tm);
            continue;
        }
        FArgs a{};
        a.st = st;
        a.ops = d_ops;
        a.stages = d_stages;
        a.stride = 1ull << n;
        a.op_begin = p.op_begin;
        a.op_end = p.op_end;
        a.stage_begin = p.stage_begin;
        a.stage_end = p.stage_end;
        // (1/sqrt2)^k: exact power of two for even k, one rounding for odd k
        a.scale = std::ldexp(1.0, -(p.hu_count / 2)) * ((p.hu_count & 1) ? kInvSqrt2 : 1.0);
        for (int i = 0; i < kHposMax; ++i) a.hpos[i] = p.hpos[i];
        a.r0 = p.r0;
        uint64_t hmask = 0;
        for (int i = 0; i < 6 + p.h - p.r0; ++i) hmask |= 1ull << p.hpos[i];
        if (hmask & range.fix_mask) fail(QSIM_ERR_RUNTIME, "sub-space launch: pass uses a fixed qubit");
        a.fix_mask = range.fix_mask;
        a.fix_val = range.fix_val;
        a.zmask = hmask | range.fix_mask;
        if (p.relayout) {
            if (frames || p.h < 4 || p.stage_end - p.stage_begin < 2)
                fail(QSIM_ERR_RUNTIME, "relayout pass outside a staged run");
            if (n - 6 - p.h != p.n_tid || p.n_tid > 32) fail(QSIM_ERR_RUNTIME, "relayout pass planned for another size");
            if (!range.alt || batch != 1) fail(QSIM_ERR_RUNTIME, "relayout pass without a second buffer");
            a.relayout = 1;
            a.dst = st == home ? range.alt : home;
            next_st = a.dst;
            a.n_tid = p.n_tid;
            for (int i = 0; i < 13; ++i) a.st_pos[i] = p.st_pos[i];
            for (int i = 0; i < 32; ++i) a.st_tid[i] = p.st_tid[i];
            int k = 0;
            for (int q = 0; q < n && k < 32; ++q)
                if (q >= p.r0 && !((hmask >> q) & 1ull)) a.nt_pos[k++] = q;
            if (k != p.n_tid) fail(QSIM_ERR_RUNTIME, "relayout pass: non-tile positions do not match");
        }
        const int lt = n - 6 - p.h - nfix;
        a.log_tpt = lt;
        a.tpt_mask = (1ull << lt) - 1ull;
        const uint64_t blocks = batch << lt;
        TimedLaunch tl(tm, "fused_tile", pass_bytes * (p.alg_bpa / 32.0), s, true);
        const hipEvent_t ev0 = tl.start(), ev1 = tl.stop();  // null unless profiling
        bool framed = false;  // does any op of this pass run conjugated by the Pauli frame?
        if (frames)
            for (int k = p.stage_begin; k < p.stage_end && !framed; ++k)
                for (int o = plan.stages[k].op_begin; o < plan.stages[k].op_end; ++o) {
                    if (plan.ops[o].step >= 0) framed = true;
                    if (plan.ops[o].cm_out) fail(QSIM_ERR_RUNTIME, "Pauli-frame pass with a tile-constant control");
                }
        if (framed) {  // batched noisy run: non-Clifford ops under the trajectory's Pauli frame
            // the framed kernels exist at the default stage width only (their stage descriptors
            // must have been built for it)
            a.frames = frames;
            a.nbatch = (int)batch;
            if (p.rb != stage_rb(p.h)) {
                if (p.h != 7 || p.rb != 3) fail(QSIM_ERR_RUNTIME, "framed pass with an unsupported stage width");
                hipExtLaunchKernelGGL((k_fused_staged<7, true, true, 3>), dim3((unsigned)blocks), dim3(1024), 0, s, ev0, ev1, 0, a);
                QSIM_HIPCHK(hipGetLastError());
                continue;
            }
            switch (p.h) {
                case 4: hipExtLaunchKernelGGL((k_fused_staged<4, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, ev0, ev1, 0, a); break;
                case 5: hipExtLaunchKernelGGL((k_fused_staged<5, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, ev0, ev1, 0, a); break;
                case 6: hipExtLaunchKernelGGL((k_fused_staged<6, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, ev0, ev1, 0, a); break;
                default: hipExtLaunchKernelGGL((k_fused_staged<7, true, true>), dim3((unsigned)blocks), dim3(stage_threads(7)), 0, s, ev0, ev1, 0, a); break;
            }
            QSIM_HIPCHK(hipGetLastError());
            continue;
        }
        const size_t pi = pidx;
        if (jm && pi < jm->fn.size() && jm->fn[pi]) {  // circuit-specialised kernel (jit.hip)
            unsigned long long stride = a.stride, tpt = a.tpt_mask, zm = a.zmask, fv = a.fix_val, ntiles = blocks;
            int lt_arg = lt;
            // (dst: the eighth parameter of relayout kernels only; other kernels take seven)
            void* args[] = {&a.st, &stride, &tpt, &lt_arg, &zm, &fv, &ntiles, &a.dst};
            const unsigned nthr = (unsigned)((64 << p.h) >> p.rb);
            // a pipelined (persistent) kernel gets the resident workgroups only and walks its tiles
            const uint64_t grid = jit_pass_pipelined(p) ? std::min<uint64_t>(blocks, pipe_workgroups(p.h)) : blocks;
            if (grid * nthr > 0xffffffffull) fail(QSIM_ERR_RUNTIME, "pass grid too large");
            // grid in work-items; the events (if any) time the dispatch packet itself
            QSIM_HIPCHK(hipExtModuleLaunchKernel(jm->fn[pi], (uint32_t)(grid * nthr), 1, 1, nthr, 1, 1, 0, s,
                                                 args, nullptr, ev0, ev1, 0));
            continue;
        }
        if (p.h >= 4 && p.rb != stage_rb(p.h)) {  // narrower stages (small states): 512 / 1024 threads
            if (p.h == 7 && p.rb == 3) {  // 13-qubit tiles, 8 amplitudes per thread
                if (nt) hipExtLaunchKernelGGL((k_fused_staged<7, true, false, 3>), dim3((unsigned)blocks), dim3(1024), 0, s, ev0, ev1, 0, a);
                else hipExtLaunchKernelGGL((k_fused_staged<7, false, false, 3>), dim3((unsigned)blocks), dim3(1024), 0, s, ev0, ev1, 0, a);
                QSIM_HIPCHK(hipGetLastError());
                continue;
            }
            if (p.h != 6 || p.rb < 2 || p.rb > 3) fail(QSIM_ERR_RUNTIME, "unsupported stage width");
            if (p.rb == 3) {
                if (nt) hipExtLaunchKernelGGL((k_fused_staged<6, true, false, 3>), dim3((unsigned)blocks), dim3(512), 0, s, ev0, ev1, 0, a);
                else hipExtLaunchKernelGGL((k_fused_staged<6, false, false, 3>), dim3((unsigned)blocks), dim3(512), 0, s, ev0, ev1, 0, a);
            } else {
                if (nt) hipExtLaunchKernelGGL((k_fused_staged<6, true, false, 2>), dim3((unsigned)blocks), dim3(1024), 0, s, ev0, ev1, 0, a);
                else hipExtLaunchKernelGGL((k_fused_staged<6, false, false, 2>), dim3((unsigned)blocks), dim3(1024), 0, s, ev0, ev1, 0, a);
            }
            QSIM_HIPCHK(hipGetLastError());
            continue;
        }
        switch (p.h) {
#define QSIM_TILE_CASE(HH) \
    case HH: hipExtLaunchKernelGGL(k_fused_tile<HH>, dim3((unsigned)blocks), dim3(256), 0, s, ev0, ev1, 0, a); break;
#define QSIM_STAGED_CASE(HH) \
    case HH:                                                                                      \
        if (nt) hipExtLaunchKernelGGL((k_fused_staged<HH, true>), dim3((unsigned)blocks), dim3(stage_threads(HH)), 0, s, ev0, ev1, 0, a); \
        else hipExtLaunchKernelGGL((k_fused_staged<HH, false>), dim3((unsigned)blocks), dim3(stage_threads(HH)), 0, s, ev0, ev1, 0, a); \
        break;
            QSIM_TILE_CASE(0)
            QSIM_TILE_CASE(1)
            QSIM_TILE_CASE(2)
            QSIM_TILE_CASE(3)
            QSIM_STAGED_CASE(4)
            QSIM_STAGED_CASE(5)
            QSIM_STAGED_CASE(6)
            QSIM_STAGED_CASE(7)
#undef QSIM_TILE_CASE
#undef QSIM_STAGED_CASE
            default: fail(QSIM_ERR_RUNTIME, "unsupported tile height");
        }
        QSIM_HIPCHK(hipGetLastError());
    }
    return next_st;
}

}  // namespace qsim_hip
