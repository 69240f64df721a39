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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "device_ops.hpp"
#include "engine.hpp"

namespace qsim_hip {

// ---------------------------------------------------------------------------------------
// Host planner
// ---------------------------------------------------------------------------------------
static uint64_t op_qubits(const Op& op) {
    uint64_t m = op.cmask | (1ull << op.t0);
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

// Group one pass's ops (tile bits) into register stages of at most `rb` target bits.
static void plan_stages(std::vector<TileOp>& pass_ops, std::vector<int>& pass_src, int tile_bits,
                        int rb, Plan& plan, FusedPass& p) {
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
            if (t.cmask == 0) ++p.hu_count;  // unnormalized butterfly in the staged kernel
            else t.sub = S_GEN;              // (no controlled H in the gate set; keep it exact)
        }
    }
    std::vector<int> rem(ops.size());
    for (size_t i = 0; i < rem.size(); ++i) rem[i] = (int)i;
    while (!rem.empty()) {
        uint32_t sbits = 0, blocked = 0;
        std::vector<int> in, deferred;
        for (int i : rem) {
            const TileOp& t = ops[i];
            const uint32_t need = t.kind == K_M1 ? (1u << t.b0) : 0u;
            const uint32_t touch = t.cmask | (1u << t.b0);
            if ((touch & blocked) == 0 && __builtin_popcount(sbits | need) <= rb) {
                sbits |= need;
                in.push_back(i);
            } else {
                deferred.push_back(i);
                blocked |= touch;
            }
        }
        // pad with the highest unused tile bits (threads then walk consecutive LDS slots)
        for (int b = tile_bits - 1; b >= 0 && __builtin_popcount(sbits) < rb; --b) sbits |= 1u << b;
        Stage st{};
        int k = 0;
        int pos_of[32];
        for (int b = 0; b < tile_bits; ++b)
            if ((sbits >> b) & 1u) {
                st.fix[k] = b;
                pos_of[b] = k;
                ++k;
            }
        for (int r = 0; r < (1 << rb); ++r) {
            uint32_t o = 0;
            for (int i = 0; i < rb; ++i)
                if ((r >> i) & 1) o |= 1u << st.fix[i];
            st.offs[r] = o;
        }
        st.op_begin = (int)plan.ops.size();
        for (int i : in) {
            TileOp t = ops[i];
            t.p0 = ((sbits >> t.b0) & 1u) ? pos_of[t.b0] : -1;  // M1 targets are always stage bits
            t.cm_reg = 0;
            for (int b = 0; b < tile_bits; ++b)
                if (((t.cmask & sbits) >> b) & 1u) t.cm_reg |= 1u << pos_of[b];
            t.cm_thr = t.cmask & ~sbits;
            plan.ops.push_back(t);
            plan.order.push_back(src[i]);
        }
        st.op_end = (int)plan.ops.size();
        plan.stages.push_back(st);
        rem.swap(deferred);
    }
    p.stage_end = (int)plan.stages.size();
}

Plan plan_fused(const std::vector<Op>& ops, int n, int hmax) {
    if (hmax < 0) {
        static const int def = [] {
            const char* e = std::getenv("QSIM_TILE_HMAX");
            const int v = e ? std::atoi(e) : kTileHMax;
            return std::min(kTileHMax, std::max(0, v));
        }();
        hmax = def;
    }
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
    const uint64_t low = 0x3full;
    std::vector<Op> remaining = ops;
    while (!remaining.empty()) {
        // The first remaining gate is never blocked; if it needs more high qubits than a tile
        // holds it runs as a per-gate step (keeps program order, guarantees progress).
        if (__builtin_popcountll(op_qubits(remaining.front()) & ~low) > heff) {
            add_single(remaining.front());
            remaining.erase(remaining.begin());
            continue;
        }
        uint64_t hi = 0, blocked = 0;
        std::vector<Op> in_pass, deferred;
        for (const Op& op : remaining) {
            const uint64_t q = op_qubits(op);
            const uint64_t qh = q & ~low;
            if ((q & blocked) == 0 && __builtin_popcountll(hi | qh) <= heff) {
                hi |= qh;
                in_pass.push_back(op);
            } else {
                deferred.push_back(op);
                blocked |= q;
            }
        }
        // Pad the tile to h = heff high qubits (uniform tile size / occupancy).
        for (int q = 6; q < n && __builtin_popcountll(hi) < heff; ++q) hi |= 1ull << q;
        FusedPass p;
        p.h = heff;
        int k = 0;
        int bit_of[64];
        for (int q = 0; q < 6; ++q) bit_of[q] = q;
        for (int q = 6; q < n; ++q)
            if ((hi >> q) & 1ull) {
                p.hpos[k] = q;
                bit_of[q] = 6 + k;
                ++k;
            }
        std::vector<TileOp> tops;
        std::vector<int> tsrc;
        for (const Op& op : in_pass) {
            uint32_t cm = 0;
            for (int q = 0; q < n; ++q)
                if ((op.cmask >> q) & 1ull) cm |= 1u << bit_of[q];
            int b0 = bit_of[op.t0], b1 = op.kind == K_SWAP ? bit_of[op.t1] : -1;
            if (op.kind == K_SWAP && b0 > b1) std::swap(b0, b1);
            tops.push_back(make_tile_op(op.kind, op.sub, b0, b1, cm, op.d0_one ? 1 : 0, op.m));
            tsrc.push_back(op.src);
        }
        if (heff >= 4) {
            plan_stages(tops, tsrc, 6 + heff, heff - 2, plan, p);
        } else {
            p.op_begin = (int)plan.ops.size();
            for (size_t i = 0; i < tops.size(); ++i) {
                plan.ops.push_back(tops[i]);
                plan.order.push_back(tsrc[i]);
            }
            p.op_end = (int)plan.ops.size();
        }
        plan.fused_gate_count += in_pass.size();
        plan.tile_passes += 1;
        plan.passes.push_back(p);
        remaining.swap(deferred);
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
    int hpos[8];
    double scale;        // applied at the store: (1/sqrt2)^(unnormalized H butterflies)
};

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

// The register stages of one tile (tile already in LDS; ends with a barrier).
template <int H>
__device__ __forceinline__ void run_stages(const FArgs& a, double2* tile) {
    constexpr int RB = H - 2;
    constexpr int R = 1 << RB;
    const int tid = threadIdx.x;
    for (int s = a.stage_begin; s < a.stage_end; ++s) {
        const Stage st = ldc(a.stages, s);
        uint32_t offs[R];
#pragma unroll
        for (int r = 0; r < R; ++r) offs[r] = st.offs[r];
        uint32_t jb = (uint32_t)tid;  // thread index spread over the non-stage tile bits
#pragma unroll
        for (int i = 0; i < RB; ++i) jb = ins0(jb, st.fix[i]);
        double2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = tile[sw(jb | offs[r])];
        for (int o = st.op_begin; o < st.op_end; ++o) stage_op<RB>(v, jb, ldc(a.ops, o));
#pragma unroll
        for (int r = 0; r < R; ++r) tile[sw(jb | offs[r])] = v[r];
        __syncthreads();
    }
}

template <int H, bool NT>
__global__ __launch_bounds__(256, 2) void k_fused_staged(FArgs a) {  // 2 WGs/CU (LDS-bound)
    constexpr int T = 64 << H;
    __shared__ double2 tile[T];
    const uint64_t tile_id = blockIdx.x;
    const uint64_t base =
        (tile_id >> a.log_tpt) * a.stride + deposit_h<H>((tile_id & a.tpt_mask) << 6, a.hpos);
    tile_load<H, NT>(a, base, tile);
    __syncthreads();
    run_stages<H>(a, tile);
    tile_store<H, NT>(a, base, tile);
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

void launch_fused(double2* st, int n, uint64_t batch, const Plan& plan, const TileOp* d_ops,
                  const Stage* d_stages, hipStream_t s, Timer* tm) {
    const double pass_bytes = 32.0 * (double)(1ull << n) * (double)batch;
    const bool nt = fused_nt();
    for (const FusedPass& p : plan.passes) {
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
        for (int i = 0; i < 8; ++i) a.hpos[i] = p.hpos[i];
        const int lt = n - 6 - p.h;
        a.log_tpt = lt;
        a.tpt_mask = (1ull << lt) - 1ull;
        const uint64_t blocks = batch << lt;
        TimedLaunch tl(tm, "fused_tile", pass_bytes, s);
        switch (p.h) {
#define QSIM_TILE_CASE(HH) \
    case HH: hipLaunchKernelGGL(k_fused_tile<HH>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
#define QSIM_STAGED_CASE(HH) \
    case HH:                                                                                      \
        if (nt) hipLaunchKernelGGL((k_fused_staged<HH, true>), dim3((unsigned)blocks), dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((k_fused_staged<HH, false>), dim3((unsigned)blocks), dim3(256), 0, s, a); \
        break;
            QSIM_TILE_CASE(0)
            QSIM_TILE_CASE(1)
            QSIM_TILE_CASE(2)
            QSIM_TILE_CASE(3)
            QSIM_STAGED_CASE(4)
            QSIM_STAGED_CASE(5)
            QSIM_STAGED_CASE(6)
#undef QSIM_TILE_CASE
#undef QSIM_STAGED_CASE
            default: fail(QSIM_ERR_RUNTIME, "unsupported tile height");
        }
        QSIM_HIPCHK(hipGetLastError());
    }
}

}  // namespace qsim_hip
