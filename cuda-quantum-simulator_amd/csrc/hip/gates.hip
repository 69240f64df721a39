// gates.hip — per-gate HBM-streaming kernels for gfx950 and the host lowering of reference
// gates to Ops.
//
// Reference behaviour followed: src/Gates.cu:19-410 (one kernel per gate type; qubit q <->
// index bit q; CNOT/CRY/CRZ args (control, target); Toffoli (c1, c2, target)).
//
// MI355X design (not a translation of the reference's thread-per-pair / thread-per-amplitude
// grids): the low 6 index bits are the 64 lanes of a wavefront, so every global access is a
// wave-wide 1 KiB contiguous dwordx4 burst.
//   * "slice" mode (target >= 6): one wave-item = 64 pairs; lanes load the 1 KiB run with the
//     target bit 0 and the 1 KiB run with it 1.  High controls are zero-inserted positions that
//     are forced to 1, so only the control==1 subspace is enumerated (CNOT reads/writes N/2
//     amplitudes, CCX N/4 — the reference launched 2^n threads with 3/4 or 7/8 idle).
//   * "lane" mode (target < 6): one wave-item = 64 consecutive amplitudes, the partner is in
//     lane ^ (1<<t) and arrives by ds_bpermute (__shfl_xor).
//   * Diagonal gates (Z/S/T/S†/T†/CZ/CRZ/Rz) never need the partner: they are per-amplitude
//     phases, and when d0 == 1 the target bit is forced to 1 too (Z on a high qubit moves N/2).
// Each lane keeps U wave-items in flight (8 outstanding 16-B loads) and a 256-thread block owns
// 4*U consecutive wave-items.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "device_ops.hpp"
#include "engine.hpp"

namespace qsim_hip {

// ---------------------------------------------------------------------------------------
// Host: validation + lowering
// ---------------------------------------------------------------------------------------
const char* gate_name(int type) {
    static const char* names[] = {"X",    "Y",    "Z",  "H",  "S",   "T",   "Sdag", "Tdag", "Rx",
                                  "Ry",   "Rz",   "CNOT", "CZ", "CRY", "CRZ", "SWAP", "Toffoli"};
    return (type >= 0 && type < QSIM_GATE_COUNT) ? names[type] : "?";
}

static int expected_arity(int type) {
    if (type <= QSIM_GATE_RZ) return 1;
    if (type <= QSIM_GATE_SWAP) return 2;
    return 3;
}

void validate_gate(const qsim_gate& g, int n) {
    if (g.type < 0 || g.type >= QSIM_GATE_COUNT)
        fail(QSIM_ERR_RUNTIME, "Unknown gate type " + std::to_string(g.type));
    const int k = expected_arity(g.type);
    if (g.nqubits != k)
        fail(QSIM_ERR_INVALID_ARGUMENT, std::string("Gate ") + gate_name(g.type) + " expects " +
                                            std::to_string(k) + " qubits");
    for (int i = 0; i < k; ++i)
        if (g.qubits[i] < 0 || g.qubits[i] >= n)
            fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(g.qubits[i]) +
                                            " out of range [0, " + std::to_string(n - 1) + "]");
    for (int i = 0; i < k; ++i)
        for (int j = i + 1; j < k; ++j)
            if (g.qubits[i] == g.qubits[j])
                fail(QSIM_ERR_INVALID_ARGUMENT, k == 2 ? "Two-qubit gate requires distinct qubits"
                                                       : "Three-qubit gate requires three distinct qubits");
    const bool param = g.type == QSIM_GATE_RX || g.type == QSIM_GATE_RY || g.type == QSIM_GATE_RZ ||
                       g.type == QSIM_GATE_CRY || g.type == QSIM_GATE_CRZ;
    if (param && !std::isfinite(g.parameter))
        fail(QSIM_ERR_INVALID_ARGUMENT, "Rotation angle must be a finite number");
}

static void set_m(Op& op, double ar, double ai, double br, double bi, double cr, double ci,
                  double dr, double di) {
    const double v[8] = {ar, ai, br, bi, cr, ci, dr, di};
    for (int i = 0; i < 8; ++i) op.m[i] = v[i];
}

Op lower_gate(const qsim_gate& g, int n) {
    validate_gate(g, n);
    Op op;
    const double th = g.parameter;
    // cos/sin(theta/2) once on the host (the reference evaluates them per thread).
    const double c = std::cos(th / 2.0), s = std::sin(th / 2.0);
    switch (g.type) {
        case QSIM_GATE_X: op.kind = K_M1; op.sub = S_X; op.t0 = g.qubits[0]; set_m(op, 0, 0, 1, 0, 1, 0, 0, 0); break;
        case QSIM_GATE_Y: op.kind = K_M1; op.sub = S_Y; op.t0 = g.qubits[0]; set_m(op, 0, 0, 0, -1, 0, 1, 0, 0); break;
        case QSIM_GATE_H:
            op.kind = K_M1; op.sub = S_H; op.t0 = g.qubits[0];
            set_m(op, kInvSqrt2, 0, kInvSqrt2, 0, kInvSqrt2, 0, -kInvSqrt2, 0);
            break;
        case QSIM_GATE_Z: op.kind = K_DIAG; op.sub = S_NEG; op.t0 = g.qubits[0]; op.d0_one = true; set_m(op, 1, 0, -1, 0, 0, 0, 0, 0); break;
        case QSIM_GATE_S: op.kind = K_DIAG; op.sub = S_I; op.t0 = g.qubits[0]; op.d0_one = true; set_m(op, 1, 0, 0, 1, 0, 0, 0, 0); break;
        case QSIM_GATE_SDAG: op.kind = K_DIAG; op.sub = S_MI; op.t0 = g.qubits[0]; op.d0_one = true; set_m(op, 1, 0, 0, -1, 0, 0, 0, 0); break;
        case QSIM_GATE_T: op.kind = K_DIAG; op.sub = S_T; op.t0 = g.qubits[0]; op.d0_one = true; set_m(op, 1, 0, kInvSqrt2, kInvSqrt2, 0, 0, 0, 0); break;
        case QSIM_GATE_TDAG: op.kind = K_DIAG; op.sub = S_TDG; op.t0 = g.qubits[0]; op.d0_one = true; set_m(op, 1, 0, kInvSqrt2, -kInvSqrt2, 0, 0, 0, 0); break;
        case QSIM_GATE_RX: op.kind = K_M1; op.t0 = g.qubits[0]; set_m(op, c, 0, 0, -s, 0, -s, c, 0); break;
        case QSIM_GATE_RY: op.kind = K_M1; op.t0 = g.qubits[0]; set_m(op, c, 0, -s, 0, s, 0, c, 0); break;
        case QSIM_GATE_RZ: op.kind = K_DIAG; op.t0 = g.qubits[0]; set_m(op, c, -s, c, s, 0, 0, 0, 0); break;
        case QSIM_GATE_CNOT:
            op.kind = K_M1; op.sub = S_X; op.t0 = g.qubits[1]; op.cmask = 1ull << g.qubits[0];
            set_m(op, 0, 0, 1, 0, 1, 0, 0, 0);
            break;
        case QSIM_GATE_CZ:
            op.kind = K_DIAG; op.sub = S_NEG; op.t0 = g.qubits[1]; op.cmask = 1ull << g.qubits[0];
            op.d0_one = true; set_m(op, 1, 0, -1, 0, 0, 0, 0, 0);
            break;
        case QSIM_GATE_CRY:  // Gates.cu:322-351
            op.kind = K_M1; op.t0 = g.qubits[1]; op.cmask = 1ull << g.qubits[0];
            set_m(op, c, 0, -s, 0, s, 0, c, 0);
            break;
        case QSIM_GATE_CRZ:  // Gates.cu:353-386
            op.kind = K_DIAG; op.t0 = g.qubits[1]; op.cmask = 1ull << g.qubits[0];
            set_m(op, c, -s, c, s, 0, 0, 0, 0);
            break;
        case QSIM_GATE_SWAP:
            op.kind = K_SWAP; op.t0 = std::min(g.qubits[0], g.qubits[1]);
            op.t1 = std::max(g.qubits[0], g.qubits[1]);
            break;
        case QSIM_GATE_TOFFOLI:  // Gates.cu:392-410
            op.kind = K_M1; op.sub = S_X; op.t0 = g.qubits[2];
            op.cmask = (1ull << g.qubits[0]) | (1ull << g.qubits[1]);
            set_m(op, 0, 0, 1, 0, 1, 0, 0, 0);
            break;
        default: fail(QSIM_ERR_RUNTIME, "Unknown gate type");
    }
    return op;
}

double op_alg_bytes(const Op& op, double amps) {
    // bytes = 2 (read+write) x 16 B x amplitudes the op can change  
    const double ctrl = std::ldexp(1.0, -op.ncontrols());
    switch (op.kind) {
        case K_M1: return 32.0 * amps * ctrl;
        case K_DIAG: return (op.d0_one ? 16.0 : 32.0) * amps * ctrl;
        case K_SWAP: return 16.0 * amps * ctrl;
    }
    return 32.0 * amps;
}

// ---------------------------------------------------------------------------------------
// Device: kernel arguments
// ---------------------------------------------------------------------------------------
struct GArgs {
    double2* st;
    uint64_t items;     // wave-items over the whole batch
    uint64_t ipt_mask;  // wave-items per trajectory - 1
    uint64_t stride;    // amplitudes per trajectory (2^n)
    uint64_t setmask;   // high control bits forced to 1
    int log_ipt;
    int nfix;
    int fix[3];         // ascending zero-inserted positions (all >= 6)
    uint32_t lane_ctrl; // control bits among index bits 0..5
    int nlanes;         // lanes carrying data (64, or 2^n for n < 6)
    int t0, t1;
    int sub, d0_one;
    double2 m0, m1, m2, m3;
    int bmap;           // work-group -> item-block order (QSIM_SLICE_BMAP / QSIM_SLICE_FAR_BMAP)
};
// 0: natural; 1: each XCD (blockIdx mod 8) streams one contiguous eighth; 2: consecutive
// work-groups alternate between the two halves of the items
__device__ __forceinline__ uint64_t slice_block(const GArgs& a) {
    const uint64_t b = blockIdx.x, G = gridDim.x;
    if (a.bmap == 1 && (G & 7ull) == 0ull) return (b & 7ull) * (G >> 3) + (b >> 3);
    if (a.bmap == 2 && (G & 1ull) == 0ull) return (b & 1ull) * (G >> 1) + (b >> 1);
    return b;
}

__device__ __forceinline__ uint64_t item_base(const GArgs& a, uint64_t item, int lane) {
    const uint64_t traj = item >> a.log_ipt;
    const uint64_t k = ((item & a.ipt_mask) << 6) | (uint64_t)lane;
    return traj * a.stride + (deposit(k, a.nfix, a.fix) | a.setmask);
}

// Slice mode: target >= 6, each wave-item is 64 pairs (two 1 KiB runs).
// MODE (far-partner targets, QSIM_SLICE_FAR_MODE): 0 the block's 4 waves interleave items and
// each lane alternates the two runs' loads; 1 the loads grouped by run (all |0> runs, then all
// |1> runs); 2 grouped, and each wave takes U consecutive items (U KiB contiguous per run).
template <int U, bool NT, int MODE>
__device__ __forceinline__ void m1_slice_body(const GArgs& a) {
    const int lane = threadIdx.x & 63;
    const uint64_t bid = slice_block(a);
    const uint64_t first = MODE == 2 ? bid * (4 * U) + (uint64_t)(threadIdx.x >> 6) * U
                                     : bid * (4 * U) + (threadIdx.x >> 6);
    const uint64_t step = MODE == 2 ? 1 : 4;
    const uint64_t tb = 1ull << a.t0;
    double2 v0[U], v1[U];
    uint64_t i0[U];
    // lanes failing a low control never load: with controls on bits >= 3 whole 128-B lines are
    // skipped (CNOT with a low control moves N/2 amplitudes, not N)
    const bool lane_ok = (lane & a.lane_ctrl) == a.lane_ctrl;
    if constexpr (MODE == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t item = first + step * u;
            if (item < a.items && lane_ok) {
                i0[u] = item_base(a, item, lane);
                v0[u] = ld<NT>(a.st + i0[u]);
                v1[u] = ld<NT>(a.st + (i0[u] | tb));
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t item = first + step * u;
            if (item < a.items && lane_ok) {
                i0[u] = item_base(a, item, lane);
                v0[u] = ld<NT>(a.st + i0[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t item = first + step * u;
            if (item < a.items && lane_ok) v1[u] = ld<NT>(a.st + (i0[u] | tb));
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + step * u;
        if (item < a.items && lane_ok) {
            m1_pair(a.sub, a.m0, a.m1, a.m2, a.m3, v0[u], v1[u]);
            st<NT>(a.st + i0[u], v0[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + step * u;
        if (item < a.items && lane_ok) st<NT>(a.st + (i0[u] | tb), v1[u]);
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_m1_slice(GArgs a) { m1_slice_body<U, NT, 0>(a); }
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_m1_slice_g(GArgs a) { m1_slice_body<U, NT, 1>(a); }
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_m1_slice_c(GArgs a) { m1_slice_body<U, NT, 2>(a); }

// Lane mode: target < 6, each wave-item is 64 consecutive amplitudes; partner via shuffle.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_m1_lane(GArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t first = slice_block(a) * (4 * U) + (threadIdx.x >> 6);
    const bool active = lane < a.nlanes;
    double2 v[U];
    uint64_t idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        v[u] = make_double2(0.0, 0.0);
        if (item < a.items && active) {
            idx[u] = item_base(a, item, lane);
            v[u] = ld<NT>(a.st + idx[u]);
        }
    }
    const int tm = 1 << a.t0;
    const int bit = (lane >> a.t0) & 1;
    const bool lane_ok = active && ((lane & a.lane_ctrl) == a.lane_ctrl);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const double2 p = shfl_xor2(v[u], tm);
        const uint64_t item = first + 4 * u;
        if (item < a.items && lane_ok) {
            st<NT>(a.st + idx[u], m1_half(a.sub, a.m0, a.m1, a.m2, a.m3, bit, v[u], p));
        }
    }
}

// Diagonal: per-amplitude phase.  Target may be a forced-1 position (d0 == 1, target >= 6).
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_diag(GArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t first = slice_block(a) * (4 * U) + (threadIdx.x >> 6);
    // a phase on the |1> side only (d0 == 1) with a low target: lanes on the |0> side never load
    const bool one_side = a.d0_one && a.t0 < 6 && !((lane >> a.t0) & 1);
    const bool lane_ok = lane < a.nlanes && ((lane & a.lane_ctrl) == a.lane_ctrl) && !one_side;
    double2 v[U];
    uint64_t idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        if (item < a.items && lane_ok) {
            idx[u] = item_base(a, item, lane);
            v[u] = ld<NT>(a.st + idx[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        if (item < a.items && lane_ok) {
            const int bit = (int)((idx[u] >> a.t0) & 1ull);
            if (bit || !a.d0_one) st<NT>(a.st + idx[u], diag_apply(a.sub, a.d0_one, a.m0, a.m1, bit, v[u]));
        }
    }
}

// SWAP, both qubits >= 6: swap the (q0=0,q1=1) and (q0=1,q1=0) 1 KiB runs.
template <int U>
__global__ __launch_bounds__(256) void k_swap_hh(GArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t first = slice_block(a) * (4 * U) + (threadIdx.x >> 6);
    const uint64_t ba = 1ull << a.t1, bb = 1ull << a.t0;
    double2 va[U], vb[U];
    uint64_t i[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        if (item < a.items) {
            i[u] = item_base(a, item, lane);
            va[u] = a.st[i[u] | ba];
            vb[u] = a.st[i[u] | bb];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        if (item < a.items) {
            a.st[i[u] | ba] = vb[u];
            a.st[i[u] | bb] = va[u];
        }
    }
}

// SWAP, q0 < 6 <= q1: both q1-runs per item; the q0 partner is a lane shuffle away.
template <int U>
__global__ __launch_bounds__(256) void k_swap_lh(GArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t first = slice_block(a) * (4 * U) + (threadIdx.x >> 6);
    const uint64_t b1 = 1ull << a.t1;
    double2 s0[U], s1[U];
    uint64_t i[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        s0[u] = make_double2(0.0, 0.0);
        s1[u] = s0[u];
        if (item < a.items) {
            i[u] = item_base(a, item, lane);
            s0[u] = a.st[i[u]];
            s1[u] = a.st[i[u] | b1];
        }
    }
    const int m = 1 << a.t0;
    const int bit = (lane >> a.t0) & 1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const double2 x0 = shfl_xor2(s0[u], m), x1 = shfl_xor2(s1[u], m);
        const uint64_t item = first + 4 * u;
        if (item < a.items) {
            // (q0=1,q1=0) <- (q0=0,q1=1) and (q0=0,q1=1) <- (q0=1,q1=0)
            if (bit) a.st[i[u]] = x1;
            else a.st[i[u] | b1] = x0;
        }
    }
}

// SWAP, both qubits < 6: lanes whose two bits differ take lane ^ (m0|m1).
template <int U>
__global__ __launch_bounds__(256) void k_swap_ll(GArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t first = slice_block(a) * (4 * U) + (threadIdx.x >> 6);
    const bool active = lane < a.nlanes;
    double2 v[U];
    uint64_t idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t item = first + 4 * u;
        v[u] = make_double2(0.0, 0.0);
        if (item < a.items && active) {
            idx[u] = item_base(a, item, lane);
            v[u] = a.st[idx[u]];
        }
    }
    const int mm = (1 << a.t0) | (1 << a.t1);
    const bool differ = (((lane >> a.t0) ^ (lane >> a.t1)) & 1) != 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const double2 p = shfl_xor2(v[u], mm);
        const uint64_t item = first + 4 * u;
        if (item < a.items && active && differ) a.st[idx[u]] = p;
    }
}

// Any number of controls (M1 or DIAG): one thread per active pair / active amplitude, the index
// built by zero insertion at every fixed position (target and controls, any height).  Used only
// when the wave-item kernels' 3 fixed high positions do not suffice (e.g. applyMatrix with 3+
// high controls); correctness path, the wave-item kernels carry the reference gate set.
struct ManyArgs {
    double2* st;
    uint64_t units;
    uint64_t setmask;
    int nfix;
    int fix[64];
    int t0, kind, sub, d0_one;
    double2 m0, m1, m2, m3;
};

__global__ __launch_bounds__(256) void k_op_many(ManyArgs a) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tb = 1ull << a.t0;
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < a.units; u += step) {
        uint64_t i = u;
        for (int k = 0; k < a.nfix; ++k) {
            const uint64_t lo = i & ((1ull << a.fix[k]) - 1ull);
            i = ((i ^ lo) << 1) | lo;
        }
        i |= a.setmask;
        if (a.kind == K_M1) {
            double2 v0 = a.st[i], v1 = a.st[i | tb];
            m1_pair(a.sub, a.m0, a.m1, a.m2, a.m3, v0, v1);
            a.st[i] = v0;
            a.st[i | tb] = v1;
        } else {
            const int bit = (int)((i >> a.t0) & 1ull);
            a.st[i] = diag_apply(a.sub, a.d0_one, a.m0, a.m1, bit, a.st[i]);
        }
    }
}

static void launch_op_many(double2* st, int n, uint64_t batch, const Op& op, hipStream_t s,
                           Timer* tm, double bytes) {
    ManyArgs a{};
    a.t0 = op.t0;
    a.kind = op.kind;
    a.sub = op.sub;
    a.d0_one = op.d0_one ? 1 : 0;
    a.m0 = make_double2(op.m[0], op.m[1]);
    a.m1 = make_double2(op.m[2], op.m[3]);
    a.m2 = make_double2(op.m[4], op.m[5]);
    a.m3 = make_double2(op.m[6], op.m[7]);
    uint64_t fixmask = op.cmask;
    a.setmask = op.cmask;
    if (op.kind == K_M1) fixmask |= 1ull << op.t0;
    if (op.kind == K_DIAG && op.d0_one) {
        fixmask |= 1ull << op.t0;
        a.setmask |= 1ull << op.t0;
    }
    for (int q = 0; q < n; ++q)
        if ((fixmask >> q) & 1ull) a.fix[a.nfix++] = q;
    TimedLaunch tl(tm, "op_many", bytes, s);
    for (uint64_t b = 0; b < batch; ++b) {
        a.st = st + (b << n);
        a.units = 1ull << (n - a.nfix);
        const uint64_t blocks = std::min<uint64_t>((a.units + 255) / 256, 256ull * 64);
        hipLaunchKernelGGL(k_op_many, dim3((unsigned)blocks), dim3(256), 0, s, a);
        QSIM_HIPCHK(hipGetLastError());
    }
}

// ---------------------------------------------------------------------------------------
// Host: launch
// ---------------------------------------------------------------------------------------
static void add_fix(GArgs& a, int pos) {
    if (a.nfix >= 3) fail(QSIM_ERR_RUNTIME, "internal: more than 3 fixed high positions");
    int i = a.nfix++;
    a.fix[i] = pos;
    while (i > 0 && a.fix[i - 1] > a.fix[i]) {
        std::swap(a.fix[i - 1], a.fix[i]);
        --i;
    }
}

// Launch-shape knobs (defaults from MI355X sweeps, DESIGN.md §per-gate kernels); overridable by
// QSIM_SLICE_U / QSIM_LANE_U / QSIM_DIAG_U (wave-items in flight per lane) and QSIM_NT (0/1:
// non-temporal HBM loads/stores) for tuning runs.
// Far-partner slice targets (QSIM_SLICE_FAR_LO..HI, default 20..25: the pair's two 1 KiB runs
// 16-512 MiB apart) stream slower (0.70-0.72 of 8 TB/s at 28 qubits vs 0.74-0.84 for the
// others); on states of >= QSIM_SLICE_FAR_MIN_QUBITS (24) they run QSIM_SLICE_FAR_MODE 2 (each
// wave takes QSIM_SLICE_U_FAR = 2 consecutive items, the |0> runs' loads before the |1> runs').
// Round-4 measurements (profiles/r04/w1q/): W-1Q 28q mean 0.7652 with this choice, 0.7613 with
// round 3's (mode 0, 4 items), 0.7519 with the far range widened to targets >= 14; no variant
// lifts targets 20-25 above 0.72.
// Work-group order (QSIM_SLICE_BMAP, QSIM_SLICE_FAR_BMAP for the far targets; default 1, round 6):
// work-groups are dispatched round-robin over the 8 XCDs, so with the natural order all eight
// stream the same region at once; mode 1 gives each XCD one contiguous eighth of the items (2: the
// two halves alternate).  28 qubits (profiles/r06/w1q/): targets 20-25 0.71 -> 0.74-0.755, lane
// targets 0-5 0.76 -> 0.81, W-1Q 0.763 -> 0.787 of 8 TB/s.
struct Tune {
    int slice_u = 1, lane_u = 2, diag_u = 2;
    int slice_u_far = 2, far_lo = 20, far_hi = 25, far_mode = 2, far_min_n = 24, far_bmap = 1, bmap = 1;
    bool nt = true;
    Tune() {
        auto env = [](const char* k, int d) {
            const char* v = std::getenv(k);
            return v ? std::atoi(v) : d;
        };
        slice_u = env("QSIM_SLICE_U", slice_u);
        slice_u_far = env("QSIM_SLICE_U_FAR", slice_u_far);
        far_lo = env("QSIM_SLICE_FAR_LO", far_lo);
        far_hi = env("QSIM_SLICE_FAR_HI", far_hi);
        far_mode = env("QSIM_SLICE_FAR_MODE", far_mode);
        far_min_n = env("QSIM_SLICE_FAR_MIN_QUBITS", far_min_n);
        far_bmap = env("QSIM_SLICE_FAR_BMAP", far_bmap);
        bmap = env("QSIM_SLICE_BMAP", bmap);
        lane_u = env("QSIM_LANE_U", lane_u);
        diag_u = env("QSIM_DIAG_U", diag_u);
        nt = env("QSIM_NT", nt ? 1 : 0) != 0;
    }
};
static const Tune& tune() {
    static const Tune t;
    return t;
}

template <typename K>
static void go(K kernel, const GArgs& a, int U, hipStream_t s, const TimedLaunch* tl = nullptr) {
    const uint64_t per_block = 4ull * U;
    const uint64_t blocks = (a.items + per_block - 1) / per_block;
    if (blocks == 0) return;
    if (blocks > 0x7fffffffull) fail(QSIM_ERR_RUNTIME, "grid too large");
    if (tl && tl->start())  // profiled: the launch times itself (no marker packets)
        hipExtLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, s, tl->start(), tl->stop(), 0, a);
    else
        hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
    QSIM_HIPCHK(hipGetLastError());
}

void launch_op(double2* st, int n, uint64_t batch, const Op& op, hipStream_t s, Timer* tm) {
    {
        // fixed high positions the wave-item kernels would need: high controls + the target
        // (M1 / one-sided DIAG with t0 >= 6) or both SWAP qubits; more than 3 -> general kernel
        int high = __builtin_popcountll(op.cmask >> 6 << 6);
        if ((op.kind == K_M1 || (op.kind == K_DIAG && op.d0_one)) && op.t0 >= 6) ++high;
        if (op.kind == K_SWAP && op.cmask)
            fail(QSIM_ERR_INVALID_ARGUMENT, "controlled SWAP is not supported");
        if (high > 3 && op.kind != K_SWAP) {
            launch_op_many(st, n, batch, op, s, tm,
                           op_alg_bytes(op, std::ldexp(1.0, n) * (double)batch));
            return;
        }
    }
    GArgs a{};
    a.st = st;
    a.stride = 1ull << n;
    a.sub = op.sub;
    a.d0_one = op.d0_one ? 1 : 0;
    a.m0 = make_double2(op.m[0], op.m[1]);
    a.m1 = make_double2(op.m[2], op.m[3]);
    a.m2 = make_double2(op.m[4], op.m[5]);
    a.m3 = make_double2(op.m[6], op.m[7]);
    a.t0 = op.t0;
    a.t1 = op.t1;
    a.nlanes = n >= 6 ? 64 : (1 << n);
    for (int q = 0; q < n; ++q) {
        if (!((op.cmask >> q) & 1ull)) continue;
        if (q < 6) a.lane_ctrl |= 1u << q;
        else {
            add_fix(a, q);
            a.setmask |= 1ull << q;
        }
    }
    const double bytes = op_alg_bytes(op, (double)a.stride * (double)batch);
    const int nlow = n >= 6 ? n - 6 : 0;  // index bits above the lane bits
    auto finish = [&]() {
        const int lb = nlow - a.nfix;
        a.log_ipt = lb;
        a.ipt_mask = (1ull << lb) - 1ull;
        a.items = batch << lb;
    };
    const Tune& T = tune();
    a.bmap = T.bmap;
#define QSIM_GO_U(KERNEL, UVAL, CHOICES)                                            \
    do {                                                                            \
        const int u_ = (UVAL);                                                      \
        if (T.nt) {                                                                 \
            CHOICES(KERNEL, true)                                                   \
        } else {                                                                    \
            CHOICES(KERNEL, false)                                                  \
        }                                                                           \
    } while (0)
#define QSIM_U248(KERNEL, NTV)                                                      \
    if (u_ <= 1) go(KERNEL<1, NTV>, a, 1, s, &tl);                                  \
    else if (u_ <= 2) go(KERNEL<2, NTV>, a, 2, s, &tl);                             \
    else if (u_ <= 4) go(KERNEL<4, NTV>, a, 4, s, &tl);                             \
    else go(KERNEL<8, NTV>, a, 8, s, &tl);
    switch (op.kind) {
        case K_M1:
            if (op.t0 >= 6) {
                add_fix(a, op.t0);
                finish();
                TimedLaunch tl(tm, "m1_slice", bytes, s, true);
                const bool far = op.t0 >= T.far_lo && op.t0 <= T.far_hi && n >= T.far_min_n;
                a.bmap = far ? T.far_bmap : T.bmap;
                if (far && T.far_mode == 1) {
                    QSIM_GO_U(k_m1_slice_g, T.slice_u_far, QSIM_U248);
                } else if (far && T.far_mode == 2) {
                    QSIM_GO_U(k_m1_slice_c, T.slice_u_far, QSIM_U248);
                } else {
                    QSIM_GO_U(k_m1_slice, far ? T.slice_u_far : T.slice_u, QSIM_U248);
                }
            } else {
                finish();
                TimedLaunch tl(tm, "m1_lane", bytes, s, true);
                QSIM_GO_U(k_m1_lane, T.lane_u, QSIM_U248);
            }
            break;
        case K_DIAG:
            if (op.t0 >= 6 && op.d0_one) {
                add_fix(a, op.t0);
                a.setmask |= 1ull << op.t0;
            }
            finish();
            {
                TimedLaunch tl(tm, "diag", bytes, s, true);
                QSIM_GO_U(k_diag, T.diag_u, QSIM_U248);
            }
            break;
        case K_SWAP:
            if (op.t0 >= 6) {
                add_fix(a, op.t0);
                add_fix(a, op.t1);
                finish();
                TimedLaunch tl(tm, "swap_hh", bytes, s, true);
                go(k_swap_hh<4>, a, 4, s, &tl);
            } else if (op.t1 >= 6) {
                add_fix(a, op.t1);
                finish();
                TimedLaunch tl(tm, "swap_lh", bytes, s, true);
                go(k_swap_lh<4>, a, 4, s, &tl);
            } else {
                finish();
                TimedLaunch tl(tm, "swap_ll", bytes, s, true);
                go(k_swap_ll<8>, a, 8, s, &tl);
            }
            break;
        default: fail(QSIM_ERR_RUNTIME, "bad op kind");
    }
}

// ---------------------------------------------------------------------------------------
// General two-qubit matrix (the k = 2 case of applyMatrix; the reference
// only has the 2x2 applyGate1Q_opt, include/OptimizedGates.cuh:91-93).  One thread per group of
// four amplitudes {b1 b0} (b0 = bit q0, b1 = bit q1) of the control == 1 subspace; the group
// index is spread over the other bits by zero insertion (fix[] ascending: q0, q1, controls).
// ---------------------------------------------------------------------------------------
struct M2Args {
    double2* st;
    uint64_t groups;
    uint64_t setmask;  // control bits forced to 1
    int nfix;
    int fix[8];
    int q0, q1;
    double2 m[16];     // row-major 4x4 on index (b1 << 1) | b0
};

__global__ __launch_bounds__(256) void k_m2(M2Args a) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.groups; g += step) {
        uint64_t i = g;
        for (int k = 0; k < a.nfix; ++k) {
            const uint64_t lo = i & ((1ull << a.fix[k]) - 1ull);
            i = ((i ^ lo) << 1) | lo;
        }
        i |= a.setmask;
        const uint64_t b0 = 1ull << a.q0, b1 = 1ull << a.q1;
        const uint64_t idx[4] = {i, i | b0, i | b1, i | b0 | b1};
        double2 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = a.st[idx[k]];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = cadd(acc, cmul(a.m[4 * r + k], v[k]));
            a.st[idx[r]] = acc;
        }
    }
}

void launch_matrix2q(double2* st, int n, int q0, int q1, const double* m, uint64_t cmask,
                     hipStream_t s, Timer* tm) {
    M2Args a{};
    a.st = st;
    a.q0 = q0;
    a.q1 = q1;
    for (int k = 0; k < 16; ++k) a.m[k] = make_double2(m[2 * k], m[2 * k + 1]);
    int pos[8], np = 0;
    pos[np++] = q0;
    pos[np++] = q1;
    for (int q = 0; q < n; ++q)
        if ((cmask >> q) & 1ull) {
            if (np == 8) fail(QSIM_ERR_INVALID_ARGUMENT, "at most 6 controls");
            pos[np++] = q;
            a.setmask |= 1ull << q;
        }
    std::sort(pos, pos + np);
    a.nfix = np;
    for (int k = 0; k < np; ++k) a.fix[k] = pos[k];
    a.groups = 1ull << (n - np);
    const uint64_t blocks = std::min<uint64_t>((a.groups + 255) / 256, 256ull * 32);
    TimedLaunch tl(tm, "matrix2q", 64.0 * (double)a.groups, s);
    hipLaunchKernelGGL(k_m2, dim3((unsigned)blocks), dim3(256), 0, s, a);
    QSIM_HIPCHK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// General k-qubit matrix, k <= 8 (SURVEY §8(f) rank 3 "k-qubit unitary with controls"; the
// reference stops at the 2x2 applyGate1Q_opt, src/OptimizedGates.cu:165-183).  A workgroup of 256
// threads holds 256 / 2^k groups of 2^k amplitudes in LDS; thread (group, r) loads amplitude r of
// its group, then computes output row r = sum_c M[r][c] v[c] from LDS (broadcast reads) and the
// transposed matrix mt[c][r] (consecutive lanes read consecutive entries; the matrix stays in
// L2), and stores it in place.  Each group is the control == 1 subspace of one assignment of the
// other qubits (zero insertion at the sorted target + control positions).
// ---------------------------------------------------------------------------------------
struct MkArgs {
    double2* st;
    const double2* mt;   // transposed matrix: mt[c * 2^k + r] = M[r][c]
    uint64_t groups;
    uint64_t setmask;    // control bits forced to 1
    int k, nfix;
    int fix[64];         // ascending target + control positions
    int tq[8];           // target qubit of matrix-index bit j
};

__global__ __launch_bounds__(256) void k_mk(MkArgs a) {
    __shared__ double2 v[256];
    const int dim = 1 << a.k;
    const int gpb = 256 >> a.k;  // groups per block
    const int t = threadIdx.x;
    const int lg = t >> a.k, r = t & (dim - 1);
    for (uint64_t g0 = (uint64_t)blockIdx.x * gpb; g0 < a.groups; g0 += (uint64_t)gridDim.x * gpb) {
        const uint64_t g = g0 + (uint64_t)lg;
        const bool live = g < a.groups;
        uint64_t idx = 0;
        if (live) {
            uint64_t i = g;
            for (int q = 0; q < a.nfix; ++q) {
                const uint64_t lo = i & ((1ull << a.fix[q]) - 1ull);
                i = ((i ^ lo) << 1) | lo;
            }
            idx = i | a.setmask;
            for (int j = 0; j < a.k; ++j)
                if ((r >> j) & 1) idx |= 1ull << a.tq[j];
            v[t] = a.st[idx];
        }
        __syncthreads();
        if (live) {
            double2 acc = make_double2(0.0, 0.0);
            const double2* grp = v + (lg << a.k);
            for (int c = 0; c < dim; ++c) acc = cadd(acc, cmul(a.mt[(uint64_t)c * dim + r], grp[c]));
            a.st[idx] = acc;
        }
        __syncthreads();
    }
}

void launch_matrixk(double2* st, int n, const int* targets, int k, const double2* d_mt,
                    uint64_t cmask, hipStream_t s, Timer* tm) {
    if (k < 1 || k > 8) fail(QSIM_ERR_INVALID_ARGUMENT, "matrix must act on 1 to 8 qubits");
    MkArgs a{};
    a.st = st;
    a.mt = d_mt;
    a.k = k;
    a.setmask = cmask;
    uint64_t fixed = cmask;
    for (int j = 0; j < k; ++j) {
        a.tq[j] = targets[j];
        fixed |= 1ull << targets[j];
    }
    for (int q = 0; q < n; ++q)
        if ((fixed >> q) & 1ull) a.fix[a.nfix++] = q;
    if (a.nfix > n) fail(QSIM_ERR_INVALID_ARGUMENT, "too many fixed qubits");
    a.groups = 1ull << (n - a.nfix);
    const uint64_t gpb = 256ull >> k;
    const uint64_t blocks = std::min<uint64_t>((a.groups + gpb - 1) / gpb, 256ull * 64);
    TimedLaunch tl(tm, "matrixk", 32.0 * (double)(a.groups << k), s);
    hipLaunchKernelGGL(k_mk, dim3((unsigned)blocks), dim3(256), 0, s, a);
    QSIM_HIPCHK(hipGetLastError());
}

}  // namespace qsim_hip
