// fused.hip — LDS-tiled multi-gate passes (the gates/s lever) and their host planner.
//
// The reference applies one kernel per gate (src/Simulator.cu:28-154), so every gate is a full
// HBM round trip of the state.  Here a pass streams the state once: each 256-thread workgroup
// owns a tile of 64 << h amplitudes spanning qubits {0..5} (the 64 lanes, 1 KiB contiguous
// runs) plus h chosen high qubits, stages it in LDS (64 KiB at h = 6, two workgroups per CU),
// applies every planned gate whose qubits lie inside the tile, and writes it back.  HBM traffic
// per pass is 32 B x 2^n, independent of how many gates the pass absorbs.
//
// The host planner walks the circuit in order and moves a gate into the current pass when its
// qubits fit the tile and it shares no qubit with an earlier gate that was deferred (gates on
// disjoint qubits commute exactly, so the product is unchanged).  Semantics of each gate are
// the per-gate kernels' (device_ops.hpp), i.e. src/Gates.cu:31-410.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <set>

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

Plan plan_fused(const std::vector<Op>& ops, int n, int hmax) {
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
        p.op_begin = (int)plan.ops.size();
        for (const Op& op : in_pass) {
            TileOp t{};
            t.kind = op.kind;
            t.sub = op.sub;
            t.b0 = bit_of[op.t0];
            t.b1 = op.kind == K_SWAP ? bit_of[op.t1] : -1;
            if (t.kind == K_SWAP && t.b0 > t.b1) std::swap(t.b0, t.b1);
            t.cmask = 0;
            for (int q = 0; q < n; ++q)
                if ((op.cmask >> q) & 1ull) t.cmask |= 1u << bit_of[q];
            t.d0_one = op.d0_one ? 1 : 0;
            for (int i = 0; i < 8; ++i) t.m[i] = op.m[i];
            plan.ops.push_back(t);
            plan.order.push_back(op.src);
        }
        p.op_end = (int)plan.ops.size();
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
    uint64_t stride;     // 2^n
    uint64_t tpt_mask;   // tiles per trajectory - 1
    int log_tpt;
    int op_begin, op_end;
    int hpos[8];
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

template <int H>
__global__ __launch_bounds__(256) void k_fused_tile(FArgs a) {
    constexpr int T = 64 << H;                 // amplitudes per tile
    constexpr int R = T >= 256 ? T / 256 : 1;  // loads per thread
    __shared__ double2 tile[T];
    const int tid = threadIdx.x;
    const uint64_t tile_id = blockIdx.x;
    const uint64_t traj = tile_id >> a.log_tpt;
    const uint64_t base =
        traj * a.stride + deposit_h<H>((tile_id & a.tpt_mask) << 6, a.hpos);

    // HBM -> LDS: element j = r*256 + tid; low 6 bits are lanes (1 KiB runs).
    double2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t j = (uint32_t)(r * 256 + tid);
        if (j < (uint32_t)T) v[r] = a.st[base | (j & 63u) | spread<H>(j >> 6, a.hpos)];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t j = (uint32_t)(r * 256 + tid);
        if (j < (uint32_t)T) tile[j] = v[r];
    }
    __syncthreads();

    for (int o = a.op_begin; o < a.op_end; ++o) {
        const TileOp& op = a.ops[o];
        const int kind = op.kind, sub = op.sub, b0 = op.b0;
        const uint32_t cm = op.cmask;
        if (kind == K_M1) {
            const double2 m0 = make_double2(op.m[0], op.m[1]), m1 = make_double2(op.m[2], op.m[3]);
            const double2 m2 = make_double2(op.m[4], op.m[5]), m3 = make_double2(op.m[6], op.m[7]);
            for (uint32_t p = tid; p < (uint32_t)T / 2; p += 256) {
                const uint32_t j0 = ins0(p, b0), j1 = j0 | (1u << b0);
                if ((j0 & cm) == cm) {
                    double2 x0 = tile[j0], x1 = tile[j1];
                    m1_pair(sub, m0, m1, m2, m3, x0, x1);
                    tile[j0] = x0;
                    tile[j1] = x1;
                }
            }
        } else if (kind == K_DIAG) {
            const double2 d0 = make_double2(op.m[0], op.m[1]), d1 = make_double2(op.m[2], op.m[3]);
            const int d0_one = op.d0_one;
            if (d0_one) {  // only the target==1 half, enumerated directly
                for (uint32_t p = tid; p < (uint32_t)T / 2; p += 256) {
                    const uint32_t j = ins0(p, b0) | (1u << b0);
                    if ((j & cm) == cm) tile[j] = diag1(sub, d1, tile[j]);
                }
            } else {
                for (uint32_t j = tid; j < (uint32_t)T; j += 256)
                    if ((j & cm) == cm)
                        tile[j] = diag_apply(sub, 0, d0, d1, (j >> b0) & 1u, tile[j]);
            }
        } else {  // K_SWAP, b0 < b1
            const int b1 = op.b1;
            for (uint32_t p = tid; p < (uint32_t)T / 4; p += 256) {
                const uint32_t j = ins0(ins0(p, b0), b1);
                const uint32_t ja = j | (1u << b1), jb = j | (1u << b0);
                if ((j & cm) == cm) {
                    const double2 xa = tile[ja], xb = tile[jb];
                    tile[ja] = xb;
                    tile[jb] = xa;
                }
            }
        }
        __syncthreads();
    }

#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t j = (uint32_t)(r * 256 + tid);
        if (j < (uint32_t)T) a.st[base | (j & 63u) | spread<H>(j >> 6, a.hpos)] = tile[j];
    }
}

void launch_fused(double2* st, int n, uint64_t batch, const Plan& plan, const TileOp* d_ops,
                  hipStream_t s, Timer* tm) {
    const double pass_bytes = 32.0 * (double)(1ull << n) * (double)batch;
    for (const FusedPass& p : plan.passes) {
        if (p.single >= 0) {
            launch_op(st, n, batch, plan.singles[p.single], s, tm);
            continue;
        }
        FArgs a{};
        a.st = st;
        a.ops = d_ops;
        a.stride = 1ull << n;
        a.op_begin = p.op_begin;
        a.op_end = p.op_end;
        for (int i = 0; i < 8; ++i) a.hpos[i] = p.hpos[i];
        const int lt = n - 6 - p.h;
        a.log_tpt = lt;
        a.tpt_mask = (1ull << lt) - 1ull;
        const uint64_t blocks = batch << lt;
        TimedLaunch tl(tm, "fused_tile", pass_bytes, s);
        switch (p.h) {
#define QSIM_FUSED_CASE(HH) \
    case HH: hipLaunchKernelGGL(k_fused_tile<HH>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
            QSIM_FUSED_CASE(0)
            QSIM_FUSED_CASE(1)
            QSIM_FUSED_CASE(2)
            QSIM_FUSED_CASE(3)
            QSIM_FUSED_CASE(4)
            QSIM_FUSED_CASE(5)
            QSIM_FUSED_CASE(6)
#undef QSIM_FUSED_CASE
            default: fail(QSIM_ERR_RUNTIME, "unsupported tile height");
        }
        QSIM_HIPCHK(hipGetLastError());
    }
}

}  // namespace qsim_hip
