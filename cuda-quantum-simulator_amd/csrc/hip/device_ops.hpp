// device_ops.hpp — device-side arithmetic shared by the per-gate, fused-tile and batched
// kernels.  Complex amplitudes are HIP double2 {x = re, y = im}, 16 B, so one lane moves one
// amplitude with one global_load/store_dwordx4.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine.hpp"

namespace qsim_hip {

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) {
    return make_double2(a.x + b.x, a.y + b.y);
}

// Insert a zero bit at each of the `nfix` ascending positions `fix[]` of k.
__device__ __forceinline__ uint64_t deposit(uint64_t k, int nfix, const int* fix) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < nfix) {
            const uint64_t lo = k & ((1ull << fix[i]) - 1ull);
            k = ((k ^ lo) << 1) | lo;
        }
    }
    return k;
}

// 2x2 update of a pair (a0 = amplitude with target bit 0, a1 = target bit 1).
// S_X/S_Y/S_H reproduce src/Gates.cu:31-104 exactly; S_GEN is [[m0,m1],[m2,m3]].
__device__ __forceinline__ void m1_pair(int sub, double2 m0, double2 m1, double2 m2, double2 m3,
                                        double2& a0, double2& a1) {
    double2 n0, n1;
    if (sub == S_X) {
        n0 = a1;
        n1 = a0;
    } else if (sub == S_Y) {
        n0 = make_double2(a1.y, -a1.x);
        n1 = make_double2(-a0.y, a0.x);
    } else if (sub == S_H) {
        const double c = kInvSqrt2;
        n0 = make_double2((a0.x + a1.x) * c, (a0.y + a1.y) * c);
        n1 = make_double2((a0.x - a1.x) * c, (a0.y - a1.y) * c);
    } else {
        n0 = cadd(cmul(m0, a0), cmul(m1, a1));
        n1 = cadd(cmul(m2, a0), cmul(m3, a1));
    }
    a0 = n0;
    a1 = n1;
}

// One side of a 2x2 update when the partner amplitude lives in another lane: `self` has target
// bit `bit`, `other` is the partner.  Same arithmetic as m1_pair.
__device__ __forceinline__ double2 m1_half(int sub, double2 m0, double2 m1, double2 m2, double2 m3,
                                           int bit, double2 self, double2 other) {
    double2 a0 = bit ? other : self;
    double2 a1 = bit ? self : other;
    m1_pair(sub, m0, m1, m2, m3, a0, a1);
    return bit ? a1 : a0;
}

// Diagonal phase on the |1> side (Gates.cu:65-175 closed forms) or general d1.
__device__ __forceinline__ double2 diag1(int sub, double2 d1, double2 a) {
    const double c = kInvSqrt2;
    switch (sub) {
        case S_NEG: return make_double2(-a.x, -a.y);
        case S_I: return make_double2(-a.y, a.x);
        case S_MI: return make_double2(a.y, -a.x);
        case S_T: return make_double2((a.x - a.y) * c, (a.x + a.y) * c);
        case S_TDG: return make_double2((a.x + a.y) * c, (-a.x + a.y) * c);
        default: return cmul(d1, a);
    }
}
__device__ __forceinline__ double2 diag_apply(int sub, int d0_one, double2 d0, double2 d1, int bit,
                                              double2 a) {
    if (bit) return diag1(sub, d1, a);
    return d0_one ? a : cmul(d0, a);
}

// Streaming HBM access: in a per-gate kernel or a fused pass every amplitude is read and written
// exactly once, so the non-temporal forms (no cache retention) are selectable per launch.
typedef double dv2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 ld(const double2* p) {
    if constexpr (NT) {
        const dv2 t = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p));
        return make_double2(t.x, t.y);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void st(double2* p, double2 v) {
    if constexpr (NT) {
        dv2 t;
        t.x = v.x;
        t.y = v.y;
        __builtin_nontemporal_store(t, reinterpret_cast<dv2*>(p));
    } else {
        *p = v;
    }
}

// Wave-uniform read of a read-only launch table (fused-pass ops, stages).  Through the constant
// address space the compiler emits scalar s_load into SGPRs (waited on lgkmcnt); a plain global
// read of the same data becomes a vector load whose s_waitcnt vmcnt(0) also drains every
// outstanding HBM load/store of the wave — one L2 round trip per op per tile.
template <class T>
__device__ __forceinline__ T ldc(const T* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) T* CP;
    return *((CP)(p) + i);
#else  // host pass of the single-source compile: never executed
    return p[i];
#endif
}

// 64-bit-lane shuffle of a complex amplitude (two ds_bpermute per double).
__device__ __forceinline__ double2 shfl_xor2(double2 v, int mask) {
    return make_double2(__shfl_xor(v.x, mask), __shfl_xor(v.y, mask));
}

}  // namespace qsim_hip
