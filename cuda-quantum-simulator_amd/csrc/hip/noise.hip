// noise.hip — single-trajectory Monte-Carlo noise (reference NoisySimulator,
// include/NoiseModel.cuh:139-214, src/NoiseModel.cu:115-314, 369-577).
//
// Semantics kept from the reference kernels: after every gate, every channel entry
// (type, qubit, p) runs one pass over the 2^(n-1) amplitude PAIRS of its qubit, and each pair
// draws its own uniform(s) (src/NoiseModel.cu:122-126): X / Z / Y / depolarizing flips act on
// the pairs whose draw falls below p, amplitude / phase damping pick a Kraus branch per pair from
// the pair's own |a1|^2 and renormalise the pair (:224-314).  Global channels (empty qubit list)
// act on no qubit (:490-494).
//
// MI355X design: no per-pair curandState array (48 B x 2^(n-1), read and written by every noise
// kernel of the reference).  A pair's uniforms come from a stateless counter hash of
// (seed, noise-pass counter, pair index), so a flip pass costs only the pairs it modifies (the
// lanes whose draw fires issue the loads; p = 0.01 touches ~1 % of the state) and a damping pass
// streams the pairs once.  Realisations differ from cuRAND XORWOW (parity unpinned);
// the per-pair distribution is the reference's: float uniform in (0, 1] (curand_uniform's range),
// thresholds 1/3 and 2/3 as floats.  oracle/numpy_oracle.py restates the same hash for exact tests.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "engine.hpp"
#include "qsim_hip.h"

namespace qsim_hip {

__device__ __forceinline__ uint64_t nz_mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static uint64_t nz_mix_host(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// float in (0, 1] from the top 24 bits
__device__ __forceinline__ float nz_uniform(uint64_t h) {
    return (float)((uint32_t)(h >> 40) + 1u) * (1.0f / 16777216.0f);
}

struct NArgs {
    double2* st;
    uint64_t pairs;  // B x 2^(n-1): pair idx of trajectory t is t * 2^(n-1) + its index in t
    int log_ppt;     // n - 1
    uint64_t key;    // noise_key(seed, counter)
    uint64_t idx0;   // global pair index of local pair 0 (trajectory-sharded ensembles)
    int target;
    double p;
};

template <int TYPE>
__global__ __launch_bounds__(256) void k_noise(NArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t mask = (1ull << a.target) - 1ull;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < a.pairs; idx += stride) {
        const uint64_t h = nz_mix(a.key ^ nz_mix(a.idx0 + idx));
        const float r1 = nz_uniform(h);
        // reference idx -> (traj, pair_idx) split (src/NoiseModel.cu:843-856); batch 1: traj 0
        const uint64_t traj = idx >> a.log_ppt, pr = idx & ((1ull << a.log_ppt) - 1ull);
        const uint64_t i0 = (traj << (a.log_ppt + 1)) | (pr & mask) | ((pr & ~mask) << 1);
        const uint64_t i1 = i0 | (1ull << a.target);
        if constexpr (TYPE == 0 || TYPE == 3 || TYPE == 4 || TYPE == 5) {  // Pauli flips
            if (!((double)r1 < a.p)) continue;  // float draw vs double p, as the reference (:195)
            int pauli = TYPE == 3 ? 1 : (TYPE == 4 ? 3 : 2);  // 1 X, 2 Y, 3 Z
            if constexpr (TYPE == 0) {                         // depolarizing (:191-216)
                const float r2 = nz_uniform(nz_mix(h ^ 0x5bd1e9955bd1e995ull));
                pauli = r2 < 1.0f / 3.0f ? 1 : (r2 < 2.0f / 3.0f ? 2 : 3);
            }
            if (pauli == 3) {
                const double2 v = a.st[i1];
                a.st[i1] = make_double2(-v.x, -v.y);
            } else {
                const double2 a0 = a.st[i0], a1 = a.st[i1];
                if (pauli == 1) {
                    a.st[i0] = a1;
                    a.st[i1] = a0;
                } else {  // Y = [[0, -i], [i, 0]] (:177-178)
                    a.st[i0] = make_double2(a1.y, -a1.x);
                    a.st[i1] = make_double2(-a0.y, a0.x);
                }
            }
        } else if constexpr (TYPE == 1) {  // amplitude damping (:224-269)
            const double2 a0 = a.st[i0], a1 = a.st[i1];
            const double g = a.p;
            const double p1 = a1.x * a1.x + a1.y * a1.y;
            const double n0 = a0.x * a0.x + a0.y * a0.y;
            if (r1 < p1 * g) {
                const double nrm = sqrt(n0 + g * p1);
                if (nrm > 1e-15) {
                    const double sg = sqrt(g);
                    a.st[i0] = make_double2((a0.x + sg * a1.x) / nrm, (a0.y + sg * a1.y) / nrm);
                    a.st[i1] = make_double2(0.0, 0.0);
                }
            } else {
                const double s1 = sqrt(1.0 - g);
                const double nrm = sqrt(n0 + (1.0 - g) * p1);
                if (nrm > 1e-15) {
                    a.st[i0] = make_double2(a0.x / nrm, a0.y / nrm);
                    a.st[i1] = make_double2(s1 * a1.x / nrm, s1 * a1.y / nrm);
                }
            }
        } else {  // phase damping (:274-314)
            const double2 a1 = a.st[i1];
            const double g = a.p;
            const double p1 = a1.x * a1.x + a1.y * a1.y;
            if (r1 < g * p1) {
                a.st[i0] = make_double2(0.0, 0.0);
                if (p1 > 1e-15) {
                    const double nrm = sqrt(p1);
                    a.st[i1] = make_double2(a1.x / nrm, a1.y / nrm);
                }
            } else {
                const double2 a0 = a.st[i0];
                const double s1 = sqrt(1.0 - g);
                const double ns = a0.x * a0.x + a0.y * a0.y + (1.0 - g) * p1;
                if (ns > 1e-15) {
                    const double nrm = sqrt(ns);
                    a.st[i0] = make_double2(a0.x / nrm, a0.y / nrm);
                    a.st[i1] = make_double2(s1 * a1.x / nrm, s1 * a1.y / nrm);
                }
            }
        }
    }
}

uint64_t noise_key(uint64_t seed, uint64_t counter) {
    return nz_mix_host(nz_mix_host(seed) ^ (counter * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull));
}

void launch_noise(double2* st, int n, int type, int qubit, double p, uint64_t seed,
                  uint64_t counter, hipStream_t s, Timer* tm, uint64_t batch, uint64_t traj0) {
    if (type < 0 || type > 5) fail(QSIM_ERR_INVALID_ARGUMENT, "unknown noise type");
    if (qubit < 0 || qubit >= n)
        fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(qubit) + " out of range");
    if (!std::isfinite(p)) fail(QSIM_ERR_INVALID_ARGUMENT, "noise probability must be finite");
    NArgs a{};
    a.st = st;
    a.pairs = batch << (n - 1);
    a.log_ppt = n - 1;
    a.key = noise_key(seed, counter);
    a.idx0 = traj0 << (n - 1);
    a.target = qubit;
    a.p = p;
    const uint64_t blocks = std::min<uint64_t>((a.pairs + 255) / 256, 256ull * 32);
    // algorithmic bytes: damping streams every pair (32 B); a flip touches ~p of the pairs
    const double pairs = (double)a.pairs;
    const double bytes = (type == 1 || type == 2) ? 32.0 * pairs
                                                  : 32.0 * pairs * std::min(1.0, std::max(0.0, p));
    TimedLaunch tl(tm, "noise", bytes, s);
    switch (type) {
        case 0: hipLaunchKernelGGL(k_noise<0>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
        case 1: hipLaunchKernelGGL(k_noise<1>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL(k_noise<2>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
        case 3: hipLaunchKernelGGL(k_noise<3>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(k_noise<4>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL(k_noise<5>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    }
    QSIM_HIPCHK(hipGetLastError());
}

}  // namespace qsim_hip
