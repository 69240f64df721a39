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
// kernel of the reference).  Damping passes: a pair's uniform comes from a stateless counter hash
// of (seed, noise-pass counter, pair index) and the pass streams the pairs once.  Flip passes
// (X / Z / Y / depolarizing) do work in proportion to the flips, not the pairs: the global pair
// index space is cut into blocks of 256 pairs, and one thread per block walks its flips with
// geometric gaps (gap = floor(log u / log(1 - P)), P = the exact probability that the
// reference's float uniform in (0, 1] falls below the double p), drawing each flip's Pauli as
// the reference does (float uniform vs 1/3f, 2/3f).  Every pair still flips independently with
// probability P — the reference's per-pair distribution — at p = 0.01 a pass costs ~1 % of the
// hashes.  Realisations differ from cuRAND XORWOW (parity unpinned);
// oracle/numpy_oracle.py restates the same streams for exact tests.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "device_ops.hpp"
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

// Flip passes by blocks of kFlipBlock global pairs: one thread walks one block's flips (draw k of
// block b: nz_mix(stream_b + k * golden); stream_b = nz_mix(key ^ nz_mix(b ^ kBlockSalt))) and
// applies those inside [lo, hi), the global pairs this launch / work-group owns.
constexpr uint64_t kFlipBlockLog = 8, kFlipBlock = 1ull << kFlipBlockLog;
constexpr uint64_t kBlockSalt = 0xb10c5a17b10c5a17ull;
struct FlipChan {
    uint64_t key;
    double lq;   // log1p(-P)
    int target;
    int type;    // 0 depolarizing, 3 X, 4 Z, 5 Y
    int always;  // P == 1: every pair flips
    float il2;   // ln 2 / lq (the single-precision first try of next_flip; 0: always double)
};
// The geometric gap of draw h: floor(ln u / lq), u = ((h >> 11) + 1) 2^-53 in (0, 1] — in double,
// exactly up to kFlipBlock (a larger value only says "past the block").  *fb (optional): set when
// the single-precision first try could not decide it.
__device__ __forceinline__ double flip_gap(uint64_t h, const FlipChan& c, bool* fb = nullptr) {
    const double u = (double)((h >> 11) + 1ull) * 0x1.0p-53;  // (0, 1]
    // gap = floor(ln u / lq) in double.  First in single precision (the hardware log2):
    // its error bound is tiny next to the distance from the nearest integer except in ~0.1 %
    // of draws (p = 0.01), which take the double path — so the result is always the double
    // one (the flips, hence the states, do not change; qsim_noise_gap_check counts both).
    double gap;
    const float gf = __log2f((float)u) * c.il2;  // (>= 0: log2 u <= 0, il2 < 0)
    // error of gf: |il2| x (rounding of u, <= 2^-24 / ln 2 absolute in log2 u, + the
    // hardware log2's error, ~2^-22 absolute near 1) + |gf| x (its relative error and two
    // roundings, ~2^-22) — bounded here by 2^-17 x |il2| + 2^-20 x |gf| (16x and 4x
    // margins).  The hardware figures are assumptions (v_log_f32 is taken to be within ~1 ulp
    // of log2 of its float input; no ISA accuracy table ships with this image), so the bound is
    // checked, not trusted: random draws (qsim_noise_gap_check, 2^26 per p) and a targeted sweep
    // of every integer boundary of the gap up to the block and of the float-rounding interval
    // around it (qsim_noise_gap_check_edges) must give the double result for every draw
    // (tests/test_batched_refnoise_gpu.py).  The margin is kept tight on purpose: a lane that falls back makes its whole
    // wave run the double log, so at p = 0.01 a 1 % per-lane fallback rate (a 2^-13 x |il2|
    // bound) left most iterations of a 64-lane wave on the slow path; this one is ~0.1 %.
    const float err = fabsf(gf) * 0x1.0p-20f + fabsf(c.il2) * 0x1.0p-17f;
    // decided when both ends of [gf - err, gf + err] have the same floor, or both lie past the
    // block (a walk only needs to know the gap ends it: at p <= 0.001 most draws)
    const float flo = fminf(floorf(gf - err), (float)kFlipBlock), fhi = fminf(floorf(gf + err), (float)kFlipBlock);
    if (c.il2 != 0.0f && flo == fhi) {
        gap = (double)fhi;
    } else {
        gap = floor(log(u) / c.lq);
        if (fb) *fb = true;
    }
    return gap;
}

// Next flip of a block's walk inside [lo, hi): false when the block is exhausted.
struct FlipCursor {
    uint64_t stream, k;
    int64_t pos;
    bool done;
};
__device__ __forceinline__ bool next_flip(FlipCursor& cur, uint64_t b, uint64_t lo, uint64_t hi,
                                          const FlipChan& c, uint64_t& g, uint64_t& h) {
    while (!cur.done) {
        h = nz_mix(cur.stream + cur.k * 0x9e3779b97f4a7c15ull);
        ++cur.k;
        if (c.always) {
            cur.pos += 1;
        } else {
            const double gap = flip_gap(h, c);
            if (gap >= (double)kFlipBlock) {
                cur.done = true;
                break;
            }
            cur.pos += (int64_t)gap + 1;
        }
        if (cur.pos >= (int64_t)kFlipBlock) {
            cur.done = true;
            break;
        }
        g = (b << kFlipBlockLog) + (uint64_t)cur.pos;  // global pair index
        if (g >= lo && g < hi) return true;           // else another shard's pair
    }
    return false;
}

// Walks block b and applies its flips.  (Batching several flips' loads before their stores was
// measured: no change — the launch is bound by random-access memory throughput, not latency.)
// bad (QSIM_NOISE_CHECK, tests): counts accesses outside the caller's pairs [lo, hi).
__device__ __forceinline__ void flip_block(double2* st, uint64_t b, uint64_t lo, uint64_t hi,
                                           uint64_t idx0, int log_ppt, const FlipChan& c,
                                           unsigned int* bad = nullptr) {
    const uint64_t mask = (1ull << c.target) - 1ull;
    FlipCursor cur{nz_mix(c.key ^ nz_mix(b ^ kBlockSalt)), 0, -1, false};
    uint64_t g = 0, h = 0;
    while (next_flip(cur, b, lo, hi, c, g, h)) {
        if (bad && (g < lo || g >= hi)) atomicAdd(bad, 1u);
        int pauli = c.type == 3 ? 1 : (c.type == 4 ? 3 : 2);  // 1 X, 2 Y, 3 Z
        if (c.type == 0) {                                      // depolarizing (:191-216)
            const float r2 = nz_uniform(nz_mix(h ^ 0x5bd1e9955bd1e995ull));
            pauli = r2 < 1.0f / 3.0f ? 1 : (r2 < 2.0f / 3.0f ? 2 : 3);
        }
        // reference idx -> (traj, pair_idx) split (src/NoiseModel.cu:843-856)
        const uint64_t idx = g - idx0;
        const uint64_t traj = idx >> log_ppt, pr = idx & ((1ull << log_ppt) - 1ull);
        const uint64_t i0 = (traj << (log_ppt + 1)) | (pr & mask) | ((pr & ~mask) << 1);
        const uint64_t i1 = i0 | (1ull << c.target);
        if (bad) {  // both amplitudes must belong to trajectories of [lo, hi)
            const uint64_t t_lo = (lo - idx0) >> log_ppt, t_hi = (hi - 1 - idx0) >> log_ppt;
            if ((i0 >> (log_ppt + 1)) < t_lo || (i1 >> (log_ppt + 1)) > t_hi) atomicAdd(bad, 1u);
            atomicAdd(bad + 1, 1u);  // flips applied (coverage)
        }
        if (pauli == 3) {
            const double2 v = st[i1];
            st[i1] = make_double2(-v.x, -v.y);
        } else {
            const double2 a0 = st[i0], a1 = st[i1];
            if (pauli == 1) {
                st[i0] = a1;
                st[i1] = a0;
            } else {  // Y = [[0, -i], [i, 0]] (:177-178)
                st[i0] = make_double2(a1.y, -a1.x);
                st[i1] = make_double2(-a0.y, a0.x);
            }
        }
    }
}

struct FArgsN {
    double2* st;
    uint64_t pairs, idx0;
    int log_ppt;
    FlipChan c;
};
__global__ __launch_bounds__(256) void k_noise_flips(FArgsN a) {
    const uint64_t b0 = a.idx0 >> kFlipBlockLog;
    const uint64_t b1 = (a.idx0 + a.pairs - 1) >> kFlipBlockLog;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = b0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= b1; b += stride)
        flip_block(a.st, b, a.idx0, a.idx0 + a.pairs, a.idx0, a.log_ppt, a.c);
}

// All flip channels that follow one gate, in one launch.  Channel order matters only within a
// trajectory (a pair never spans two), so each work-group owns an aligned unit of 2^log_unit
// global pairs — whole trajectories and whole blocks — and runs the channels in order over it with
// a work-group barrier between channels (its global writes are visible to its own waves after the
// barrier: one CU).  Same draws and the same result as one k_noise_flips launch per channel.
constexpr int kMaxUnitChannels = 32;
struct UArgs {
    double2* st;
    uint64_t pairs, idx0;
    int log_ppt, log_unit, nch;
    int bmap;  // work-group order (QSIM_NOISE_BMAP)
    FlipChan ch[kMaxUnitChannels];
};
// Why this is race-free (the round-2 "batched-load variant" that returned
// wrong states when lanes also walked blocks wholly outside [lo, hi) was never committed and
// cannot be recovered, so the argument is made for this kernel and checked on the device):
//   1. a work-group loads and stores only amplitudes of its own pairs [lo, hi): next_flip
//      filters every flip by [lo, hi) BEFORE flip_block touches memory, so a block outside the
//      range (or the foreign part of a block that straddles a shard boundary) costs hashes only;
//      units are disjoint, so no amplitude has two writers;
//   2. within one channel two flips are two different pairs (positions strictly increase within
//      a block, blocks are disjoint) and the pairs of one target partition the amplitudes, so no
//      two lanes touch the same amplitude;
//   3. between channels the barrier (s_waitcnt vmcnt(0) then s_barrier) retires every lane's
//      stores before any lane's next loads, and the work-group's waves share one CU's L1.
// The failure class left open by the variant's description is a write-back of a loaded value
// for a flip that the range test rejects AFTER the load (a branch-free batched form: load K
// flips, select, store K): that rewrites another work-group's pair with a stale value while its
// owner flips it — exactly "wrong states only when lanes walk blocks outside the range".  This
// kernel has no such store.  QSIM_NOISE_CHECK=1 runs it with every access range-checked on the
// device (violations counted with atomics and turned into an error by the launcher);
// tests/test_batched_refnoise_gpu.py runs that check on units that start and end mid-block.
// Work-group order: 1 gives each of the 8 XCDs (blockIdx mod 8, round-robin dispatch) one
// contiguous eighth of the grid (gates.hip slice_block), 0 the natural order.  QSIM_NOISE_BMAP
// (in-tile gate + noise kernel and the suffix push, default 1: W-BATCH 1.980 -> 1.997 M
// trajectory-gates/s, profiles/r06/xcd_order/); QSIM_PULL_BMAP (the pulled pass, default 0: its
// partner reads hit L2 more when every XCD streams the same region, 1 259 vs 1 193 gates/s).
__device__ __forceinline__ uint64_t xcd_block(int mode) {
    const uint64_t b = blockIdx.x, G = gridDim.x;
    if (mode == 1 && (G & 7ull) == 0ull) return (b & 7ull) * (G >> 3) + (b >> 3);
    return b;
}
static int env_bmap(const char* k, int dflt) {  // (read per launch: tests switch it)
    const char* e = std::getenv(k);
    return e ? std::atoi(e) : dflt;
}

template <bool CHECK>
__global__ __launch_bounds__(256) void k_noise_units(UArgs a, unsigned int* bad) {
    const uint64_t base = ((a.idx0 >> a.log_unit) + xcd_block(a.bmap)) << a.log_unit;
    const uint64_t lo = base > a.idx0 ? base : a.idx0;
    const uint64_t end = a.idx0 + a.pairs, top = base + (1ull << a.log_unit);
    const uint64_t hi = top < end ? top : end;
    // the blocks that overlap [lo, hi)
    const uint64_t b0 = lo >> kFlipBlockLog, nb = ((hi - 1) >> kFlipBlockLog) - b0 + 1;
    for (int c = 0; c < a.nch; ++c) {
        if (c) __syncthreads();
        for (uint64_t j = threadIdx.x; j < nb; j += blockDim.x)
            flip_block(a.st, b0 + j, lo, hi, a.idx0, a.log_ppt, a.ch[c], CHECK ? bad : nullptr);
    }
}

// P(float uniform in (0, 1] < p): the reference compares curand_uniform's (k + 1) / 2^24,
// k uniform in [0, 2^24), with the double p.
double flip_probability(double p) {
    if (!(p > 0.0)) return 0.0;
    const double c = std::ceil(p * 16777216.0) - 1.0;  // #{k : (k + 1) / 2^24 < p}
    return std::min(16777216.0, std::max(0.0, c)) / 16777216.0;
}

// Damping channels: every pair draws (counter hash of the global pair index) and is rewritten.
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
        if constexpr (TYPE == 1) {  // amplitude damping (:224-269)
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

static void check_channel(int n, int type, int qubit, double p) {
    if (type < 0 || type > 5) fail(QSIM_ERR_INVALID_ARGUMENT, "unknown noise type");
    if (qubit < 0 || qubit >= n)
        fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(qubit) + " out of range");
    if (!std::isfinite(p)) fail(QSIM_ERR_INVALID_ARGUMENT, "noise probability must be finite");
}

// false when the channel never fires (P == 0)
static bool flip_channel(int type, int qubit, double p, uint64_t key, FlipChan& c) {
    const double P = flip_probability(p);
    if (P <= 0.0) return false;
    c.key = key;
    c.target = qubit;
    c.type = type;
    c.always = P >= 1.0 ? 1 : 0;
    c.lq = c.always ? -1.0 : std::log1p(-P);
    // (QSIM_NOISE_FAST_LOG=0: the double log for every draw — tests and measurements; read per
    // channel set-up, on the host)
    const char* fe = std::getenv("QSIM_NOISE_FAST_LOG");
    const bool fast = fe == nullptr || std::atoi(fe) != 0;
    c.il2 = fast && !c.always ? (float)(0.69314718055994530942 / c.lq) : 0.0f;
    return true;
}

uint64_t noise_check_flips = 0;  // flips applied by range-checked launches (qsim_noise_check_flips)

void launch_noise_after_gate(double2* st, int n, const std::vector<NoiseChan>& chans, uint64_t seed,
                             uint64_t& counter, hipStream_t s, Timer* tm, uint64_t batch, uint64_t traj0) {
    const int log_ppt = n - 1;
    // whole trajectories, >= 128 blocks of 256 pairs (QSIM_NOISE_UNIT_LOG: experiments, >= n - 1;
    // W-BATCH config 4: two trajectories per work-group, 2^16 pairs — round 5 measured one
    // trajectory faster for the push alone (0.137 vs 0.140 ms, profiles/r05/batch_unit/), but in
    // the two-stream step two are: 1.953-1.958 M -> 1.976-1.982 M trajectory-gates/s over two
    // runs each, four trajectories 1.956 M (r6p run))
    static const int unit_log_env = [] {
        const char* e = std::getenv("QSIM_NOISE_UNIT_LOG");
        return e ? std::atoi(e) : 16;
    }();
    const int log_unit = std::max(log_ppt, unit_log_env);
    const uint64_t pairs = batch << log_ppt, idx0 = traj0 << log_ppt;
    const uint64_t units = ((idx0 + pairs - 1) >> log_unit) - (idx0 >> log_unit) + 1;
    bool flips = true;
    for (const NoiseChan& c : chans) flips = flips && (c.type == 0 || c.type >= 3);
    // QSIM_NOISE_UNIT_MIN (default 128): fewest units for the one-launch path (tests force both)
    const char* e = std::getenv("QSIM_NOISE_UNIT_MIN");
    const uint64_t unit_min = e ? (uint64_t)std::max(1ll, std::atoll(e)) : 128;
    if (!flips || units < unit_min || units > 0x7fffffffull) {  // few work-groups: one launch per channel
        for (const NoiseChan& c : chans)
            launch_noise(st, n, c.type, c.qubit, c.p, seed, counter++, s, tm, batch, traj0);
        return;
    }
    for (size_t c0 = 0; c0 < chans.size(); c0 += kMaxUnitChannels) {
        UArgs u{};
        u.st = st;
        u.bmap = env_bmap("QSIM_NOISE_BMAP", 1);
        u.pairs = pairs;
        u.idx0 = idx0;
        u.log_ppt = log_ppt;
        u.log_unit = log_unit;
        double bytes = 0.0;
        for (size_t c = c0; c < std::min(chans.size(), c0 + kMaxUnitChannels); ++c) {
            const NoiseChan& ch = chans[c];
            check_channel(n, ch.type, ch.qubit, ch.p);
            const uint64_t key = noise_key(seed, counter++);
            if (flip_channel(ch.type, ch.qubit, ch.p, key, u.ch[u.nch])) ++u.nch;
            bytes += 32.0 * (double)pairs * std::min(1.0, std::max(0.0, ch.p));
        }
        if (!u.nch) continue;
        const char* ce = std::getenv("QSIM_NOISE_CHECK");
        if (ce && std::atoi(ce) != 0) {  // range-checked launch (tests): violations -> error
            unsigned int* d_bad = nullptr;
            QSIM_HIPCHK(hipMalloc((void**)&d_bad, 2 * sizeof(unsigned int)));
            QSIM_HIPCHK(hipMemsetAsync(d_bad, 0, 2 * sizeof(unsigned int), s));
            hipLaunchKernelGGL(k_noise_units<true>, dim3((unsigned)units), dim3(256), 0, s, u, d_bad);
            QSIM_HIPCHK(hipGetLastError());
            unsigned int h_bad[2] = {0, 0};
            QSIM_HIPCHK(hipMemcpyAsync(h_bad, d_bad, sizeof h_bad, hipMemcpyDeviceToHost, s));
            QSIM_HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(d_bad);
            noise_check_flips += h_bad[1];
            if (h_bad[0])
                fail(QSIM_ERR_RUNTIME, "noise unit kernel touched " + std::to_string(h_bad[0]) +
                                           " amplitudes outside its pairs");
            continue;
        }
        TimedLaunch tl(tm, "noise", bytes, s);
        // one work-group per unit (fewer work-groups looping over units measured slower: the
        // walk is latency-bound)
        hipLaunchKernelGGL(k_noise_units<false>, dim3((unsigned)units), dim3(256), 0, s, u, nullptr);
        QSIM_HIPCHK(hipGetLastError());
    }
}

void launch_noise(double2* st, int n, int type, int qubit, double p, uint64_t seed,
                  uint64_t counter, hipStream_t s, Timer* tm, uint64_t batch, uint64_t traj0) {
    check_channel(n, type, qubit, p);
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
    if (type == 0 || type >= 3) {  // flips: geometric walk per block of pairs
        FArgsN f{};
        f.st = st;
        f.pairs = a.pairs;
        f.idx0 = a.idx0;
        f.log_ppt = a.log_ppt;
        if (!flip_channel(type, qubit, p, a.key, f.c)) return;
        const uint64_t nb = ((a.idx0 + a.pairs - 1) >> kFlipBlockLog) - (a.idx0 >> kFlipBlockLog) + 1;
        const uint64_t fb = std::min<uint64_t>((nb + 255) / 256, 256ull * 32);
        hipLaunchKernelGGL(k_noise_flips, dim3((unsigned)fb), dim3(256), 0, s, f);
    } else if (type == 1) {
        hipLaunchKernelGGL(k_noise<1>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_noise<2>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    }
    QSIM_HIPCHK(hipGetLastError());
}


// ---------------------------------------------------------------------------------------
// Gate + in-tile noise (BatchedSimulator's reference process: the default from 12 qubits).
//
// One gate step = the gate, then every channel entry in order.  A work-group owns a TILE of
// 4096 amplitudes of one trajectory — qubits 0..10 plus one more, u (the gate's target when it is
// >= 11, else 11) — and applies the gate and then the longest PREFIX of the channel list whose
// qubits lie in the tile (every such channel's flips are pairs inside the tile).  The suffix (the
// remaining channels) runs as the one-launch push kernel afterwards.
//
// The prefix's flips form a signed permutation P of the tile (X swaps a pair, Y swaps it with
// phases -i / +i, Z negates its |1> member), so P is never applied channel by channel (round 4's
// form: one LDS phase and barrier per channel, ~24 us per channel per launch).  Instead:
//   1. the tile's 16 loads per thread are issued into registers;
//   2. meanwhile the blocks of every prefix channel are walked (the push kernels' draws: blocks of
//      256 global pairs, geometric gaps from the same counter hash), one walk per thread, and each
//      flip's 2-bit code (1 X, 2 Y, 3 Z) is ORed into field c of the CODE WORD of both members of
//      its pair (LDS, 24 bits per amplitude, 12 KiB);
//   3. the registers go to LDS and the gate runs there;
//   4. each output amplitude k is PULLED through P: walking its word's non-zero fields from the
//      last channel down (X / Y move k to the pair partner and re-read the word there, keeping the
//      fields below; Y and Z add a phase i^e), out[k] = i^e v[k'] — a zero word (~89 % of them at
//      p = 0.01 on 12 channels) is a plain copy — and stored straight to HBM.
// Exact: out[k] equals applying the channels in order (every step is a swap / sign change of
// doubles), so the same states bit for bit as the gate kernel + push kernel.  Three barriers per
// tile whatever the channel count; LDS 76 KiB (two work-groups per CU).
// ---------------------------------------------------------------------------------------
constexpr int kGnTile = 12;
constexpr int kGnMaxPrefix = 12;  // 2-bit fields of a 24-bit packed word
struct GnArgs {
    double2* st;
    int n;
    int u;                 // the tile's 12th qubit (>= 11)
    uint64_t idx0;         // global pair index of this object's pair 0
    int kind;              // K_M1, K_DIAG, K_SWAP, or -1: no gate
    int sub, t0, t1, d0_one;
    uint32_t cm_in;        // controls inside the tile, as tile-local bits
    uint64_t cm_out;       // controls outside the tile (trajectory-local index bits)
    double2 m[4];
    int np;                // prefix channels
    int pq[kGnMaxPrefix];  // tile-local position of each prefix channel's qubit
    uint64_t pqpack;       // the same, 4 bits per channel (a per-lane channel index then costs no load)
    FlipChan ch[kGnMaxPrefix];
    // precomputed flip lists of this step (k_gn_lists, built on a second stream during the step
    // before), or null: the work-group walks the blocks itself.  Per tile and prefix channel, cap
    // entries (tile pair-local index << 2 | code) and the flip count (> cap: overflow, walked here)
    const uint16_t* list;
    const uint32_t* cnt;
    int cap, lcap;         // cap = 2^lcap
    int skip;              // QSIM_NOISE_TILE_SKIP (measurement only, wrong states): 1 no flip
                           // codes written, 2 no pulled walks (outputs read in place), 3 both
    int bmap;              // work-group order (QSIM_NOISE_BMAP)
};
__device__ __forceinline__ int gn_local_pos(int q, int u) { return q <= 10 ? q : (q == u ? 11 : -1); }

// Tile b of a step: its trajectory and its non-tile index bits (11 .. n-1 except u, ascending,
// from the low bits of b); tile-local j -> gbase | (j & 2047) | (j >> 11) << u.
__device__ __forceinline__ uint64_t gn_tile_base(uint64_t b, int n, int u, uint64_t* traj_out, uint64_t* loc_out) {
    const int nfree = n - kGnTile;
    const uint64_t traj = b >> nfree;
    const uint64_t m = b & ((1ull << nfree) - 1ull);
    uint64_t loc = 0;
    int j = 0;
    for (int q = 11; q < n; ++q) {
        if (q == u) continue;
        loc |= ((m >> j) & 1ull) << q;
        ++j;
    }
    *traj_out = traj;
    *loc_out = loc;
    return (traj << n) | loc;
}
// Walk block jb (of 8) of prefix channel c over the tile at gbase: f(x, code) for every flip, x
// the tile pair-local index.  The push kernels' draws exactly (flip_block: blocks of 256 global
// pairs, geometric gaps from the same counter hash).
template <class F>
__device__ __forceinline__ void gn_walk(const GnArgs& a, int c, int jb, uint64_t traj, uint64_t gbase, F&& f) {
    const FlipChan& ch = a.ch[c];
    const int q = ch.target;
    const uint64_t tl = gbase & ((1ull << a.n) - 1ull);  // trajectory-local base
    // pair index (within the trajectory) of the tile's first pair of this channel
    const uint64_t prb = ((tl >> (q + 1)) << q) | (tl & ((1ull << q) - 1ull));
    uint64_t pr0;  // first pair of this walk's run
    int run_base;  // tile pair-local index of that pair
    if (q == a.u) {
        pr0 = prb + (uint64_t)jb * 256;
        run_base = jb * 256;
    } else {  // two runs of 1024 pairs, bit u of the index -> pair bit u - 1
        const int y = jb >> 2;
        pr0 = prb + ((uint64_t)y << (a.u - 1)) + (uint64_t)(jb & 3) * 256;
        run_base = (y << 10) + (jb & 3) * 256;
    }
    const uint64_t gb = (a.idx0 + (traj << (a.n - 1)) + pr0) >> kFlipBlockLog;
    FlipCursor cur{nz_mix(ch.key ^ nz_mix(gb ^ kBlockSalt)), 0, -1, false};
    uint64_t g = 0, h = 0;
    const uint64_t lo = gb << kFlipBlockLog, hi = lo + kFlipBlock;
    while (next_flip(cur, gb, lo, hi, ch, g, h)) {
        uint32_t code = ch.type == 3 ? 1u : (ch.type == 4 ? 3u : 2u);
        if (ch.type == 0) {
            const float r2 = nz_uniform(nz_mix(h ^ 0x5bd1e9955bd1e995ull));
            code = r2 < 1.0f / 3.0f ? 1u : (r2 < 2.0f / 3.0f ? 2u : 3u);
        }
        f(run_base + (int)(g - lo), code);
    }
}

// The flip lists of one step: one thread per (tile, prefix channel) walks that channel's 8 blocks
// over the tile (DP log per draw; run on a second stream beside the previous step's suffix push)
// and writes the first cap flips in walk order, then the count (> cap: the tile kernel ignores the
// list and walks the channel itself).  (One thread per block with atomic slot reservation measured
// slower: 67.3 vs 58.2 ms per W-BATCH step.)
// The same lists with one lane per (tile, channel, block): the 8 lanes of a (tile, channel) count
// their blocks' flips, place them by a prefix sum over those lanes, and walk again to write —
// twice the draws, but chains of one block instead of eight (the walks are latency-bound), and
// the entries land in the same order as the one-lane form's, so the lists are identical.
__global__ __launch_bounds__(256) void k_gn_lists8(GnArgs a, uint16_t* list, uint32_t* cnt, uint64_t tiles) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t grp = tid >> 3;  // (tile, channel); 8 lanes each, aligned within a wave
    const int jb = (int)(tid & 7);
    const bool live = grp < tiles * (uint64_t)a.np;
    const uint64_t b = live ? grp / (uint64_t)a.np : 0;
    const int c = live ? (int)(grp - b * (uint64_t)a.np) : 0;
    uint64_t traj = 0, loc = 0;
    const uint64_t gbase = gn_tile_base(b, a.n, a.u, &traj, &loc);
    uint32_t k = 0;
    if (live) gn_walk(a, c, jb, traj, gbase, [&](int, uint32_t) { ++k; });
    // exclusive prefix of k over the 8 lanes of the group (every lane takes part: shuffles)
    uint32_t incl = k;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 8);
        if (jb >= d) incl += o;
    }
    const uint32_t total = __shfl(incl, 7, 8);
    if (!live) return;
    uint32_t pos = incl - k;
    uint16_t* out = list + (b * kGnMaxPrefix + (uint64_t)c) * (uint64_t)a.cap;
    if (pos < (uint32_t)a.cap)
        gn_walk(a, c, jb, traj, gbase, [&](int x, uint32_t code) {
            if (pos < (uint32_t)a.cap) out[pos] = (uint16_t)((x << 2) | (int)code);
            ++pos;
        });
    if (jb == 0) cnt[b * kGnMaxPrefix + (uint64_t)c] = total;
}

__global__ __launch_bounds__(256) void k_gn_lists(GnArgs a, uint16_t* list, uint32_t* cnt, uint64_t tiles) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= tiles * (uint64_t)a.np) return;
    const uint64_t b = tid / (uint64_t)a.np;
    const int c = (int)(tid - b * (uint64_t)a.np);
    uint64_t traj = 0, loc = 0;
    const uint64_t gbase = gn_tile_base(b, a.n, a.u, &traj, &loc);
    uint16_t* out = list + (b * kGnMaxPrefix + (uint64_t)c) * (uint64_t)a.cap;
    uint32_t k = 0;
    for (int jb = 0; jb < 8; ++jb)
        gn_walk(a, c, jb, traj, gbase, [&](int x, uint32_t code) {
            if (k < (uint32_t)a.cap) out[k] = (uint16_t)((x << 2) | (int)code);
            ++k;
        });
    cnt[b * kGnMaxPrefix + (uint64_t)c] = k;
}

__global__ __launch_bounds__(256) void k_gate_noise_tile(GnArgs a) {
    __shared__ double2 v[1 << kGnTile];
    // code words packed to 24 bits per amplitude (12 KiB, so two work-groups fit a CU's 160 KiB
    // LDS with room to spare): fields of channels 0-7 in 16-bit halves of wlo, 8-11 in bytes of whi
    __shared__ uint32_t wlo[1 << (kGnTile - 1)], whi[1 << (kGnTile - 2)];
    auto word_or = [&](int j, int c, uint32_t code) {
        if (c < 8) atomicOr(&wlo[j >> 1], code << (2 * c + 16 * (j & 1)));
        else atomicOr(&whi[j >> 2], code << (2 * (c - 8) + 8 * (j & 3)));
    };
    auto word_at = [&](int j) {
        return ((wlo[j >> 1] >> (16 * (j & 1))) & 0xffffu) | (((whi[j >> 2] >> (8 * (j & 3))) & 0xffu) << 16);
    };
    // tile-local position of prefix channel c's qubit (c may differ between lanes: unpacked from
    // a kernel argument, not indexed out of the argument block)
    auto pq_of = [&](int c) { return (int)((a.pqpack >> (4 * c)) & 15ull); };
    // a flip of prefix channel c on tile pair-local pair x: its code into both members' words
    auto flip_or = [&](int c, int x, uint32_t code) {
        const int pq = pq_of(c);
        int j0;
        if (pq == 11) {
            j0 = x;
        } else {
            const int xl = x & 1023, y = x >> 10;
            const int lo2 = xl & ((1 << pq) - 1);
            j0 = (((xl ^ lo2) << 1) | lo2) | (y << 11);
        }
        word_or(j0, c, code);
        word_or(j0 | (1 << pq), c, code);
    };
    __shared__ uint32_t cnt_s[kGnMaxPrefix];
    const int t = threadIdx.x;
    uint64_t traj = 0, loc = 0;
    const uint64_t tb = xcd_block(a.bmap);
    const uint64_t gbase = gn_tile_base(tb, a.n, a.u, &traj, &loc);
    auto gidx = [&](int j) { return gbase | (uint64_t)(j & 2047) | ((uint64_t)(j >> 11) << a.u); };
    // 1. this tile's flip lists, then the tile's loads, all in flight during the flip phase (the
    // lists first: the flip phase then waits only for them — loads retire in order)
    constexpr int kSlots = kGnMaxPrefix;  // list slots per thread: np * cap <= 12 * 256
    uint16_t le[kSlots];
    const int nsl = a.list ? a.np << a.lcap : 0;  // slots of this tile (cap = 2^lcap per channel)
    const uint16_t* L = a.list + tb * kGnMaxPrefix * (uint64_t)(1u << a.lcap);
    const uint32_t* C = a.cnt + tb * kGnMaxPrefix;
    uint32_t cl = 0;
    if (a.list && t < a.np) cl = C[t];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) le[k] = k * 256 + t < nsl ? L[k * 256 + t] : (uint16_t)0;
    double2 r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = ld<true>(a.st + gidx(k * 256 + t));
    if (a.list && t < a.np) cnt_s[t] = cl;
#pragma unroll
    for (int k = 0; k < 8; ++k) wlo[k * 256 + t] = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) whi[k * 256 + t] = 0u;
    __syncthreads();
    // 2. the prefix channels' flips into the code words
    if (a.skip & 1) {
    } else if (a.list) {
#pragma unroll
        for (int k = 0; k < kSlots; ++k) {
            const int sl = k * 256 + t;
            if (sl >= nsl) break;
            const int c = sl >> a.lcap, e = sl & ((1 << a.lcap) - 1);
            if ((uint32_t)e < cnt_s[c] && cnt_s[c] <= (uint32_t)a.cap) flip_or(c, (int)(le[k] >> 2), le[k] & 3u);
        }
        // (an overflowing list, > cap flips, holds an arbitrary part of them: that channel is
        // walked here instead, one block per thread)
        if (t < a.np * 8 && cnt_s[t >> 3] > (uint32_t)a.cap) {
            const int c = t >> 3;
            gn_walk(a, c, t & 7, traj, gbase, [&](int x, uint32_t code) { flip_or(c, x, code); });
        }
    } else if (t < a.np * 8) {  // one walk per thread
        const int c = t >> 3;
        gn_walk(a, c, t & 7, traj, gbase, [&](int x, uint32_t code) { flip_or(c, x, code); });
    }
    // 3. registers -> LDS, the gate
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k * 256 + t] = r[k];
    __syncthreads();
    const bool on_out = (loc & a.cm_out) == a.cm_out;
    if (a.kind >= 0 && on_out) {  // (uniform per work-group)
        const int p0 = gn_local_pos(a.t0, a.u);
        if (a.kind == K_M1) {
            for (int i = t; i < 2048; i += 256) {
                const int lo = i & ((1 << p0) - 1);
                const int j0 = ((i ^ lo) << 1) | lo, j1 = j0 | (1 << p0);
                if (((uint32_t)j0 & a.cm_in) != a.cm_in) continue;
                double2 x0 = v[j0], x1 = v[j1];
                m1_pair(a.sub, a.m[0], a.m[1], a.m[2], a.m[3], x0, x1);
                v[j0] = x0;
                v[j1] = x1;
            }
        } else if (a.kind == K_DIAG) {
            for (int j = t; j < 4096; j += 256) {
                if (((uint32_t)j & a.cm_in) != a.cm_in) continue;
                v[j] = diag_apply(a.sub, a.d0_one, a.m[0], a.m[1], (j >> p0) & 1, v[j]);
            }
        } else {  // SWAP (both qubits in the tile)
            const int p1 = gn_local_pos(a.t1, a.u);
            for (int j = t; j < 4096; j += 256) {
                if (((j >> p0) & 1) == 0 && ((j >> p1) & 1) == 1 && ((uint32_t)j & a.cm_in) == a.cm_in) {
                    const int k = j ^ ((1 << p0) | (1 << p1));
                    const double2 x = v[j];
                    v[j] = v[k];
                    v[k] = x;
                }
            }
        }
        __syncthreads();
    }
    // 4. out[k] = (P v)[k], pulled through the code words, stored in place.  The walks of a
    // thread's 16 amplitudes advance in lockstep (one step of every unfinished walk per round, the
    // word loads of a round independent), so LDS latency is paid once per round, not per step of
    // every amplitude (in a wave some lane almost always has a non-zero word).
    int jj[16], ee[16];
    uint32_t ww[16];
#pragma unroll
    for (int k0 = 0; k0 < 16; ++k0) {
        jj[k0] = k0 * 256 + t;
        ee[k0] = 0;
        ww[k0] = word_at(jj[k0]);
    }
    for (;;) {
        if (a.skip & 2) break;
        uint32_t any = 0;
#pragma unroll
        for (int k0 = 0; k0 < 16; ++k0) any |= ww[k0];
        if (!any) break;
        bool mv[16];
        uint32_t keep[16];
#pragma unroll
        for (int k0 = 0; k0 < 16; ++k0) {
            mv[k0] = false;
            keep[k0] = 0u;
            const uint32_t w = ww[k0];
            if (!w) continue;
            const int c = (31 - __builtin_clz(w)) >> 1;  // the last channel that flips jj's pair
            const uint32_t code = (w >> (2 * c)) & 3u;
            const int pqc = pq_of(c);
            const int bit = (jj[k0] >> pqc) & 1;
            keep[k0] = (1u << (2 * c)) - 1u;  // the channels before it
            ww[k0] = w & keep[k0];
            if (code == 3u) {  // Z: -1 on the |1> member
                ee[k0] += 2 * bit;
            } else {           // X: partner; Y: partner with -i (|0> member) / +i (|1>)
                if (code == 2u) ee[k0] += bit ? 1 : 3;
                jj[k0] ^= 1 << pqc;
                mv[k0] = true;
            }
        }
#pragma unroll
        for (int k0 = 0; k0 < 16; ++k0)
            if (mv[k0]) ww[k0] = word_at(jj[k0]) & keep[k0];
    }
#pragma unroll
    for (int k0 = 0; k0 < 16; ++k0) {
        const double2 x = v[jj[k0]];
        double2 y;
        switch (ee[k0] & 3) {
            case 0: y = x; break;
            case 1: y = make_double2(-x.y, x.x); break;   // i
            case 2: y = make_double2(-x.x, -x.y); break;  // -1
            default: y = make_double2(x.y, -x.x); break;  // -i
        }
        st<true>(a.st + gidx(k0 * 256 + t), y);
    }
}

bool gate_noise_tile_supported(int n, const Op* op) {
    const char* e = std::getenv("QSIM_NOISE_TILE");  // (read per run: tests switch it; 0 = push)
    if (e && std::atoi(e) == 0) return false;
    if (n < kGnTile) return false;
    if (!op) return true;
    if (op->kind == K_SWAP) {
        const int hi0 = op->t0 >= 11, hi1 = op->t1 >= 11;
        if (hi0 && hi1) return false;  // (two qubits above 10: not one tile)
    }
    return true;
}

// One step's kernel arguments: the gate and the prefix channels (keys from counter0, one counter
// per channel entry whether it can fire or not, as the push kernels); *used: entries in the prefix
// (the rest is the suffix).
static GnArgs gn_args(double2* st, int n, uint64_t traj0, const Op* op, const std::vector<NoiseChan>& chans,
                      uint64_t seed, uint64_t counter0, size_t* used_out) {
    GnArgs a{};
    a.st = st;
    a.n = n;
    a.idx0 = traj0 << (n - 1);
    int u = 11;
    if (op) {
        if (op->t0 >= 11) u = op->t0;
        if (op->kind == K_SWAP && op->t1 >= 11) u = op->t1;
    }
    a.u = u;
    a.kind = op ? op->kind : -1;
    if (op) {
        a.sub = op->sub;
        a.t0 = op->t0;
        a.t1 = op->t1;
        a.d0_one = op->d0_one ? 1 : 0;
        for (int q = 0; q < n; ++q) {
            if (!((op->cmask >> q) & 1ull)) continue;
            const int p = q <= 10 ? q : (q == u ? 11 : -1);
            if (p >= 0) a.cm_in |= 1u << p;
            else a.cm_out |= 1ull << q;
        }
        for (int i = 0; i < 4; ++i) a.m[i] = make_double2(op->m[2 * i], op->m[2 * i + 1]);
    }
    // the prefix: channel entries in order whose qubit is in the tile (a channel that cannot fire
    // is skipped but still uses its counter, as the push kernels do)
    uint64_t c = counter0;
    size_t used = 0;
    const char* pe = std::getenv("QSIM_NOISE_TILE_PREFIX");  // (measurement: cap on the prefix)
    const size_t cap = pe ? (size_t)std::max(0, std::atoi(pe)) : chans.size();
    for (; used < chans.size() && used < cap; ++used) {
        const NoiseChan& ch = chans[used];
        check_channel(n, ch.type, ch.qubit, ch.p);
        const bool in = ch.qubit <= 10 || ch.qubit == u;
        if (!in || !(ch.type == 0 || ch.type >= 3)) break;
        if (flip_probability(ch.p) > 0.0) {
            if (a.np == kGnMaxPrefix) break;  // (the rest goes to the push kernel)
            flip_channel(ch.type, ch.qubit, ch.p, noise_key(seed, c), a.ch[a.np]);
            a.pq[a.np] = ch.qubit <= 10 ? ch.qubit : 11;
            a.pqpack |= (uint64_t)a.pq[a.np] << (4 * a.np);
            ++a.np;
        }
        ++c;
    }
    *used_out = used;
    const char* sk = std::getenv("QSIM_NOISE_TILE_SKIP");  // (measurement only)
    a.skip = sk ? std::atoi(sk) : 0;
    a.bmap = env_bmap("QSIM_NOISE_BMAP", 1);
    return a;
}

static void launch_gn_tile(const GnArgs& a, uint64_t batch, hipStream_t s, Timer* tm) {
    TimedLaunch tl(tm, "gate_noise", 32.0 * (double)(batch << a.n), s);
    const uint64_t blocks = (batch << a.n) >> kGnTile;
    hipLaunchKernelGGL(k_gate_noise_tile, dim3((unsigned)blocks), dim3(256), 0, s, a);
    QSIM_HIPCHK(hipGetLastError());
}

void launch_gate_noise_step(double2* st, int n, uint64_t batch, uint64_t traj0, const Op* op,
                            const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t& counter, hipStream_t s,
                            Timer* tm) {
    size_t used = 0;
    const GnArgs a = gn_args(st, n, traj0, op, chans, seed, counter, &used);
    launch_gn_tile(a, batch, s, tm);
    counter += used;
    if (used < chans.size()) {
        const std::vector<NoiseChan> rest(chans.begin() + (long)used, chans.end());
        launch_noise_after_gate(st, n, rest, seed, counter, s, tm, batch, traj0);
    }
}

// List capacity per (tile, channel) for the largest flip probability of `chans` (0: no lists —
// above p ~ 0.1 the lists would outweigh the walks): mean 2048 P flips, cap = the power of two
// >= mean + 6 sigma + 8 (p = 0.01: 64; P(overflow) ~ 1e-12 per list); a list that overflows is
// walked by its tile kernel (exact either way).
static int gn_list_cap(const std::vector<NoiseChan>& chans) {
    double P = 0.0;
    for (const NoiseChan& c : chans)
        if (c.type == 0 || c.type >= 3) P = std::max(P, flip_probability(c.p));
    if (!(P > 0.0)) return 0;
    auto pow2 = [](int x) {
        int c = 8;
        while (c < x) c <<= 1;
        return c;
    };
    const char* e = std::getenv("QSIM_NOISE_LIST_CAP");  // (tests: a small cap forces overflows)
    if (e && std::atoi(e) > 0) return pow2(std::atoi(e));
    const double lam = 2048.0 * P;
    const int cap = pow2((int)std::ceil(lam + 6.0 * std::sqrt(lam) + 8.0));
    return cap <= 256 ? cap : 0;
}
size_t gate_noise_lists_bytes(int n, uint64_t batch, const std::vector<NoiseChan>& chans) {
    const char* e = std::getenv("QSIM_NOISE_TILE_LISTS");  // (read per run: 0 = walks in the tile kernel)
    if (e && std::atoi(e) == 0) return 0;
    const int cap = gn_list_cap(chans);
    if (!cap || n < kGnTile) return 0;
    const uint64_t tiles = (batch << n) >> kGnTile;
    return (size_t)(tiles * kGnMaxPrefix * ((uint64_t)cap * sizeof(uint16_t) + sizeof(uint32_t)));
}

void launch_gate_noise_run(double2* st, int n, uint64_t batch, uint64_t traj0, const std::vector<Op>& ops,
                           const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t& counter, hipStream_t s,
                           Timer* tm, const GnLists* L) {
    const size_t G = ops.size(), nch = chans.size();
    const uint64_t c0 = counter;
    std::vector<GnArgs> args(G);
    std::vector<size_t> used(G, 0);
    for (size_t i = 0; i < G; ++i)
        args[i] = gn_args(st, n, traj0, ops[i].kind >= 0 ? &ops[i] : nullptr, chans, seed, c0 + i * nch, &used[i]);
    const int cap = L ? gn_list_cap(chans) : 0;
    const uint64_t tiles = (batch << n) >> kGnTile;
    const bool lists = L && cap && L->set_bytes >= (size_t)(tiles * kGnMaxPrefix *
                                                            ((uint64_t)cap * sizeof(uint16_t) + sizeof(uint32_t)));
    auto set_of = [&](size_t i, uint16_t** list, uint32_t** cnt) {
        char* base = (char*)L->buf[i & 1];
        *list = (uint16_t*)base;
        *cnt = (uint32_t*)(base + tiles * kGnMaxPrefix * (uint64_t)cap * sizeof(uint16_t));
    };
    auto build = [&](size_t i) {
        if (i >= 2) QSIM_HIPCHK(hipStreamWaitEvent(L->ms, L->used[i & 1], 0));  // tile kernel i - 2 done
        GnArgs b = args[i];
        b.cap = cap;
        b.lcap = __builtin_ctz((unsigned)cap);
        uint16_t* list = nullptr;
        uint32_t* cnt = nullptr;
        set_of(i, &list, &cnt);
        if (b.np) {
            // QSIM_NOISE_LISTS8 (default 1): one lane per (tile, channel, block), k_gn_lists8;
            // 0: one lane per (tile, channel)
            const char* l8e = std::getenv("QSIM_NOISE_LISTS8");
            const bool l8 = l8e == nullptr || std::atoi(l8e) != 0;
            const uint64_t threads = tiles * (uint64_t)b.np * (l8 ? 8u : 1u);
            TimedLaunch tl(tm, "noise_lists", 0.0, L->ms);
            if (l8)
                hipLaunchKernelGGL(k_gn_lists8, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, L->ms, b, list,
                                   cnt, tiles);
            else
                hipLaunchKernelGGL(k_gn_lists, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, L->ms, b, list,
                                   cnt, tiles);
            QSIM_HIPCHK(hipGetLastError());
        }
        QSIM_HIPCHK(hipEventRecord(L->built[i & 1], L->ms));
    };
    if (lists) {  // (the previous run's tile kernels may still read both sets)
        QSIM_HIPCHK(hipEventRecord(L->start, s));
        QSIM_HIPCHK(hipStreamWaitEvent(L->ms, L->start, 0));
        for (size_t i = 0; i < std::min<size_t>(G, 2); ++i) build(i);
    }
    for (size_t i = 0; i < G; ++i) {
        GnArgs a = args[i];
        if (lists) {
            QSIM_HIPCHK(hipStreamWaitEvent(s, L->built[i & 1], 0));
            uint16_t* list = nullptr;
            uint32_t* cnt = nullptr;
            set_of(i, &list, &cnt);
            a.list = list;
            a.cnt = cnt;
            a.cap = cap;
            a.lcap = __builtin_ctz((unsigned)cap);
        }
        launch_gn_tile(a, batch, s, tm);
        // the lists of step i + 2 reuse this step's set: built once this step's tile kernel is
        // done, beside the suffix push (measured: beside the next tile pass instead, the build
        // slowed that pass by more than it slowed the push)
        if (lists && i + 2 < G) {
            QSIM_HIPCHK(hipEventRecord(L->used[i & 1], s));
            build(i + 2);
        }
        uint64_t c = c0 + i * nch + used[i];
        if (used[i] < nch) {
            const std::vector<NoiseChan> rest(chans.begin() + (long)used[i], chans.end());
            launch_noise_after_gate(st, n, rest, seed, c, s, tm, batch, traj0);
        }
    }
    counter = c0 + G * nch;
}

// ---------------------------------------------------------------------------------------
// Pulled noise: the flips after gate g applied by the NEXT gate's pass (BatchedSimulator's
// reference process, NoisySimulator's flip channels).
//
// The flips of one noise step (every channel entry after one gate, applied in channel order) form
// a signed permutation P of the amplitudes (X swaps a pair, Y swaps it with phases -i / +i, Z
// negates its |1> member).  Pushing P into the state costs random 16-B reads and writes over most
// of the lines (one noise step ~ one streaming pass of line traffic).  Instead the next
// gate's kernel reads its inputs through P: (P psi)[k] = i^e psi[s(k)], found by walking the
// channels from the last to the first (a flip of the pair holding the current index moves it
// along the channel's qubit, or only adds a phase), and writes U (P psi) out of place — one
// streaming pass per gate step instead of two.
//
// The draws are exactly the push kernels' (flip_block: blocks of 256 global pairs, geometric
// walks from the same counter hash), so both paths produce the same states:
//   k_noise_words  per step, one work-group per region of 2^12 amplitudes (the whole trajectory
//                  below 12 qubits): walks every block of pairs with a member in the region, for
//                  every channel at once (one walk per thread), and ORs each flip's 2-bit code
//                  (1 X, 2 Y, 3 Z) into the CODE WORD of both members in LDS (field c: bits
//                  2c, 2c + 1), then stores the region's words (4 B per amplitude up to 16
//                  channels, 8 B up to 32), coalesced.  A zero word: no channel flips a pair
//                  holding that amplitude.
//   k_pull_gate    the gate (2x2 / diagonal / SWAP with controls, or the identity after the last
//                  gate) over the pulled inputs, src -> dst.  Amplitude, word and partner loads are
//                  issued together (the common case, a zero word, is a plain streaming pass); a
//                  non-zero word is walked from its highest field down, one dependent word load
//                  per move (X / Y), none for Z.
// Needs n >= 9, every channel a flip channel, <= 32 that can fire.
// ---------------------------------------------------------------------------------------
constexpr int kRegionLogMax = 12;
constexpr int kMinPullQubits = 9;
constexpr int kMaxPullChannels = 32;
constexpr int kWordThreads = 256;
struct MapArgs {
    void* words;
    int skip;            // QSIM_MAP_SKIP (measurement only, wrong states): 1 no walks, 2 no stores
    int rpw;             // (fused into the pull pass) regions per work-group
    uint64_t amps;       // batch << n (this object's)
    uint64_t idx0;       // global pair index of local pair 0
    int n, rl;           // qubits per trajectory, region log (min(12, n))
    int nch;
    int task_off[kMaxPullChannels + 1];  // walks per region before channel c (prefix sums)
    FlipChan ch[kMaxPullChannels];
};

// Sparse code words (QSIM_NOISE_SPARSE, default on): 16 bits per amplitude instead of 32 / 64.  At
// p = 0.01 a code word holds at most two non-zero fields for all but ~0.2 % of the amplitudes
// (26 channels), so the word of amplitude k is stored as up to two (channel, code) entries —
// bits 0-4 channel and 5-6 code of the highest flipping channel, 7-11 / 12-13 of the next, 14-15
// the entry count — and a word with three or more non-zero fields as count 3, its full 64-bit
// word at ovf[k] (a second array of the same index space, touched only at those amplitudes).  The
// pull pass then streams 2 B of words per amplitude instead of 8 (26 channels) or 4 (<= 16).
__device__ __forceinline__ uint16_t sparse_encode(unsigned long long w, bool* over) {
    const unsigned long long nz = (w | (w >> 1)) & 0x5555555555555555ull;  // bit 2c: field c != 0
    const int cnt = __popcll(nz);
    *over = cnt > 2;
    if (cnt == 0) return 0;
    if (cnt > 2) return (uint16_t)0xC000u;
    const int c1 = (63 - __clzll((long long)nz)) >> 1;
    uint32_t r = (uint32_t)c1 | ((uint32_t)((w >> (2 * c1)) & 3ull) << 5) | ((uint32_t)cnt << 14);
    if (cnt == 2) {
        const unsigned long long rest = nz & ~(1ull << (2 * c1));
        const int c2 = (63 - __clzll((long long)rest)) >> 1;
        r |= ((uint32_t)c2 << 7) | ((uint32_t)((w >> (2 * c2)) & 3ull) << 12);
    }
    return (uint16_t)r;
}
// The full word of amplitude k from its sparse entry r (ovf: the overflow words).
template <class W>
__device__ __forceinline__ W sparse_decode(uint16_t r, const unsigned long long* ovf, uint64_t k) {
    const uint32_t cnt = (uint32_t)r >> 14;
    if (cnt == 3) return (W)ovf[k];
    W f = 0;
    if (cnt >= 1) f |= (W)((r >> 5) & 3u) << (2 * (r & 31u));
    if (cnt == 2) f |= (W)((r >> 12) & 3u) << (2 * ((r >> 7) & 31u));
    return f;
}
bool noise_sparse_words() {
    const char* e = std::getenv("QSIM_NOISE_SPARSE");  // (read per launch: tests switch it)
    return e == nullptr || std::atoi(e) != 0;
}
// Byte offset of the overflow words behind the 16-bit entries of `amps` amplitudes.
__host__ __device__ inline uint64_t sparse_ovf_offset(uint64_t amps) { return (amps * sizeof(uint16_t) + 255) & ~255ull; }

// One block's walk: flips (local pair l in [0, 256) of block gb) handed to `f(l, code)`.
template <class F>
__device__ __forceinline__ void walk_block(uint64_t gb, const FlipChan& c, F&& f) {
    FlipCursor cur{nz_mix(c.key ^ nz_mix(gb ^ kBlockSalt)), 0, -1, false};
    uint64_t g = 0, h = 0;
    const uint64_t lo = gb << kFlipBlockLog, hi = lo + kFlipBlock;
    while (next_flip(cur, gb, lo, hi, c, g, h)) {
        int code = c.type == 3 ? 1 : (c.type == 4 ? 3 : 2);  // X / Z / Y (flip_block's picks)
        if (c.type == 0) {
            const float r2 = nz_uniform(nz_mix(h ^ 0x5bd1e9955bd1e995ull));
            code = r2 < 1.0f / 3.0f ? 1 : (r2 < 2.0f / 3.0f ? 2 : 3);
        }
        f((uint32_t)(g - lo), (uint32_t)code);
    }
}

// Walk task `task` (channel c, j-th block of pairs with a member in the region starting at
// amplitude K0 of 2^a.rl) and OR its flips' codes into the region's LDS words w.
// (chs / toff: the channel table and the task offsets, staged in LDS by the caller — indexed per
// lane, they would otherwise be vector loads from the kernel-argument segment in every task)
template <class W>
__device__ __forceinline__ void map_task(const MapArgs& a, const FlipChan* chs, const int* toff, W* w, uint64_t K0,
                                         int task) {
    const uint64_t traj = K0 >> a.n, r0 = K0 & ((1ull << a.n) - 1ull);
    int c = 0;
    while (task >= toff[c + 1]) ++c;
    const int j = task - toff[c];
    const FlipChan ch = chs[c];
    const int q = ch.target;
    const W sh = (W)(2 * c);
    uint64_t lbase;  // the first pair (this object's pair index) with a member in the region
    if (q < a.rl) {  // both members in the region: 2^(rl-1) pairs
        lbase = (traj << (a.n - 1)) + (r0 >> 1);
    } else {         // one member in the region (bit q fixed): 2^rl consecutive pairs
        lbase = (traj << (a.n - 1)) + (((r0 >> (q + 1)) << q) | (r0 & ((1ull << q) - 1ull)));
    }
    const uint64_t gb = ((a.idx0 + lbase) >> kFlipBlockLog) + (uint64_t)j;
    walk_block(gb, ch, [&](uint32_t l, uint32_t code) {
        const uint32_t lp = (uint32_t)j * (uint32_t)kFlipBlock + l;  // region-local pair
        if (q < a.rl) {
            const uint32_t lo = lp & ((1u << q) - 1u);
            const uint32_t a0 = ((lp ^ lo) << 1) | lo;
            atomicOr(&w[a0], (W)code << sh);
            atomicOr(&w[a0 | (1u << q)], (W)code << sh);
        } else {
            atomicOr(&w[lp], (W)code << sh);
        }
    });
}

template <class W, bool SPARSE = false>
__global__ __launch_bounds__(kWordThreads) void k_noise_words(MapArgs a) {
    __shared__ W w[1 << kRegionLogMax];
    __shared__ FlipChan chs[kMaxPullChannels];
    __shared__ int toff[kMaxPullChannels + 1];
    const int t = threadIdx.x;
    const int R = 1 << a.rl;
    for (int i = t; i < R; i += kWordThreads) w[i] = 0;
    if (t < a.nch) chs[t] = a.ch[t];
    if (t <= a.nch) toff[t] = a.task_off[t];
    __syncthreads();
    const uint64_t K0 = (uint64_t)blockIdx.x << a.rl;  // the region's first amplitude (this object)
    if (!(a.skip & 1))
        for (int task = t; task < toff[a.nch]; task += kWordThreads) map_task(a, chs, toff, w, K0, task);
    __syncthreads();
    if constexpr (SPARSE) {
        // (measured and not kept, 26 qubits / 26 channels: the encode in 32-bit halves 0.266 ms,
        // four words per lane with one 8-byte store 0.267, zeros first and then only the touched
        // words from an LDS list 0.307 (its one append counter serialises) — against 0.247 ms)
        uint16_t* out = static_cast<uint16_t*>(a.words) + K0;
        unsigned long long* ovf =
            reinterpret_cast<unsigned long long*>(static_cast<char*>(a.words) + sparse_ovf_offset(a.amps)) + K0;
        if (!(a.skip & 2))
            for (int i = t; i < R; i += kWordThreads) {
                bool over = false;
                out[i] = sparse_encode((unsigned long long)w[i], &over);
                if (over) ovf[i] = (unsigned long long)w[i];
            }
    } else {
        W* out = static_cast<W*>(a.words) + K0;
        if (!(a.skip & 2))
            for (int i = t; i < R; i += kWordThreads) out[i] = w[i];
    }
}

struct PullArgs {
    const double2* src;
    double2* dst;
    int bmap;            // work-group order (QSIM_PULL_BMAP; 0 with MAP)
    const void* words;
    uint64_t amps;       // amplitudes of this object (where sparse words keep their overflow words)
    uint64_t items;      // pairs (2x2 / diagonal) or amplitudes (SWAP / identity)
    int nch;
    int q[kMaxPullChannels];
    int kind;            // K_M1, K_DIAG, K_SWAP, or -1: identity
    int sub, t0, t1, d0_one;
    uint64_t cmask;
    double2 m[4];
};

// (P psi)[k] for a non-zero code word w of k: the fields from the highest down; a move (X / Y)
// re-reads the word at the new index, restricted to the channels below the one that moved it.
// The code word of amplitude k: dense (W per amplitude) or sparse (16-bit entries + overflow words).
template <class W, bool SPARSE>
struct WordSrc {
    const W* w;
    __device__ __forceinline__ W raw(uint64_t k) const { return w[k]; }
    __device__ __forceinline__ W full(uint64_t, W r) const { return r; }
    __device__ __forceinline__ W at(uint64_t k) const { return w[k]; }
};
template <class W>
struct WordSrc<W, true> {
    const uint16_t* w;
    const unsigned long long* ovf;
    __device__ __forceinline__ uint16_t raw(uint64_t k) const { return w[k]; }
    __device__ __forceinline__ W full(uint64_t k, uint16_t r) const { return sparse_decode<W>(r, ovf, k); }
    __device__ __forceinline__ W at(uint64_t k) const { return sparse_decode<W>(w[k], ovf, k); }
};
template <class W, class WS>
__device__ __forceinline__ double2 pull_walk(const PullArgs& a, const int* sq, const WS& words, uint64_t k, W w,
                                             double2 v) {
    int e = 0;  // phase i^e
    bool moved = false;
    int hi = a.nch;  // fields [0, hi) still to apply
    while (true) {
        const W m = hi >= (int)(4 * sizeof(W)) ? w : (w & (((W)1 << (2 * hi)) - 1));
        if (!m) break;
        const int c = (int)(8 * sizeof(W) - 1 - (sizeof(W) == 8 ? __clzll((long long)m) : __clz((int)m))) >> 1;
        const int code = (int)((w >> (2 * c)) & 3);
        const int q = sq[c];
        const int bit = (int)((k >> q) & 1ull);
        hi = c;
        if (code == 3) {  // Z: |1> <- -v[k1] (the index stays)
            if (bit) e += 2;
            continue;
        }
        if (code == 2) e += bit ? 1 : 3;  // Y: |0> <- -i v[k1], |1> <- +i v[k0]
        k ^= 1ull << q;                  // X / Y: the partner's amplitude
        moved = true;
        w = words.at(k);
    }
    if (moved) v = a.src[k];
    switch (e & 3) {
        case 1: return make_double2(-v.y, v.x);
        case 2: return make_double2(-v.x, -v.y);
        case 3: return make_double2(v.y, -v.x);
        default: return v;
    }
}

// U items per thread, all of their word and amplitude loads issued before any is used.
//   PAIR (2x2 with target >= 6): item = pair; both members' runs are contiguous across lanes.
//   else item = amplitude: a 2x2 on a target below 6 takes the partner from the lane 2^t0 away
//   (a wave holds both members), diagonals act per amplitude, SWAP / identity read their source.
// MAP: the work-group also builds the NEXT step's code words (m: its channels and keys, regions
// of 2^m.rl amplitudes, m.rpw of them per work-group) while its own loads are in flight — the word
// map's hash-and-log walks fill the pull pass's memory stalls instead of running as a kernel of
// their own beside it (the two share HBM and overlapped by ~2 %, profiles/r05/noisy_probe/).
constexpr int kMapRegionLog = 10;  // 1 024 amplitudes per region in the fused form
template <class W, bool MAP>
struct PullMapLds {
    W w[2 << kMapRegionLog];
};
template <class W>
struct PullMapLds<W, false> {
    W w[1];
};
template <class W, bool PAIR, int kPullU, bool NT, bool MAP = false, bool SPARSE = false>
__global__ __launch_bounds__(256) void k_pull_gate(PullArgs a, MapArgs m) {
    __shared__ int sq[kMaxPullChannels];
    __shared__ PullMapLds<W, MAP> lds;
    __shared__ FlipChan mchs[MAP ? kMaxPullChannels : 1];
    __shared__ int mtoff[MAP ? kMaxPullChannels + 1 : 1];
    if (threadIdx.x < kMaxPullChannels) sq[threadIdx.x] = a.q[threadIdx.x];
    if constexpr (MAP) {
        const int R = m.rpw << m.rl;
        for (int i = threadIdx.x; i < R; i += 256) lds.w[i] = 0;
        if ((int)threadIdx.x < m.nch) mchs[threadIdx.x] = m.ch[threadIdx.x];
        if ((int)threadIdx.x <= m.nch) mtoff[threadIdx.x] = m.task_off[threadIdx.x];
    }
    __syncthreads();
    // the next step's words for regions blockIdx.x * rpw .. + rpw - 1 (after this work-group's
    // loads are issued; their stores before its pulled walks)
    auto build_map = [&]() {
        if constexpr (MAP) {
            const int tasks = m.task_off[m.nch];
            for (int t = threadIdx.x; t < tasks * m.rpw; t += 256) {
                const int r = t / tasks;
                const uint64_t K0 = ((uint64_t)blockIdx.x * (uint64_t)m.rpw + (uint64_t)r) << m.rl;
                map_task(m, mchs, mtoff, lds.w + (r << m.rl), K0, t - r * tasks);
            }
            __syncthreads();
            W* out = static_cast<W*>(m.words) + (((uint64_t)blockIdx.x * (uint64_t)m.rpw) << m.rl);
            for (int i = threadIdx.x; i < (m.rpw << m.rl); i += 256) out[i] = lds.w[i];
        }
    };
    using Raw = std::conditional_t<SPARSE, uint16_t, W>;
    WordSrc<W, SPARSE> words;
    if constexpr (SPARSE) {
        words.w = static_cast<const uint16_t*>(a.words);
        words.ovf = reinterpret_cast<const unsigned long long*>(static_cast<const char*>(a.words) +
                                                                sparse_ovf_offset(a.amps));
    } else {
        words.w = static_cast<const W*>(a.words);
    }
    const uint64_t base = (xcd_block(a.bmap) * kPullU) << 8;
    // items is a multiple of 256, so each item group u (256 consecutive items) is wholly in or
    // wholly out of range for the whole work-group; groups past the end do nothing (a 9- or
    // 10-qubit state has fewer items than one work-group's kPullU groups)
    const int nu = (int)std::min<uint64_t>((uint64_t)kPullU, (a.items - std::min(a.items, base)) >> 8);
    if (nu == 0) {
        if constexpr (MAP) build_map();
        return;
    }
    if constexpr (PAIR) {
        uint64_t j0[kPullU];
        Raw w0[kPullU], w1[kPullU];
        double2 x0[kPullU], x1[kPullU];
#pragma unroll
        for (int u = 0; u < kPullU; ++u) {
            if (u >= nu) break;
            const uint64_t i = base + ((uint64_t)u << 8) + threadIdx.x;
            const uint64_t lo = i & ((1ull << a.t0) - 1ull);
            j0[u] = ((i ^ lo) << 1) | lo;
            const uint64_t j1 = j0[u] | (1ull << a.t0);
            w0[u] = words.raw(j0[u]);
            w1[u] = words.raw(j1);
            x0[u] = ld<NT>(a.src + j0[u]);
            x1[u] = ld<NT>(a.src + j1);
        }
        build_map();
#pragma unroll
        for (int u = 0; u < kPullU; ++u) {
            if (u >= nu) break;
            if (w0[u]) x0[u] = pull_walk<W>(a, sq, words, j0[u], words.full(j0[u], w0[u]), x0[u]);
            if (w1[u]) {
                const uint64_t j1 = j0[u] | (1ull << a.t0);
                x1[u] = pull_walk<W>(a, sq, words, j1, words.full(j1, w1[u]), x1[u]);
            }
            if ((j0[u] & a.cmask) == a.cmask) m1_pair(a.sub, a.m[0], a.m[1], a.m[2], a.m[3], x0[u], x1[u]);
            st<NT>(a.dst + j0[u], x0[u]);
            st<NT>(a.dst + (j0[u] | (1ull << a.t0)), x1[u]);
        }
    } else {
        uint64_t sk[kPullU];
        Raw w[kPullU];
        double2 x[kPullU];
#pragma unroll
        for (int u = 0; u < kPullU; ++u) {
            if (u >= nu) break;
            const uint64_t k = base + ((uint64_t)u << 8) + threadIdx.x;
            uint64_t s = k;
            if (a.kind == K_SWAP && (k & a.cmask) == a.cmask) {
                const uint64_t b0 = (k >> a.t0) & 1ull, b1 = (k >> a.t1) & 1ull;
                if (b0 != b1) s = k ^ ((1ull << a.t0) | (1ull << a.t1));
            }
            sk[u] = s;
            w[u] = words.raw(s);
            x[u] = ld<NT>(a.src + s);
        }
        build_map();
#pragma unroll
        for (int u = 0; u < kPullU; ++u) {
            if (u >= nu) break;
            const uint64_t k = base + ((uint64_t)u << 8) + threadIdx.x;
            if (w[u]) x[u] = pull_walk<W>(a, sq, words, sk[u], words.full(sk[u], w[u]), x[u]);
            double2 y = x[u];
            const bool on = (k & a.cmask) == a.cmask;
            const int bit = (int)((k >> a.t0) & 1ull);
            if (a.kind == K_M1) {  // (target < 6: the partner is lane ^ 2^t0 of this wave)
                double2 p;
                p.x = __shfl_xor(y.x, 1 << a.t0);
                p.y = __shfl_xor(y.y, 1 << a.t0);
                if (on) y = m1_half(a.sub, a.m[0], a.m[1], a.m[2], a.m[3], bit, y, p);
            } else if (a.kind == K_DIAG) {
                if (on) y = diag_apply(a.sub, a.d0_one, a.m[0], a.m[1], bit, y);
            }
            st<NT>(a.dst + k, y);
        }
    }
}

bool pull_noise_supported(int n, const std::vector<NoiseChan>& chans, bool default_on) {
    const char* e = std::getenv("QSIM_NOISE_PULL");  // (read per run: tests switch it)
    const bool on = e == nullptr ? default_on : std::atoi(e) != 0;
    if (!on || n < kMinPullQubits || chans.empty()) return false;
    int live = 0;
    for (const NoiseChan& c : chans) {
        if (!(c.type == 0 || c.type >= 3)) return false;  // damping channels stream every pair
        live += flip_probability(c.p) > 0.0;
    }
    return live <= kMaxPullChannels;
}

// Bytes of one step's code words: 4 per amplitude up to 16 channel entries, else 8.
size_t pull_noise_codes_bytes(int n, uint64_t batch, size_t nch) {
    const uint64_t amps = batch << n;
    const size_t dense = amps * (nch <= 16 ? sizeof(uint32_t) : sizeof(uint64_t));
    const size_t sparse = sparse_ovf_offset(amps) + amps * sizeof(unsigned long long);
    return std::max(dense, sparse);  // (either layout fits: QSIM_NOISE_SPARSE may change between runs)
}

// The live (can-fire) channels of one noise step, keyed like the push kernels' passes.
static void pull_channels(int n, const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t counter0,
                          MapArgs& m, PullArgs& a) {
    uint64_t counter = counter0;
    for (const NoiseChan& ch : chans) {
        check_channel(n, ch.type, ch.qubit, ch.p);
        const uint64_t key = noise_key(seed, counter++);
        if (m.nch >= kMaxPullChannels && flip_probability(ch.p) > 0.0)
            fail(QSIM_ERR_RUNTIME, "too many channels for the pulled noise path");
        if (!flip_channel(ch.type, ch.qubit, ch.p, key, m.ch[m.nch])) continue;
        a.q[m.nch] = ch.qubit;
        ++m.nch;
    }
    a.nch = m.nch;
}

void launch_noise_map(int n, uint64_t batch, uint64_t traj0, const std::vector<NoiseChan>& chans, uint64_t seed,
                      uint64_t counter0, void* words, hipStream_t s, Timer* tm) {
    if (n < kMinPullQubits) fail(QSIM_ERR_RUNTIME, "pulled noise needs >= 9 qubits");
    const uint64_t amps = batch << n;
    MapArgs m{};
    PullArgs a{};
    m.words = words;
    m.amps = amps;
    m.idx0 = traj0 << (n - 1);
    m.n = n;
    {  // QSIM_NOISE_REGION_LOG (9..12, default 12): amplitudes per word-map work-group (measurements)
        const char* re = std::getenv("QSIM_NOISE_REGION_LOG");
        const int rl = re ? std::max(9, std::min(kRegionLogMax, std::atoi(re))) : kRegionLogMax;
        m.rl = std::min(n, rl);
    }
    pull_channels(n, chans, seed, counter0, m, a);
    const char* ske = std::getenv("QSIM_MAP_SKIP");
    m.skip = ske ? std::atoi(ske) : 0;
    const bool sparse = noise_sparse_words();
    const size_t wb = sparse ? sizeof(uint16_t) : chans.size() <= 16 ? sizeof(uint32_t) : sizeof(uint64_t);
    if (!m.nch) {  // no channel can fire: every word zero
        QSIM_HIPCHK(hipMemsetAsync(words, 0, amps * wb, s));
        return;
    }
    for (int c = 0; c < m.nch; ++c)
        m.task_off[c + 1] = m.task_off[c] + (1 << (m.ch[c].target < m.rl ? m.rl - 9 : m.rl - 8));
    TimedLaunch tl(tm, "noise_map", 0.0, s);
    const dim3 grid((unsigned)(amps >> m.rl));
    // (256-thread work-groups: one round of 320 threads for the 320 walks of a 26-qubit region
    // shortens the map alone, 0.240 -> 0.218 ms, but the overlapped step loses: 1 112 -> 1 067
    // gates/s, profiles/r05/fast_log/)
    if (sparse) {
        if (chans.size() <= 16) hipLaunchKernelGGL((k_noise_words<uint32_t, true>), grid, dim3(kWordThreads), 0, s, m);
        else hipLaunchKernelGGL((k_noise_words<unsigned long long, true>), grid, dim3(kWordThreads), 0, s, m);
    } else if (wb == sizeof(uint32_t)) {
        hipLaunchKernelGGL(k_noise_words<uint32_t>, grid, dim3(kWordThreads), 0, s, m);
    } else {
        hipLaunchKernelGGL(k_noise_words<unsigned long long>, grid, dim3(kWordThreads), 0, s, m);
    }
    QSIM_HIPCHK(hipGetLastError());
}

void launch_pull_gate(const double2* src, double2* dst, int n, uint64_t batch, const std::vector<NoiseChan>& chans,
                      const Op* op, const void* words, hipStream_t s, Timer* tm, const PullMapNext* next) {
    const uint64_t amps = batch << n, pairs = amps >> 1;
    MapArgs m{};
    PullArgs a{};
    pull_channels(n, chans, 0, 0, m, a);  // (the live channels and their qubits; keys unused)
    // the next step's words built by this pass (below), or by the word map before it
    MapArgs nm{};
    bool fuse = false;
    if (next) {
        PullArgs tmp{};
        nm.words = next->words;
        nm.amps = amps;
        nm.idx0 = next->traj0 << (n - 1);
        nm.n = n;
        nm.rl = std::min(n, kMapRegionLog);
        pull_channels(n, chans, next->seed, next->counter0, nm, tmp);
        for (int c = 0; c < nm.nch; ++c)
            nm.task_off[c + 1] = nm.task_off[c] + (1 << (nm.ch[c].target < nm.rl ? nm.rl - 9 : nm.rl - 8));
        fuse = nm.nch > 0;
        if (!fuse) launch_noise_map(n, batch, next->traj0, chans, next->seed, next->counter0, next->words, s, tm);
    }
    a.src = src;
    a.dst = dst;
    a.words = words;
    a.amps = amps;
    a.bmap = fuse ? 0 : env_bmap("QSIM_PULL_BMAP", 0);
    a.kind = op ? op->kind : -1;
    if (op) {
        a.sub = op->sub;
        a.t0 = op->t0;
        a.t1 = op->t1;
        a.d0_one = op->d0_one ? 1 : 0;
        a.cmask = op->cmask;
        for (int i = 0; i < 4; ++i) a.m[i] = make_double2(op->m[2 * i], op->m[2 * i + 1]);
    }
    const bool pair = a.kind == K_M1 && a.t0 >= 6;
    a.items = pair ? pairs : amps;  // (multiples of 256: n >= 9)
    if (n < kMinPullQubits || a.items % 256 != 0) fail(QSIM_ERR_RUNTIME, "pulled noise pass: bad shape");
    if (!pair && a.kind == K_M1 && a.t0 >= 6) fail(QSIM_ERR_RUNTIME, "pulled noise pass: lane partner");
    // QSIM_PULL_U (items per thread, 1 / 2 / 4 / 8), QSIM_PULL_NT (non-temporal amplitude
    // traffic, default 1): read per launch (measurement sweeps)
    const char* ue = std::getenv("QSIM_PULL_U");
    const char* ne = std::getenv("QSIM_PULL_NT");
    const bool sparse = noise_sparse_words();
    // (sparse words: 2 items per thread by default — NoisySimulator 26q / 26 channels 1 169 -> 1 257
    // gates/s: twice the work-groups interleave better with the next step's word map on the
    // other stream; 8 items 956; dense words keep 4)
    const int U = ue ? std::atoi(ue) : (sparse ? 2 : 4);
    const bool nt = ne == nullptr || std::atoi(ne) != 0;
    const int Uc = U <= 1 ? 1 : U == 2 ? 2 : (U >= 8 ? 8 : 4);
    const dim3 grid((unsigned)((a.items + 256 * Uc - 1) / (256 * Uc)));
    const bool w32 = chans.size() <= 16;
    if (fuse && sparse) {  // (the fused map writes dense words: build them apart instead)
        fuse = false;
        launch_noise_map(n, batch, next->traj0, chans, next->seed, next->counter0, next->words, s, tm);
    }
    if (fuse) {  // the fused form: 4 items per thread, non-temporal, 1 or 2 whole regions per group
        const uint64_t regions = amps >> nm.rl;
        nm.rpw = (int)(regions / grid.x);
        if (Uc != 4 || !nt || (nm.rpw != 1 && nm.rpw != 2) || (uint64_t)nm.rpw * grid.x != regions) {
            fuse = false;
            launch_noise_map(n, batch, next->traj0, chans, next->seed, next->counter0, next->words, s, tm);
        }
    }
    TimedLaunch tl(tm, fuse ? "pull_gate_map" : "pull_gate", 32.0 * (double)amps, s);
    if (fuse) {
        if (w32) {
            if (pair) hipLaunchKernelGGL((k_pull_gate<uint32_t, true, 4, true, true>), grid, dim3(256), 0, s, a, nm);
            else hipLaunchKernelGGL((k_pull_gate<uint32_t, false, 4, true, true>), grid, dim3(256), 0, s, a, nm);
        } else {
            if (pair) hipLaunchKernelGGL((k_pull_gate<unsigned long long, true, 4, true, true>), grid, dim3(256), 0, s, a, nm);
            else hipLaunchKernelGGL((k_pull_gate<unsigned long long, false, 4, true, true>), grid, dim3(256), 0, s, a, nm);
        }
        QSIM_HIPCHK(hipGetLastError());
        return;
    }
#define QSIM_PULL_LAUNCH(W_, UU, NTT)                                                                      \
    do {                                                                                                 \
        if (sparse && pair) hipLaunchKernelGGL((k_pull_gate<W_, true, UU, NTT, false, true>), grid, dim3(256), 0, s, a, m); \
        else if (sparse) hipLaunchKernelGGL((k_pull_gate<W_, false, UU, NTT, false, true>), grid, dim3(256), 0, s, a, m); \
        else if (pair) hipLaunchKernelGGL((k_pull_gate<W_, true, UU, NTT>), grid, dim3(256), 0, s, a, m); \
        else hipLaunchKernelGGL((k_pull_gate<W_, false, UU, NTT>), grid, dim3(256), 0, s, a, m);        \
    } while (0)
#define QSIM_PULL_LAUNCH_U(W_, NTT)                  \
    do {                                           \
        if (Uc == 1) QSIM_PULL_LAUNCH(W_, 1, NTT);  \
        else if (Uc == 2) QSIM_PULL_LAUNCH(W_, 2, NTT);  \
        else if (Uc == 8) QSIM_PULL_LAUNCH(W_, 8, NTT); \
        else QSIM_PULL_LAUNCH(W_, 4, NTT);         \
    } while (0)
    if (w32) {
        if (nt) QSIM_PULL_LAUNCH_U(uint32_t, true);
        else QSIM_PULL_LAUNCH_U(uint32_t, false);
    } else {
        if (nt) QSIM_PULL_LAUNCH_U(unsigned long long, true);
        else QSIM_PULL_LAUNCH_U(unsigned long long, false);
    }
#undef QSIM_PULL_LAUNCH_U
#undef QSIM_PULL_LAUNCH
    QSIM_HIPCHK(hipGetLastError());
}

void launch_pull_noise_step(const double2* src, double2* dst, int n, uint64_t batch, uint64_t traj0,
                            const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t counter0,
                            const Op* op, void* words, hipStream_t s, Timer* tm) {
    launch_noise_map(n, batch, traj0, chans, seed, counter0, words, s, tm);
    launch_pull_gate(src, dst, n, batch, chans, op, words, s, tm);
}

}  // namespace qsim_hip

namespace qsim_hip {
// draws single-precision-first gaps (flip_gap) against the double formula: out[0] mismatches,
// out[1] draws that fell back to the double log
__global__ __launch_bounds__(256) void k_gap_check(FlipChan c, uint64_t key, uint64_t draws,
                                                   unsigned long long* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long mm = 0, fb = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < draws; i += stride) {
        const uint64_t h = nz_mix(key + i * 0x9e3779b97f4a7c15ull);
        bool f = false;
        const double g = flip_gap(h, c, &f);
        const double u = (double)((h >> 11) + 1ull) * 0x1.0p-53;
        const double ref = floor(log(u) / c.lq), blk = (double)kFlipBlock;
        if (!((g < blk ? g : blk) == (ref < blk ? ref : blk))) ++mm;
        fb += f ? 1ull : 0ull;
    }
    if (mm) atomicAdd(&out[0], mm);
    if (fb) atomicAdd(&out[1], fb);
}
// The same comparison on targeted draws: every u index K in [center - half, center + half) of each
// center (the host's boundary candidates, qsim_noise_gap_check_edges), u = (K + 1) 2^-53.
__global__ __launch_bounds__(256) void k_gap_edges(FlipChan c, const uint64_t* centers, uint64_t ncent,
                                                   uint64_t half, unsigned long long* out) {
    const uint64_t per = 2 * half, total = ncent * per;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long mm = 0, fb = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t ctr = centers[i / per];
        const uint64_t off = i % per;
        const uint64_t K = ctr + off >= half ? ctr + off - half : 0;
        if (K >= (1ull << 53)) continue;
        const uint64_t h = K << 11;
        bool f = false;
        const double g = flip_gap(h, c, &f);
        const double u = (double)((h >> 11) + 1ull) * 0x1.0p-53;
        const double ref = floor(log(u) / c.lq), blk = (double)kFlipBlock;
        if (!((g < blk ? g : blk) == (ref < blk ? ref : blk))) ++mm;
        fb += f ? 1ull : 0ull;
    }
    if (mm) atomicAdd(&out[0], mm);
    if (fb) atomicAdd(&out[1], fb);
}
}  // namespace qsim_hip

// Targeted boundary sweep: the single-precision first try of flip_gap can only be wrong
// where ln u / lq lies within its error of an integer m.  For every m in [0, 256] the centers are the
// double boundary u_m = exp(m lq) and both ends of the interval of doubles that round to the float
// nearest u_m (where the float path's input is fixed while the double answer changes), each swept
// over 2 x half consecutive u indices.
extern "C" int qsim_noise_gap_check_edges(double p, uint64_t half, uint64_t* mismatches, uint64_t* fallbacks,
                                          uint64_t* draws) {
    using namespace qsim_hip;
    if (!mismatches || !fallbacks || !draws || !(p > 0.0) || p > 1.0 || half == 0 || half > (1ull << 24))
        return QSIM_ERR_INVALID_ARGUMENT;
    FlipChan c{};
    if (!flip_channel(0, 0, p, 0, c) || c.always) {
        *mismatches = *fallbacks = *draws = 0;
        return QSIM_OK;
    }
    std::vector<uint64_t> cent;
    auto kof = [](double u) -> uint64_t {  // u index K with (K + 1) 2^-53 nearest u
        const double k = std::floor(u * 0x1.0p53) - 1.0;
        return k < 0.0 ? 0ull : (k >= 0x1.0p53 ? (1ull << 53) - 1 : (uint64_t)k);
    };
    for (int m = 0; m <= (int)kFlipBlock; ++m) {
        const double um = std::exp((double)m * c.lq);
        if (!(um > 0.0)) break;
        cent.push_back(kof(um));
        const float uf = (float)um;
        const double lo = 0.5 * ((double)std::nextafter(uf, 0.0f) + (double)uf);
        const double hi = 0.5 * ((double)uf + (double)std::nextafter(uf, 2.0f));
        cent.push_back(kof(lo));
        cent.push_back(kof(std::min(hi, 1.0)));
    }
    uint64_t* d_c = nullptr;
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d_c, cent.size() * sizeof(uint64_t)) != hipSuccess) return QSIM_ERR_DEVICE;
    if (hipMalloc((void**)&d, 2 * sizeof(unsigned long long)) != hipSuccess) {
        (void)hipFree(d_c);
        return QSIM_ERR_DEVICE;
    }
    unsigned long long hcnt[2] = {0, 0};
    bool ok = hipMemcpy(d_c, cent.data(), cent.size() * sizeof(uint64_t), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemset(d, 0, sizeof(hcnt)) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_gap_edges, dim3(1024), dim3(256), 0, 0, c, d_c, (uint64_t)cent.size(), half, d);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(hcnt, d, sizeof(hcnt), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    (void)hipFree(d_c);
    if (!ok) return QSIM_ERR_DEVICE;
    *mismatches = hcnt[0];
    *fallbacks = hcnt[1];
    *draws = (uint64_t)cent.size() * 2 * half;
    return QSIM_OK;
}

extern "C" int qsim_noise_gap_check(double p, uint64_t draws, uint64_t key, uint64_t* mismatches,
                                    uint64_t* fallbacks) {
    using namespace qsim_hip;
    if (!mismatches || !fallbacks || !(p > 0.0) || p > 1.0) return QSIM_ERR_INVALID_ARGUMENT;
    FlipChan c{};
    if (!flip_channel(0, 0, p, key, c) || c.always) {  // (nothing to draw: no gaps)
        *mismatches = *fallbacks = 0;
        return QSIM_OK;
    }
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(unsigned long long)) != hipSuccess) return QSIM_ERR_DEVICE;
    unsigned long long hcnt[2] = {0, 0};
    bool ok = hipMemset(d, 0, sizeof(hcnt)) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_gap_check, dim3(1024), dim3(256), 0, 0, c, key, draws, d);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(hcnt, d, sizeof(hcnt), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    if (!ok) return QSIM_ERR_DEVICE;
    *mismatches = hcnt[0];
    *fallbacks = hcnt[1];
    return QSIM_OK;
}

extern "C" int qsim_noise_check_flips(uint64_t* flips) {
    if (!flips) return QSIM_ERR_INVALID_ARGUMENT;
    *flips = qsim_hip::noise_check_flips;
    return QSIM_OK;
}
