// batched.hip — B independent trajectories of 2^n amplitudes (reference BatchedSimulator,
// include/NoiseModel.cuh:231-297, src/NoiseModel.cu:653-972) with Monte-Carlo Pauli noise.
//
// Layout: trajectory-major [B][2^n] like the reference (d_states_, NoiseModel.cu:657-673), so
// each gate is the single-state kernel with a batch dimension (launch_op(..., batch, ...)).
//
// Noise (deliberate redesign): the reference draws one curand number per amplitude
// PAIR and keeps a 48-B curandState per pair (1.5 GiB at 16q x 1024).  Here each trajectory
// draws once per channel per gate from a stateless counter hash keyed by (seed, step, channel,
// trajectory); the Pauli picks of all channels of one gate are composed into one Pauli string
// i^e X^x Z^z per trajectory, and only trajectories whose string is not the identity are
// touched (one read+write of that trajectory).  This is the physical depolarizing channel on a
// pure-state trajectory; statistics, not per-trajectory realizations, match the reference.
// Channel types the reference batched mode ignores (F5: only Depolarizing) are Pauli-free here
// too: BitFlip/PhaseFlip/BitPhaseFlip are applied (X/Z/Y), damping channels are ignored.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "device_ops.hpp"
#include "engine.hpp"
#include "qsim_hip.h"

using namespace qsim_hip;

namespace qsim_hip {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// uniform double in [0,1) from 53 bits
__device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

struct DevChannel {
    int type;
    int qubit;
    double p;
};

// This step's Pauli picks of trajectory b, composed into i^e X^x Z^z (channels in order).
// b is the GLOBAL trajectory index (qsim_batch_set_trajectory_offset): a sharded ensemble draws
// exactly what one object holding every trajectory draws.
__device__ __forceinline__ void draw_step(const DevChannel* ch, int nch, uint64_t seed, uint64_t step,
                                          uint64_t b, uint64_t& x, uint64_t& z, int& e) {
    x = 0;
    z = 0;
    e = 0;
    for (int c = 0; c < nch; ++c) {
        const uint64_t key = mix64(seed ^ mix64(step * 0x100000001b3ull + (uint64_t)c) ^
                                   (b << 20));
        const double r1 = u01(mix64(key));
        int pauli = 0;  // 1 X, 2 Y, 3 Z
        const int t = ch[c].type;
        if (r1 < ch[c].p) {
            if (t == 0) {  // depolarizing: uniform X/Y/Z (reference thresholds 1/3, 2/3)
                const double r2 = u01(mix64(key ^ 0x5bd1e995ull));
                pauli = r2 < 1.0 / 3.0 ? 1 : (r2 < 2.0 / 3.0 ? 2 : 3);
            } else if (t == 3) pauli = 1;       // bit flip
            else if (t == 4) pauli = 3;         // phase flip
            else if (t == 5) pauli = 2;         // bit-phase flip
        }
        if (!pauli) continue;
        const uint64_t q = 1ull << ch[c].qubit;
        if (pauli == 1) {
            x ^= q;
        } else if (pauli == 3) {
            if (x & q) e += 2;
            z ^= q;
        } else {  // Y = i X Z
            e += 1 + ((x & q) ? 2 : 0);
            x ^= q;
            z ^= q;
        }
    }
    e &= 3;
}

// One thread per trajectory: compose this step's Pauli picks into (e, x, z).
__global__ void k_pauli_draw(const DevChannel* ch, int nch, uint64_t seed, uint64_t step,
                             int batch, uint64_t traj0, uint64_t* xz, int* ephase) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    uint64_t x, z;
    int e;
    draw_step(ch, nch, seed, step, traj0 + (uint64_t)b, x, z, e);
    xz[2 * b] = x;
    xz[2 * b + 1] = z;
    ephase[b] = e;
}

// Pauli frames for a whole run.  With the frame Phi = i^E X^F Z^G (state = Phi * stored vector),
// the noise P = i^e X^x Z^z after step s updates Phi <- P Phi = i^(e+E) (-1)^popc(z & F)
// X^(x^F) Z^(z^G); frames[s] is the frame in force BEFORE gate s (gates are applied to the stored
// vector conjugated by it, fused.hip), fin the frame after the last step (materialised with
// k_pauli_apply).  Same draws as k_pauli_draw.  Two kernels: every (step, trajectory) draw in
// parallel (written into frames[s] as (x, z) plus ephase[s]), then one thread per trajectory
// scans the steps in order, replacing each draw by the frame before it.
__global__ void k_draw_steps(const DevChannel* ch, int nch, uint64_t seed, uint64_t step0,
                             int count, int batch, uint64_t traj0, uint64_t* frames, int* ephase) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)count * batch) return;
    const int s = (int)(i / batch), b = (int)(i - (uint64_t)s * batch);
    uint64_t x, z;
    int e;
    draw_step(ch, nch, seed, step0 + (uint64_t)s, traj0 + (uint64_t)b, x, z, e);
    frames[2 * i] = x;
    frames[2 * i + 1] = z;
    ephase[i] = e;
}

// Clifford gates move the frame instead of being conjugated by it (Pauli-frame propagation):
// for a Clifford U, U Phi = (U Phi U^dag) U, so U runs on the stored vector unchanged and the
// frame becomes U Phi U^dag — again a Pauli.  Per step: {code, q0, q1}; code 0 = not Clifford (the
// gate is conjugated by the frame in the pass kernels instead).  Rules for Phi = i^E X^F Z^G:
//   X_q: E += 2 G_q            Z_q: E += 2 F_q              Y_q: E += 2 (F_q ^ G_q)
//   H_q: swap F_q, G_q; E += 2 (F_q & G_q)
//   S_q: G_q ^= F_q; E += F_q   Sdag_q: G_q ^= F_q; E += 3 F_q
//   CNOT(c, t): F_t ^= F_c; G_c ^= G_t      CZ(a, b): G_a ^= F_b; G_b ^= F_a; E += 2 (F_a & F_b)
//   SWAP(a, b): exchange bits a and b of F and of G.
enum CliffordCode : int { CL_NONE = 0, CL_X, CL_Y, CL_Z, CL_H, CL_S, CL_SDG, CL_CNOT, CL_CZ, CL_SWAP };
struct StepClifford {
    int code, q0, q1, _pad;
};

__device__ __forceinline__ void clifford_update(const StepClifford& c, uint64_t& F, uint64_t& G, int& E) {
    const uint64_t a = 1ull << c.q0, bm = 1ull << (c.q1 < 0 ? 0 : c.q1);
    const int fa = (F & a) != 0, ga = (G & a) != 0;
    switch (c.code) {
        case CL_X: E += 2 * ga; break;
        case CL_Z: E += 2 * fa; break;
        case CL_Y: E += 2 * (fa ^ ga); break;
        case CL_H:
            E += 2 * (fa & ga);
            F = (F & ~a) | (ga ? a : 0ull);
            G = (G & ~a) | (fa ? a : 0ull);
            break;
        case CL_S: E += fa; if (fa) G ^= a; break;
        case CL_SDG: E += 3 * fa; if (fa) G ^= a; break;
        case CL_CNOT: {  // q0 control, q1 target
            if (fa) F ^= bm;
            if (G & bm) G ^= a;
            break;
        }
        case CL_CZ: {
            const int fb = (F & bm) != 0;
            E += 2 * (fa & fb);
            if (fb) G ^= a;
            if (fa) G ^= bm;
            break;
        }
        case CL_SWAP: {
            const int fb = (F & bm) != 0, gb = (G & bm) != 0;
            F = (F & ~(a | bm)) | (fb ? a : 0ull) | (fa ? bm : 0ull);
            G = (G & ~(a | bm)) | (gb ? a : 0ull) | (ga ? bm : 0ull);
            break;
        }
        default: break;
    }
}

// carry: start from the frame in fin_xz / fin_e (the last run's, not materialised) instead of 1.
__global__ void k_frame_build(int count, int batch, uint64_t* frames, const int* ephase,
                              const StepClifford* cl, uint64_t* fin_xz, int* fin_e, int carry) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    uint64_t F = carry ? fin_xz[2 * b] : 0ull, G = carry ? fin_xz[2 * b + 1] : 0ull;
    int E = carry ? fin_e[b] : 0;
    for (int s = 0; s < count; ++s) {
        const uint64_t i = (uint64_t)s * batch + b;
        uint64_t* fr = frames + 2 * i;
        const uint64_t x = fr[0], z = fr[1];
        fr[0] = F;  // the frame gate s is conjugated by (when it is not Clifford)
        fr[1] = G;
        clifford_update(cl[s], F, G, E);
        E += ephase[i] + ((__popcll(z & F) & 1) ? 2 : 0);  // then this step's noise: P Phi
        F ^= x;
        G ^= z;
    }
    fin_xz[2 * b] = F;
    fin_xz[2 * b + 1] = G;
    fin_e[b] = E & 3;
}

__device__ __forceinline__ double2 mul_ipow(double2 a, int e) {
    switch (e & 3) {
        case 1: return make_double2(-a.y, a.x);
        case 2: return make_double2(-a.x, -a.y);
        case 3: return make_double2(a.y, -a.x);
        default: return a;
    }
}

// new[j] = i^e (-1)^{popc(z & (j^x))} old[j^x]; pairs (j, j^x) with bit h of j == 0.
__global__ __launch_bounds__(256) void k_pauli_apply(double2* st, int n, const uint64_t* xz,
                                                     const int* ephase, uint64_t items_per_traj) {
    const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t b = item / items_per_traj;
    const uint64_t k = item - b * items_per_traj;
    const uint64_t x = xz[2 * b], z = xz[2 * b + 1];
    const int e = ephase[b];
    if (x == 0 && z == 0 && e == 0) return;
    double2* s = st + (b << n);
    if (x == 0) {  // diagonal: k enumerates all 2^n amplitudes (items_per_traj == 2^(n-1)): 2 each
        for (int r = 0; r < 2; ++r) {
            const uint64_t j = 2 * k + r;
            const double2 a = s[j];
            const int sign = __popcll(z & j) & 1;
            double2 v = mul_ipow(a, e + 2 * sign);
            s[j] = v;
        }
        return;
    }
    const int h = 63 - __clzll(x);
    const uint64_t lo = k & ((1ull << h) - 1ull);
    const uint64_t j = ((k ^ lo) << 1) | lo;  // bit h == 0
    const uint64_t jp = j ^ x;
    const double2 a = s[j], ap = s[jp];
    // new[j] uses old[jp]; sign from z & (j ^ x) = z & jp
    const double2 nj = mul_ipow(ap, e + 2 * (__popcll(z & jp) & 1));
    const double2 njp = mul_ipow(a, e + 2 * (__popcll(z & j) & 1));
    s[j] = nj;
    s[jp] = njp;
}

}  // namespace qsim_hip

struct qsim_batch {
    int n = 0, batch = 0, device = 0;
    double2* d = nullptr;
    hipStream_t stream = nullptr;
    uint64_t seed = 0, step = 0;
    uint64_t traj0 = 0;     // global index of trajectory 0 (trajectory-sharded ensembles)
    uint64_t ncounter = 0;  // per-pair noise passes so far (QSIM_BATCH_REFERENCE_NOISE)
    uint64_t* d_xz = nullptr;
    int* d_e = nullptr;
    DevChannel* d_ch = nullptr;
    size_t ch_cap = 0;
    uint64_t* d_frames = nullptr;  // Pauli frames of the current run, [steps][batch][2]
    int* d_fe = nullptr;           // per-(step, trajectory) draw phases (frame build scratch)
    size_t frames_cap = 0;
    DevBuf ops, stages;             // fused-plan descriptors
    DevBuf cliff;                   // per-step Clifford codes of the current run (frame build)
    PlanCache plans;
    Timer timer;
    Scratch scratch, scratch2;
    int last_passes = 0, last_jit_passes = 0;
    // Layout-aware relabeling (relabel.hip) of the qubits inside every trajectory: logical q at
    // physical perm[q] (empty: identity); basis: every trajectory is |0..0> (create / reset).
    std::vector<int> perm;
    bool basis = true;
    // The Pauli frames of the last fused noisy run (d_xz, d_e; physical positions) are not yet
    // materialised: every trajectory's state is Phi * stored vector.  The next fused run starts
    // its frame build from them (frames compose: no Pauli pass per run); everything that reads
    // or writes amplitudes otherwise materialises them first (materialize), and so does sync.
    bool frame_pending = false;
    // Pulled reference noise (noise.hip: launch_pull_noise_step) writes out of place: the
    // ensemble alternates between d0 (allocated at create) and d1 (allocated on the first pulled
    // run when the device has room; otherwise the push kernels run).  d is the current one.
    // pinned: a raw pointer to d0 was handed out, so a run that ends in d1 copies back.
    double2* d0 = nullptr;
    double2* d1 = nullptr;
    // Two sets of per-step code words (one per amplitude; noise steps alternate), so the next
    // step's words are built on map_stream while this step's pass runs.
    unsigned char* d_codes = nullptr;
    size_t codes_cap = 0;           // bytes of ONE set
    // Two sets of per-step flip lists of the in-tile noise kernel (noise.hip: k_gn_lists), built
    // on map_stream one step ahead.
    char* d_lists = nullptr;
    size_t lists_cap = 0;           // bytes of ONE set
    // QSIM_NOISE_SPLIT=k (default 2): the in-tile path runs the ensemble as k trajectory parts on
    // k streams (part 0 on `stream`), so one part's tile pass can overlap another's suffix push
    struct SplitPart {
        hipStream_t s = nullptr, ms = nullptr;
        hipEvent_t built[2] = {}, used[2] = {}, start = nullptr, fork = nullptr, join = nullptr;
        char* lists = nullptr;
        size_t cap = 0;
    };
    std::vector<SplitPart> split;
    hipStream_t map_stream = nullptr;
    hipEvent_t ev_map[2] = {}, ev_pull[2] = {}, ev_start = nullptr;
    bool pinned = false;
    ~qsim_batch() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (map_stream) (void)hipStreamSynchronize(map_stream);
        for (hipEvent_t e : {ev_map[0], ev_map[1], ev_pull[0], ev_pull[1], ev_start})
            if (e) (void)hipEventDestroy(e);
        if (map_stream) (void)hipStreamDestroy(map_stream);
        if (d0) (void)hipFree(d0);
        if (d1) (void)hipFree(d1);
        if (d_codes) (void)hipFree(d_codes);
        if (d_lists) (void)hipFree(d_lists);
        for (SplitPart& p : split) {
            if (p.s) (void)hipStreamSynchronize(p.s);
            if (p.ms) (void)hipStreamSynchronize(p.ms);
            for (hipEvent_t e : {p.built[0], p.built[1], p.used[0], p.used[1], p.start, p.fork, p.join})
                if (e) (void)hipEventDestroy(e);
            if (p.s) (void)hipStreamDestroy(p.s);
            if (p.ms) (void)hipStreamDestroy(p.ms);
            if (p.lists) (void)hipFree(p.lists);
        }
        if (d_xz) (void)hipFree(d_xz);
        if (d_e) (void)hipFree(d_e);
        if (d_ch) (void)hipFree(d_ch);
        if (d_frames) (void)hipFree(d_frames);
        if (d_fe) (void)hipFree(d_fe);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {
template <typename F>
int bguard(F&& f) {
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
void need(const qsim_batch* b) {
    if (!b) fail(QSIM_ERR_INVALID_ARGUMENT, "null batch handle");
}
qsim_gate map_gate(const qsim_batch* b, const qsim_gate& g) {
    qsim_gate m = g;
    if (!b->perm.empty())
        for (int j = 0; j < g.nqubits && j < 3; ++j)
            if (g.qubits[j] >= 0 && g.qubits[j] < b->n) m.qubits[j] = b->perm[g.qubits[j]];
    return m;
}
// The ensemble back in its first buffer (after a pulled run that ended in the second one).
void settle_in_d0(qsim_batch* b) {
    if (b->d == b->d0) return;
    QSIM_HIPCHK(hipMemcpyAsync(b->d0, b->d, ((uint64_t)b->batch * sizeof(double2)) << b->n,
                               hipMemcpyDeviceToDevice, b->stream));
    b->d = b->d0;
}
// map_stream and its events (the pulled path's word maps, the tile path's flip lists).
void ensure_map_stream(qsim_batch* b) {
    if (b->map_stream) return;
    // QSIM_NOISE_STREAM_PRIO (experiments): 1 = the side stream at the lowest priority, so the
    // list builds yield the CUs to the main stream's kernels
    const char* pe = std::getenv("QSIM_NOISE_STREAM_PRIO");
    if (pe && std::atoi(pe) != 0) {
        int lo = 0, hi = 0;
        QSIM_HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        QSIM_HIPCHK(hipStreamCreateWithPriority(&b->map_stream, hipStreamNonBlocking, lo));
    } else {
        QSIM_HIPCHK(hipStreamCreateWithFlags(&b->map_stream, hipStreamNonBlocking));
    }
    for (hipEvent_t* e : {&b->ev_map[0], &b->ev_map[1], &b->ev_pull[0], &b->ev_pull[1], &b->ev_start})
        QSIM_HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
}
// Two sets of flip lists of `bytes` each, when the device has room beside a margin (false: the
// tile kernels walk the blocks themselves).
bool ensure_list_buffers(qsim_batch* b, size_t bytes) {
    if (bytes > b->lists_cap) {
        if (b->d_lists) {
            QSIM_HIPCHK(hipStreamSynchronize(b->stream));
            if (b->map_stream) QSIM_HIPCHK(hipStreamSynchronize(b->map_stream));
            (void)hipFree(b->d_lists);
            b->d_lists = nullptr;
            b->lists_cap = 0;
        }
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (free_b < 2 * bytes + (256ull << 20)) return false;
        if (hipMalloc((void**)&b->d_lists, 2 * bytes) != hipSuccess) {
            (void)hipGetLastError();
            b->d_lists = nullptr;
            return false;
        }
        b->lists_cap = bytes;
    }
    ensure_map_stream(b);
    return true;
}
// The in-tile run over k trajectory parts on k streams (QSIM_NOISE_SPLIT, default 2): part 0 on the object's
// stream with its list sets, part j > 0 on a stream of its own with its own side stream and lists;
// every part draws with the global pair index, so the states are the one-part run's.  false (nothing
// launched): a part's list buffers do not fit beside the margin ensure_list_buffers keeps — the
// caller runs the ensemble as one part instead (a near-full device must not turn a run
// that fits as one part into an error).
bool split_tile_run(qsim_batch* b, const std::vector<Op>& ops, const std::vector<NoiseChan>& dep, int k,
                    const GnLists& L0) {
    const uint64_t B = (uint64_t)b->batch;
    if ((int)b->split.size() < k - 1) b->split.resize(k - 1);
    const uint64_t c0 = b->ncounter;
    uint64_t c_end = c0;
    std::vector<GnLists> Ls(k);
    std::vector<uint64_t> first(k + 1);
    for (int j = 0; j <= k; ++j) first[j] = B * (uint64_t)j / (uint64_t)k;
    Ls[0] = L0;
    for (int j = 1; j < k; ++j) {  // every part's list buffers first, so a refusal launches nothing
        qsim_batch::SplitPart& p = b->split[j - 1];
        const size_t lb = gate_noise_lists_bytes(b->n, first[j + 1] - first[j], dep);
        if (lb <= p.cap) continue;
        if (p.lists) {
            QSIM_HIPCHK(hipStreamSynchronize(p.s));
            QSIM_HIPCHK(hipStreamSynchronize(p.ms));
            (void)hipFree(p.lists);
            p.lists = nullptr;
            p.cap = 0;
        }
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (free_b < 2 * lb + (256ull << 20)) return false;
        if (hipMalloc((void**)&p.lists, 2 * lb) != hipSuccess) {
            (void)hipGetLastError();
            p.lists = nullptr;
            return false;
        }
        p.cap = lb;
    }
    for (int j = 1; j < k; ++j) {
        qsim_batch::SplitPart& p = b->split[j - 1];
        if (!p.s) {
            QSIM_HIPCHK(hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking));
            QSIM_HIPCHK(hipStreamCreateWithFlags(&p.ms, hipStreamNonBlocking));
            for (hipEvent_t* e : {&p.built[0], &p.built[1], &p.used[0], &p.used[1], &p.start, &p.fork, &p.join})
                QSIM_HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        }
        GnLists& L = Ls[j];
        L.buf[0] = p.lists;
        L.buf[1] = p.lists + p.cap;
        L.set_bytes = p.cap;
        L.ms = p.ms;
        L.built[0] = p.built[0];
        L.built[1] = p.built[1];
        L.used[0] = p.used[0];
        L.used[1] = p.used[1];
        L.start = p.start;
        QSIM_HIPCHK(hipEventRecord(p.fork, b->stream));  // (after everything before this run)
        QSIM_HIPCHK(hipStreamWaitEvent(p.s, p.fork, 0));
    }
    for (int j = 0; j < k; ++j) {
        hipStream_t sj = j == 0 ? b->stream : b->split[j - 1].s;
        uint64_t c = c0;
        launch_gate_noise_run(b->d + (first[j] << b->n), b->n, first[j + 1] - first[j], b->traj0 + first[j], ops, dep,
                              b->seed, c, sj, &b->timer, &Ls[j]);
        c_end = c;
    }
    for (int j = 1; j < k; ++j) {
        QSIM_HIPCHK(hipEventRecord(b->split[j - 1].join, b->split[j - 1].s));
        QSIM_HIPCHK(hipStreamWaitEvent(b->stream, b->split[j - 1].join, 0));
    }
    b->ncounter = c_end;
    return true;
}
// Buffers of the pulled noise path (second ensemble buffer, flip codes, touched bits), allocated
// when the device has room for them beside a margin; false: run the push kernels instead.
bool ensure_pull_buffers(qsim_batch* b, size_t nch) {
    const uint64_t amps = (uint64_t)b->batch << b->n;
    const size_t state_b = amps * sizeof(double2);
    const size_t codes_b = pull_noise_codes_bytes(b->n, (uint64_t)b->batch, nch);
    size_t need_b = (b->d1 ? 0 : state_b) + (codes_b > b->codes_cap ? 2 * codes_b : 0);
    if (need_b == 0) return true;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (free_b < need_b + (256ull << 20)) return false;
    auto grab = [&](void** p, size_t bytes) {
        if (hipMalloc(p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            return false;
        }
        return true;
    };
    if (!b->d1 && !grab((void**)&b->d1, state_b)) return false;
    if (codes_b > b->codes_cap) {
        if (b->d_codes) {
            QSIM_HIPCHK(hipStreamSynchronize(b->stream));
            (void)hipFree(b->d_codes);
            b->d_codes = nullptr;
            b->codes_cap = 0;
        }
        if (!grab((void**)&b->d_codes, 2 * codes_b)) return false;
        b->codes_cap = codes_b;
    }
    ensure_map_stream(b);
    return true;
}
// Apply the carried Pauli frames to the stored vectors (one pass), frames back to 1.
void materialize(qsim_batch* b) {
    if (!b->frame_pending) return;
    b->frame_pending = false;
    const uint64_t N = 1ull << b->n;
    const uint64_t items_per_traj = N / 2 > 0 ? N / 2 : 1;
    const uint64_t total = items_per_traj * (uint64_t)b->batch;
    TimedLaunch tl(&b->timer, "pauli_apply", 0.0, b->stream);
    hipLaunchKernelGGL(k_pauli_apply, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, b->stream, b->d, b->n,
                       b->d_xz, b->d_e, items_per_traj);
    QSIM_HIPCHK(hipGetLastError());
}
// Undo the relabeling in every trajectory (fused SWAP network over the batch, exact data
// movement) before anything reads or writes amplitudes by index; carried frames first.
void canonicalize(qsim_batch* b) {
    materialize(b);
    if (b->perm.empty()) return;
    const int n = b->n;
    std::vector<int> p = b->perm, inv(n);
    for (int q = 0; q < n; ++q) inv[p[q]] = q;
    std::vector<Op> swaps;
    for (int q = 0; q < n; ++q) {
        if (p[q] == q) continue;
        const int at = p[q], r = inv[q];
        qsim_gate g{};
        g.type = QSIM_GATE_SWAP;
        g.nqubits = 2;
        g.qubits[0] = q;
        g.qubits[1] = at;
        swaps.push_back(lower_gate(g, n));
        swaps.back().src = -1;
        p[r] = at;
        inv[at] = r;
        p[q] = q;
        inv[q] = q;
    }
    b->perm.clear();
    if (swaps.empty()) return;
    PlanCache::Entry& pe = b->plans.get(swaps, n, b->stream);
    b->ops.upload(pe.plan.ops.data(), pe.plan.ops.size() * sizeof(TileOp), b->stream);
    b->stages.upload(pe.plan.stages.data(), pe.plan.stages.size() * sizeof(Stage), b->stream);
    launch_fused(b->d, n, (uint64_t)b->batch, pe.plan, (const TileOp*)b->ops.ptr, (const Stage*)b->stages.ptr,
                 b->stream, &b->timer);
}
}  // namespace

extern "C" {

int qsim_batch_create(int n_qubits, int batch_size, qsim_batch** out) {
    return bguard([&] {
        if (!out) fail(QSIM_ERR_INVALID_ARGUMENT, "null out");
        *out = nullptr;
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > QSIM_MAX_QUBITS_SINGLE)
            fail(QSIM_ERR_INVALID_ARGUMENT, "Number of qubits must be between 1 and 30");
        if (batch_size < 1) fail(QSIM_ERR_INVALID_ARGUMENT, "batch_size must be positive");
        auto b = std::make_unique<qsim_batch>();
        b->n = n_qubits;
        b->batch = batch_size;
        QSIM_HIPCHK(hipGetDevice(&b->device));
        QSIM_HIPCHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
        b->timer.stream = b->stream;
        QSIM_HIPCHK(hipMalloc((void**)&b->d0, ((uint64_t)batch_size * sizeof(double2)) << n_qubits));
        b->d = b->d0;
        QSIM_HIPCHK(hipMalloc((void**)&b->d_xz, 2 * sizeof(uint64_t) * batch_size));
        QSIM_HIPCHK(hipMalloc((void**)&b->d_e, sizeof(int) * batch_size));
        b->seed = std::random_device{}();  // reference seeds from random_device (NoiseModel.cu:663)
        launch_init_basis(b->d, n_qubits, batch_size, 0, b->stream);
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
        *out = b.release();
    });
}

int qsim_batch_destroy(qsim_batch* b) {
    return bguard([&] { delete b; });
}

int qsim_batch_reset(qsim_batch* b) {
    return bguard([&] {
        need(b);
        launch_init_basis(b->d, b->n, b->batch, 0, b->stream);
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
        b->frame_pending = false;
        b->perm.clear();
        b->basis = true;
    });
}

int qsim_batch_set_seed(qsim_batch* b, uint64_t seed) {
    return bguard([&] {
        need(b);
        b->seed = seed;
        b->step = 0;
        b->ncounter = 0;
    });
}

int qsim_batch_set_trajectory_offset(qsim_batch* b, uint64_t first) {
    return bguard([&] {
        need(b);
        if (first > (1ull << 40)) fail(QSIM_ERR_INVALID_ARGUMENT, "trajectory offset out of range");
        b->traj0 = first;
    });
}

int qsim_batch_run(qsim_batch* b, const qsim_gate* gates, size_t count,
                   const qsim_noise_channel* channels, size_t n_channels, int flags) {
    return bguard([&] {
        need(b);
        if (!gates && count) fail(QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        std::vector<DevChannel> ch;
        for (size_t i = 0; i < n_channels; ++i) {
            const auto& c = channels[i];
            if (c.qubit < 0 || c.qubit >= b->n) fail(QSIM_ERR_OUT_OF_RANGE, "noise qubit out of range");
            if (c.type == 0 || c.type == 3 || c.type == 4 || c.type == 5)
                ch.push_back(DevChannel{c.type, c.qubit, c.probability});
        }
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], b->n);
        static const bool fused_env = [] {
            const char* e = std::getenv("QSIM_BATCH_FUSED");
            return e == nullptr || std::atoi(e) != 0;
        }();
        const bool fused_path = b->n >= 10 && fused_env && !(flags & QSIM_BATCH_PER_GATE) &&
                                !(flags & QSIM_BATCH_REFERENCE_NOISE);
        if (flags & QSIM_BATCH_REFERENCE_NOISE) canonicalize(b);  // per-pair draws name positions
        const bool frame_path = fused_path && b->n >= 10;  // (as the branch below)
        if (!frame_path) materialize(b);  // per-gate paths act on the plain vectors
        if (fused_path && b->basis && b->perm.empty() && count > 0) {
            // First fused run of |0..0> trajectories: relabel for the plan's tile layouts when
            // the whole batch is HBM-sized (as the JIT threshold, it counts every trajectory).
            int eff = b->n;
            while ((1ll << (eff - b->n)) < (long long)b->batch) ++eff;
            if (relabel_enabled(eff)) {
                auto lower_under = [&](const std::vector<int>& pi) {
                    std::vector<Op> lops;
                    for (size_t i = 0; i < count; ++i) {
                        qsim_gate g = gates[i];
                        if ((flags & QSIM_BATCH_REFERENCE_GATESET) &&
                            !(g.type <= QSIM_GATE_H || g.type == QSIM_GATE_CNOT))
                            continue;
                        for (int j = 0; j < g.nqubits && j < 3; ++j) g.qubits[j] = pi[g.qubits[j]];
                        lops.push_back(lower_gate(g, b->n));
                        lops.back().src = -1;
                    }
                    return lops;
                };
                const int kind = 1 + (flags & QSIM_BATCH_REFERENCE_GATESET ? 1 : 0);
                // (chosen under the tile-control rule the frame path plans with, and memoised
                // under it)
                std::unique_ptr<CtrlOutOff> ctrl_off;
                if (frame_path) ctrl_off = std::make_unique<CtrlOutOff>();
                if (!layout_memo_get(b->n, kind, gates, count * sizeof(qsim_gate), b->perm)) {
                    b->perm = choose_layout(b->n, lower_under, relabel_tries()).perm;
                    layout_memo_put(b->n, kind, gates, count * sizeof(qsim_gate), b->perm);
                }
            }
        }
        b->basis = false;
        for (DevChannel& c : ch)
            if (!b->perm.empty()) c.qubit = b->perm[c.qubit];
        if (ch.size() > b->ch_cap) {
            if (b->d_ch) {
                QSIM_HIPCHK(hipStreamSynchronize(b->stream));
                QSIM_HIPCHK(hipFree(b->d_ch));
            }
            QSIM_HIPCHK(hipMalloc((void**)&b->d_ch, ch.size() * sizeof(DevChannel)));
            b->ch_cap = ch.size();
        }
        if (!ch.empty())
            QSIM_HIPCHK(hipMemcpyAsync(b->d_ch, ch.data(), ch.size() * sizeof(DevChannel),
                                       hipMemcpyHostToDevice, b->stream));
        std::vector<Op> ops;
        for (size_t i = 0; i < count; ++i) {
            const qsim_gate g = map_gate(b, gates[i]);
            if (flags & QSIM_BATCH_REFERENCE_GATESET) {
                // src/NoiseModel.cu:742-763, 808-812, 821-825: only X/Y/Z/H and CNOT act.
                const bool ok = g.type <= QSIM_GATE_H || g.type == QSIM_GATE_CNOT;
                validate_gate(g, b->n);
                ops.push_back(ok ? lower_gate(g, b->n) : Op{});
                if (!ok) ops.back().kind = -1;
            } else {
                ops.push_back(lower_gate(g, b->n));
            }
        }
        const uint64_t N = 1ull << b->n;
        const uint64_t items_per_traj = N / 2 > 0 ? N / 2 : 1;
        if (flags & QSIM_BATCH_REFERENCE_NOISE) {
            // The reference's process (src/NoiseModel.cu:815-892): each gate, then for every
            // Depolarizing channel entry (the only type batched mode applies, F5) one pass over
            // all B x 2^(n-1) amplitude pairs; every pair draws its own uniform (counter hash of
            // (seed, pass, global pair index) in place of its curandState) and, below p, a second
            // one picks X / Y / Z at 1/3, 2/3 — applied to that pair only (F7).
            std::vector<NoiseChan> dep;
            for (size_t i = 0; i < n_channels; ++i)
                if (channels[i].type == 0) dep.push_back(NoiseChan{0, channels[i].qubit, channels[i].probability});
            if (pull_noise_supported(b->n, dep, false) && ensure_pull_buffers(b, dep.size())) {
                // Pulled: the noise after gate i is applied by gate i+1's pass (out of place),
                // the noise after the last gate by one identity pass; same draws, same states.
                // The map of noise step i (codes set i & 1) is built on map_stream while the pass
                // of step i - 1 runs; the pass of step i waits for it, the map of step i + 2
                // waits for that pass (QSIM_NOISE_MAP_OVERLAP=0: one stream, one set in turn).
                const char* oe = std::getenv("QSIM_NOISE_MAP_OVERLAP");
                const bool overlap = oe == nullptr || std::atoi(oe) != 0;
                const size_t G = ops.size();
                auto codes_of = [&](size_t i) { return (void*)(b->d_codes + (i & 1) * b->codes_cap); };
                const uint64_t c0 = b->ncounter;
                b->ncounter += (uint64_t)G * dep.size();  // (one pass counter per channel entry, as the push path)
                hipStream_t ms = overlap ? b->map_stream : b->stream;
                auto map = [&](size_t i) {
                    if (overlap && i >= 2) QSIM_HIPCHK(hipStreamWaitEvent(ms, b->ev_pull[i & 1], 0));
                    launch_noise_map(b->n, (uint64_t)b->batch, b->traj0, dep, b->seed, c0 + i * dep.size(), codes_of(i), ms,
                                     &b->timer);
                    if (overlap) QSIM_HIPCHK(hipEventRecord(b->ev_map[i & 1], ms));
                };
                if (overlap) {  // (the previous run's passes may still read both sets)
                    QSIM_HIPCHK(hipEventRecord(b->ev_start, b->stream));
                    QSIM_HIPCHK(hipStreamWaitEvent(ms, b->ev_start, 0));
                    for (size_t i = 0; i < std::min<size_t>(G, 2); ++i) map(i);
                }
                if (G && ops[0].kind >= 0) launch_op(b->d, b->n, (uint64_t)b->batch, ops[0], b->stream, &b->timer);
                for (size_t i = 0; i < G; ++i) {
                    if (overlap) {
                        QSIM_HIPCHK(hipStreamWaitEvent(b->stream, b->ev_map[i & 1], 0));
                    } else {
                        map(i);
                    }
                    const Op* op = i + 1 < G && ops[i + 1].kind >= 0 ? &ops[i + 1] : nullptr;
                    double2* dst = b->d == b->d0 ? b->d1 : b->d0;
                    launch_pull_gate(b->d, dst, b->n, (uint64_t)b->batch, dep, op, codes_of(i), b->stream,
                                     &b->timer);
                    b->d = dst;
                    if (overlap && i + 2 < G) {
                        QSIM_HIPCHK(hipEventRecord(b->ev_pull[i & 1], b->stream));
                        map(i + 2);
                    }
                }
                if (b->pinned) settle_in_d0(b);
                return;
            }
            bool all_tile = !ops.empty();
            for (const Op& op : ops) all_tile = all_tile && gate_noise_tile_supported(b->n, op.kind >= 0 ? &op : nullptr);
            if (all_tile) {
                // noise.hip: gate + in-tile channels in LDS per step, each step's flip lists built on
                // map_stream during the step before (when the device has room for them)
                const size_t lb = gate_noise_lists_bytes(b->n, (uint64_t)b->batch, dep);
                GnLists L{};
                const bool lists = lb && ensure_list_buffers(b, lb);
                if (lists) {
                    L.buf[0] = b->d_lists;
                    L.buf[1] = b->d_lists + b->lists_cap;
                    L.set_bytes = b->lists_cap;
                    L.ms = b->map_stream;
                    L.built[0] = b->ev_map[0];
                    L.built[1] = b->ev_map[1];
                    L.used[0] = b->ev_pull[0];
                    L.used[1] = b->ev_pull[1];
                    L.start = b->ev_start;
                }
                // two trajectory halves on two streams (QSIM_NOISE_SPLIT, read per run; default 2):
                // one half's tile pass overlaps the other's DRAM-random suffix push — W-BATCH config 4
                // 57.8 -> 54.1 ms per step (3 parts 62.5, 4 parts 58.6)
                const char* se = std::getenv("QSIM_NOISE_SPLIT");
                const int k = se ? std::max(1, std::min(4, std::atoi(se))) : 2;
                if (k > 1 && b->batch >= k && lists && split_tile_run(b, ops, dep, k, L)) return;
                launch_gate_noise_run(b->d, b->n, (uint64_t)b->batch, b->traj0, ops, dep, b->seed, b->ncounter,
                                      b->stream, &b->timer, lists ? &L : nullptr);
                return;
            }
            for (const Op& op : ops) {
                const Op* o = op.kind >= 0 ? &op : nullptr;
                if (gate_noise_tile_supported(b->n, o)) {  // (noise.hip: gate + in-tile channels in LDS)
                    launch_gate_noise_step(b->d, b->n, (uint64_t)b->batch, b->traj0, o, dep, b->seed, b->ncounter,
                                           b->stream, &b->timer);
                    continue;
                }
                if (o) launch_op(b->d, b->n, (uint64_t)b->batch, op, b->stream, &b->timer);
                launch_noise_after_gate(b->d, b->n, dep, b->seed, b->ncounter, b->stream, &b->timer,
                                        (uint64_t)b->batch, b->traj0);
            }
            return;
        }
        if (b->n >= 10 && fused_env && !(flags & QSIM_BATCH_PER_GATE)) {
            // Fused tile passes over all trajectories (a tile never straddles two).  Noise is
            // carried as per-trajectory Pauli frames: no noise kernel per gate, one frame build
            // before and one materialising Pauli pass after the circuit.
            // a carried frame must be propagated (Cliffords) and conjugated (the rest) like noise
            const bool noisy = (!ch.empty() || b->frame_pending) && count > 0;
            std::vector<Op> fops;
            std::vector<StepClifford> cl(count, StepClifford{CL_NONE, 0, -1, 0});
            for (size_t i = 0; i < ops.size(); ++i) {
                if (ops[i].kind < 0) continue;  // ignored by the reference gate set
                const qsim_gate g = map_gate(b, gates[i]);
                static const int code_of[QSIM_GATE_COUNT] = {
                    CL_X, CL_Y, CL_Z, CL_H, CL_S, CL_NONE /*T*/, CL_SDG, CL_NONE /*Tdag*/,
                    CL_NONE, CL_NONE, CL_NONE /*Rx Ry Rz*/, CL_CNOT, CL_CZ, CL_NONE, CL_NONE /*CRY CRZ*/,
                    CL_SWAP, CL_NONE /*Toffoli*/};
                cl[i] = StepClifford{code_of[g.type], g.qubits[0], g.nqubits > 1 ? g.qubits[1] : -1, 0};
                fops.push_back(ops[i]);
                // circuit step = frame index for ops conjugated by the frame; Clifford gates move
                // the frame instead and run unconjugated (src -1)
                fops.back().src = (noisy && cl[i].code == CL_NONE) ? (int)i : -1;
            }
            if (noisy) {
                const size_t need_frames = 2 * count * (size_t)b->batch;
                if (need_frames > b->frames_cap) {
                    QSIM_HIPCHK(hipStreamSynchronize(b->stream));
                    if (b->d_frames) QSIM_HIPCHK(hipFree(b->d_frames));
                    if (b->d_fe) QSIM_HIPCHK(hipFree(b->d_fe));
                    b->d_frames = nullptr;
                    b->d_fe = nullptr;
                    QSIM_HIPCHK(hipMalloc((void**)&b->d_frames, need_frames * sizeof(uint64_t)));
                    QSIM_HIPCHK(hipMalloc((void**)&b->d_fe, need_frames / 2 * sizeof(int)));
                    b->frames_cap = need_frames;
                }
                TimedLaunch tl(&b->timer, "pauli_frames", 0.0, b->stream);
                const uint64_t draws = (uint64_t)count * b->batch;
                hipLaunchKernelGGL(k_draw_steps, dim3((unsigned)((draws + 255) / 256)), dim3(256), 0,
                                   b->stream, b->d_ch, (int)ch.size(), b->seed, b->step, (int)count,
                                   b->batch, b->traj0, b->d_frames, b->d_fe);
                b->cliff.upload(cl.data(), cl.size() * sizeof(StepClifford), b->stream);
                hipLaunchKernelGGL(k_frame_build, dim3((b->batch + 63) / 64), dim3(64), 0, b->stream,
                                   (int)count, b->batch, b->d_frames, b->d_fe,
                                   (const StepClifford*)b->cliff.ptr, b->d_xz, b->d_e, b->frame_pending ? 1 : 0);
                QSIM_HIPCHK(hipGetLastError());
            }
            if (!fops.empty()) {
                const CtrlOutOff ctrl_off;  // (Pauli-frame passes: every control is a tile bit)
                PlanCache::Entry& pe = b->plans.get(fops, b->n, b->stream);
                const Plan& plan = pe.plan;
                // circuit-specialised kernels for the passes no frame conjugation reaches (all of
                // them for a Clifford circuit); the JIT threshold counts the whole batch
                int eff = b->n;
                while ((1ll << (eff - b->n)) < (long long)b->batch) ++eff;
                const JitModule* jm = jit_for(pe.jit, plan, eff);
                b->ops.upload(plan.ops.data(), plan.ops.size() * sizeof(TileOp), b->stream);
                b->stages.upload(plan.stages.data(), plan.stages.size() * sizeof(Stage), b->stream);
                launch_fused(b->d, b->n, (uint64_t)b->batch, plan, (const TileOp*)b->ops.ptr,
                             (const Stage*)b->stages.ptr, b->stream, &b->timer, jm,
                             noisy ? b->d_frames : nullptr);
                b->last_passes = (int)plan.passes.size();
                b->last_jit_passes = 0;
                if (jm)
                    for (hipFunction_t f : jm->fn) b->last_jit_passes += f != nullptr;
            }
            if (noisy) {
                if (!ch.empty()) b->step += count;
                b->frame_pending = true;  // materialised by the next reader (or composed by the next run)
            }
            return;
        }
        for (const Op& op : ops) {
            if (op.kind >= 0) launch_op(b->d, b->n, (uint64_t)b->batch, op, b->stream, &b->timer);
            if (!ch.empty()) {
                {
                    TimedLaunch tl(&b->timer, "pauli_draw", 0.0, b->stream);
                    hipLaunchKernelGGL(k_pauli_draw, dim3((b->batch + 255) / 256), dim3(256), 0,
                                       b->stream, b->d_ch, (int)ch.size(), b->seed, b->step,
                                       b->batch, b->traj0, b->d_xz, b->d_e);
                    QSIM_HIPCHK(hipGetLastError());
                }
                ++b->step;
                const uint64_t total = items_per_traj * (uint64_t)b->batch;
                TimedLaunch tl(&b->timer, "pauli_apply", 0.0, b->stream);
                hipLaunchKernelGGL(k_pauli_apply, dim3((unsigned)((total + 255) / 256)), dim3(256),
                                   0, b->stream, b->d, b->n, b->d_xz, b->d_e, items_per_traj);
                QSIM_HIPCHK(hipGetLastError());
            }
        }
    });
}

int qsim_batch_avg_probabilities(qsim_batch* b, double* dst) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        const uint64_t N = 1ull << b->n;
        double* d_p = (double*)b->scratch.get(N * sizeof(double), b->stream);
        launch_avg_probabilities(b->d, b->n, (uint64_t)b->batch, d_p, b->stream);
        QSIM_HIPCHK(hipMemcpyAsync(dst, d_p, N * sizeof(double), hipMemcpyDeviceToHost, b->stream));
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
    });
}

int qsim_batch_traj_probabilities(qsim_batch* b, int traj, double* dst) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        if (traj < 0 || traj >= b->batch) fail(QSIM_ERR_OUT_OF_RANGE, "Invalid trajectory index");
        const uint64_t N = 1ull << b->n;
        double* d_p = (double*)b->scratch.get(N * sizeof(double), b->stream);
        launch_probabilities(b->d + (uint64_t)traj * N, N, d_p, b->stream);
        QSIM_HIPCHK(hipMemcpyAsync(dst, d_p, N * sizeof(double), hipMemcpyDeviceToHost, b->stream));
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
    });
}

int qsim_batch_sample(qsim_batch* b, const double* uniforms, int shots, int64_t* out) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        if (shots < 0) fail(QSIM_ERR_INVALID_ARGUMENT, "n_shots must be non-negative");
        if (shots > 0 && (!uniforms || !out)) fail(QSIM_ERR_INVALID_ARGUMENT, "null buffer");
        sample_indices(b->d, b->n, (uint64_t)b->batch, uniforms, shots, out, b->stream, b->scratch);
    });
}

int qsim_batch_histogram(qsim_batch* b, const double* uniforms, int shots, int64_t* hist) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        if (shots < 0) fail(QSIM_ERR_INVALID_ARGUMENT, "n_shots must be non-negative");
        if (!hist || (shots > 0 && !uniforms)) fail(QSIM_ERR_INVALID_ARGUMENT, "null buffer");
        const uint64_t N = 1ull << b->n, nshots = (uint64_t)shots * (uint64_t)b->batch;
        std::vector<int64_t> idx(nshots);
        sample_indices(b->d, b->n, (uint64_t)b->batch, uniforms, shots, idx.data(), b->stream,
                       b->scratch);
        // counts on the device: scratch2 = [hist N x u64][indices nshots x i64]
        char* base = (char*)b->scratch2.get(N * 8 + std::max<uint64_t>(1, nshots) * 8, b->stream);
        unsigned long long* d_h = (unsigned long long*)base;
        int64_t* d_idx = (int64_t*)(base + N * 8);
        QSIM_HIPCHK(hipMemsetAsync(d_h, 0, N * sizeof(unsigned long long), b->stream));
        if (nshots) {
            QSIM_HIPCHK(hipMemcpyAsync(d_idx, idx.data(), nshots * sizeof(int64_t),
                                       hipMemcpyHostToDevice, b->stream));
            launch_histogram(d_idx, nshots, N, d_h, b->stream);
        }
        QSIM_HIPCHK(hipMemcpyAsync(hist, d_h, N * sizeof(int64_t), hipMemcpyDeviceToHost, b->stream));
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
    });
}

int qsim_batch_traj_state(qsim_batch* b, int traj, double* dst) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        if (traj < 0 || traj >= b->batch) fail(QSIM_ERR_OUT_OF_RANGE, "Invalid trajectory index");
        const uint64_t N = 1ull << b->n;
        QSIM_HIPCHK(hipMemcpyAsync(dst, b->d + (uint64_t)traj * N, N * sizeof(double2),
                                   hipMemcpyDeviceToHost, b->stream));
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
    });
}

int qsim_batch_device_ptr(qsim_batch* b, void** dptr) {
    return bguard([&] {
        need(b);
        canonicalize(b);
        b->basis = false;  // the caller may write through the pointer
        settle_in_d0(b);   // (pulled runs copy their result back to this buffer from now on)
        b->pinned = true;
        *dptr = b->d;
    });
}

int qsim_batch_last_run(qsim_batch* b, int* passes, int* jit_passes) {
    return bguard([&] {
        need(b);
        if (passes) *passes = b->last_passes;
        if (jit_passes) *jit_passes = b->last_jit_passes;
    });
}

int qsim_batch_sync(qsim_batch* b) {
    return bguard([&] {
        need(b);
        materialize(b);  // the carried frames are queued work too
        QSIM_HIPCHK(hipStreamSynchronize(b->stream));
    });
}

int qsim_batch_profile(qsim_batch* b, int enable) {
    return bguard([&] {
        need(b);
        b->timer.enabled = enable != 0;
    });
}

int qsim_batch_profile_count(qsim_batch* b, int* n) {
    return bguard([&] {
        need(b);
        b->timer.resolve();
        *n = (int)b->timer.stats.size();
    });
}

int qsim_batch_profile_get(qsim_batch* b, int i, char* name, size_t name_len, double* total_ms,
                           int64_t* launches, double* alg_bytes) {
    return bguard([&] {
        need(b);
        b->timer.resolve();
        if (i < 0 || i >= (int)b->timer.stats.size()) fail(QSIM_ERR_OUT_OF_RANGE, "bad index");
        const auto& st = b->timer.stats[i];
        if (name && name_len) {
            std::strncpy(name, st.name.c_str(), name_len - 1);
            name[name_len - 1] = 0;
        }
        if (total_ms) *total_ms = st.ms;
        if (launches) *launches = st.launches;
        if (alg_bytes) *alg_bytes = st.bytes;
    });
}

}  // extern "C"
