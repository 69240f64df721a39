// capi.hip — extern "C" implementation of include/qsim_hip.h for single-GPU states.
//
// Each qsim_state owns its device buffer (2^n x 16 B) and a non-blocking HIP stream; gate
// application is asynchronous on that stream (as the reference's launches are on the legacy
// stream, src/Simulator.cu:95-97) and every readout synchronizes it (src/StateVector.cu:204-233).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "qsim_hip.h"

using namespace qsim_hip;

// ---------------------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------------------
static thread_local std::string g_last_error;
namespace qsim_hip {
void set_last_error(const char* msg) { g_last_error = msg; }
}  // namespace qsim_hip

template <typename F>
static int guarded(F&& f) {
    try {
        f();
        return QSIM_OK;
    } catch (const Error& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "host allocation failed";
        return QSIM_ERR_RUNTIME;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return QSIM_ERR_RUNTIME;
    }
}
#define QSIM_REQUIRE(cond, code, msg) \
    do {                              \
        if (!(cond)) fail(code, msg); \
    } while (0)

// ---------------------------------------------------------------------------------------
// Timer
// ---------------------------------------------------------------------------------------
namespace qsim_hip {
int Timer::slot_of(const char* name) {
    for (size_t i = 0; i < stats.size(); ++i)
        if (stats[i].name == name) return (int)i;
    stats.push_back(Stat{name});
    return (int)stats.size() - 1;
}
static hipEvent_t take_event(std::vector<hipEvent_t>& pool) {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    QSIM_HIPCHK(hipEventCreate(&e));
    return e;
}
void Timer::begin(const char* name, double, hipEvent_t* a_out, int* slot_out) {
    *slot_out = slot_of(name);
    *a_out = take_event(pool);
    QSIM_HIPCHK(hipEventRecord(*a_out, stream));
}
void Timer::end(int slot, hipEvent_t a, double bytes) {
    hipEvent_t b = take_event(pool);
    QSIM_HIPCHK(hipEventRecord(b, stream));
    pending.push_back(Pending{slot, a, b, bytes});
}
void Timer::begin_ext(const char* name, hipEvent_t* a_out, hipEvent_t* b_out, int* slot_out) {
    *slot_out = slot_of(name);
    *a_out = take_event(pool);
    *b_out = take_event(pool);
}
void Timer::finish(int slot, hipEvent_t a, hipEvent_t b, double bytes) {
    pending.push_back(Pending{slot, a, b, bytes});
}
void Timer::resolve() {
    for (auto& p : pending) {
        QSIM_HIPCHK(hipEventSynchronize(p.b));
        float ms = 0.f;
        QSIM_HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        stats[p.slot].ms += ms;
        stats[p.slot].launches += 1;
        stats[p.slot].bytes += p.bytes;
        pool.push_back(p.a);
        pool.push_back(p.b);
    }
    pending.clear();
}
void Timer::reset() {
    resolve();
    stats.clear();
}
Timer::~Timer() {
    for (auto& p : pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
}
void DevBuf::upload(const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return;
    if (shadow.size() == bytes && std::memcmp(shadow.data(), src, bytes) == 0) return;
    if (copied) QSIM_HIPCHK(hipEventSynchronize(copied));  // previous copy done reading shadow
    if (bytes > cap) {
        if (ptr) {
            QSIM_HIPCHK(hipStreamSynchronize(s));
            QSIM_HIPCHK(hipFree(ptr));
            ptr = nullptr;
        }
        cap = std::max<size_t>(bytes, 16384);
        QSIM_HIPCHK(hipMalloc(&ptr, cap));
    }
    shadow.assign((const unsigned char*)src, (const unsigned char*)src + bytes);
    QSIM_HIPCHK(hipMemcpyAsync(ptr, shadow.data(), bytes, hipMemcpyHostToDevice, s));
    if (!copied) QSIM_HIPCHK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
    QSIM_HIPCHK(hipEventRecord(copied, s));
}
void* Scratch::get(size_t bytes, hipStream_t s) {
    bytes = std::max<size_t>(bytes, 256);
    if (bytes > cap) {
        if (ptr) {
            QSIM_HIPCHK(hipStreamSynchronize(s));
            QSIM_HIPCHK(hipFree(ptr));
            ptr = nullptr;
            cap = 0;
        }
        QSIM_HIPCHK(hipMalloc(&ptr, bytes));
        cap = bytes;
    }
    return ptr;
}
Scratch::~Scratch() {
    if (ptr) (void)hipFree(ptr);
}
DevBuf::~DevBuf() {
    if (copied) {
        (void)hipEventSynchronize(copied);
        (void)hipEventDestroy(copied);
    }
    if (ptr) (void)hipFree(ptr);
}
TimedLaunch::TimedLaunch(Timer* t, const char* name, double by, hipStream_t s, bool e)
    : tm(t), bytes(by), ext(e), stream(s) {
    if (tm && tm->enabled) {
        tm->stream = s;
        if (ext) tm->begin_ext(name, &a, &b, &slot);
        else tm->begin(name, by, &a, &slot);
    } else {
        tm = nullptr;
    }
}
TimedLaunch::~TimedLaunch() {
    if (tm) {
        try {
            tm->stream = stream;  // a nested launch on another stream may have moved it
            if (ext) tm->finish(slot, a, b, bytes);
            else tm->end(slot, a, bytes);
        } catch (...) {
        }
    }
}
}  // namespace qsim_hip

// ---------------------------------------------------------------------------------------
// state object
// ---------------------------------------------------------------------------------------
struct qsim_state {
    int n = 0;
    int device = 0;
    double2* d = nullptr;
    void* base = nullptr;  // the allocation d lies in
    hipStream_t stream = nullptr;
    double* d_partials = nullptr;
    double* d_result = nullptr;
    DevBuf ops, stages;  // fused-plan descriptors, re-uploaded only when the plan changes
    PlanCache plans;
    Timer timer;
    int last_passes = 0, last_jit_passes = 0;  // of the last fused run (qsim_state_last_run)
    Scratch scratch;
    // Layout-aware relabeling (relabel.hip): logical qubit q lives at physical position perm[q]
    // (empty: identity).  basis: the amplitudes are the computational basis state basis_idx
    // (physical index) — set by create / init, cleared by anything else that writes them.
    std::vector<int> perm;
    bool basis = true;
    uint64_t basis_idx = 0;
    // tile height chosen for this state by the first-run calibration (-1: the size rule), and
    // whether its layout was chosen by timing candidates on the device
    int tile_h = -1;
    bool calibrated = false;
    bool relayout = false;  // the first-run choice is a relayout plan (relayout.hip)
    // Relayout passes write out of place: the state alternates between two buffers (d is the
    // current one; alt_base is allocated on the first relayout run).  pinned: a raw device
    // pointer was handed out, so the amplitudes are copied back to it after such a run.
    void* alt_base = nullptr;
    double2* alt = nullptr;
    double2* base_d = nullptr;  // the amplitudes' address inside `base` (d == base_d or alt_base)
    bool pinned = false;
    // pulled noise (NoisySimulator flip channels, noise.hip): two sets of per-step code words
    // (steps alternate), so the next step's words are built on noise_stream during this pass
    unsigned char* noise_codes = nullptr;
    size_t noise_codes_cap = 0;  // bytes of ONE set
    // in-tile noise (noise.hip launch_gate_noise_run): two sets of per-step flip lists, built on
    // noise_stream one step ahead
    char* noise_lists = nullptr;
    size_t noise_lists_cap = 0;  // bytes of ONE set
    hipStream_t noise_stream = nullptr;
    hipEvent_t nev_map[2] = {}, nev_pull[2] = {}, nev_start = nullptr;
    ~qsim_state() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (noise_stream) (void)hipStreamSynchronize(noise_stream);
        for (hipEvent_t e : {nev_map[0], nev_map[1], nev_pull[0], nev_pull[1], nev_start})
            if (e) (void)hipEventDestroy(e);
        if (noise_stream) (void)hipStreamDestroy(noise_stream);
        if (base) (void)hipFree(base);
        if (alt_base) (void)hipFree(alt_base);
        if (noise_codes) (void)hipFree(noise_codes);
        if (noise_lists) (void)hipFree(noise_lists);
        if (d_partials) (void)hipFree(d_partials);
        if (d_result) (void)hipFree(d_result);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) QSIM_HIPCHK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

static void check_state(const qsim_state* s) {
    if (!s) fail(QSIM_ERR_INVALID_ARGUMENT, "null state handle");
}

// The second 2^n buffer relayout passes write into (they run out of place).  Allocated only
// when the device has room for it beside a margin; a refused or failed allocation is cleared and
// reported as false, so the caller keeps the in-place fixed-layout plan (the reference's
// StateVector owns exactly one buffer, and coexisting states must not fail where it would not).
static constexpr size_t kAltMarginBytes = 256ull << 20;
static bool ensure_alt(qsim_state* s) {
    if (s->alt) return true;
    static const bool off = [] {  // QSIM_RELAYOUT_NO_ALT=1: behave as if it never fits (tests)
        const char* e = std::getenv("QSIM_RELAYOUT_NO_ALT");
        return e != nullptr && std::atoi(e) != 0;
    }();
    if (off) return false;
    const size_t bytes = sizeof(double2) << s->n;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (free_b < bytes + kAltMarginBytes) return false;
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();  // (clear the sticky error: the state itself is intact)
        return false;
    }
    s->alt_base = p;
    s->alt = reinterpret_cast<double2*>(p);
    return true;
}
// Free the buffer the amplitudes are not in (the state goes back to one 2^n buffer).
static void release_alt(qsim_state* s) {
    if (!s->alt_base) return;
    QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    if (s->d != s->base_d) {  // the amplitudes live in alt_base: it becomes the state's buffer
        (void)hipFree(s->base);
        s->base = s->alt_base;
        s->base_d = s->d;
    } else {
        (void)hipFree(s->alt_base);
    }
    s->alt_base = nullptr;
    s->alt = nullptr;
}

// The noise side stream and its events (the pulled path's code-word maps, the in-tile path's lists).
static void ensure_noise_stream(qsim_state* s) {
    if (s->noise_stream) return;
    QSIM_HIPCHK(hipStreamCreateWithFlags(&s->noise_stream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&s->nev_map[0], &s->nev_map[1], &s->nev_pull[0], &s->nev_pull[1], &s->nev_start})
        QSIM_HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
}
// Buffers of the pulled noise path: the second state buffer, two sets of per-step code words.
static bool ensure_noise_buffers(qsim_state* s, size_t nch) {
    const size_t codes_b = pull_noise_codes_bytes(s->n, 1, nch);
    // Allocate only when the device keeps room for another state of this size beside the new
    // buffers — the rule trim_noise_buffers keeps them by — so a device with between one and two
    // states of room runs the push kernels instead of allocating and freeing a second state on
    // every run.
    const size_t need = (s->alt ? 0 : (sizeof(double2) << s->n)) + (codes_b > s->noise_codes_cap ? 2 * codes_b : 0);
    if (need) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (free_b < need + (sizeof(double2) << s->n) + kAltMarginBytes) return false;
    }
    if (!ensure_alt(s)) return false;
    auto grab = [&](unsigned char** p, size_t bytes) {
        if (hipMalloc((void**)p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            return false;
        }
        return true;
    };
    if (codes_b > s->noise_codes_cap) {
        if (s->noise_codes) {
            QSIM_HIPCHK(hipStreamSynchronize(s->stream));
            (void)hipFree(s->noise_codes);
            s->noise_codes = nullptr;
            s->noise_codes_cap = 0;
        }
        if (!grab(&s->noise_codes, 2 * codes_b)) return false;
        s->noise_codes_cap = codes_b;
    }
    ensure_noise_stream(s);
    return true;
}

// Two sets of the in-tile path's flip lists, when they fit beside a margin (false: the tile
// kernels walk the draws themselves).
static bool ensure_noise_lists(qsim_state* s, size_t bytes) {
    if (bytes > s->noise_lists_cap) {
        if (s->noise_lists) {
            QSIM_HIPCHK(hipStreamSynchronize(s->stream));
            if (s->noise_stream) QSIM_HIPCHK(hipStreamSynchronize(s->noise_stream));
            (void)hipFree(s->noise_lists);
            s->noise_lists = nullptr;
            s->noise_lists_cap = 0;
        }
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (free_b < 2 * bytes + kAltMarginBytes) return false;
        if (hipMalloc((void**)&s->noise_lists, 2 * bytes) != hipSuccess) {
            (void)hipGetLastError();
            s->noise_lists = nullptr;
            return false;
        }
        s->noise_lists_cap = bytes;
    }
    ensure_noise_stream(s);
    return true;
}

// After a pulled noisy run: free the second buffer (unless a relayout plan owns it) and the
// code words when the device no longer has room for another 2^n buffer beside a margin.
static void trim_noise_buffers(qsim_state* s) {
    static const int keep = [] {  // QSIM_NOISE_KEEP_BUFFERS: 1 always keep, 0 always free (tests)
        const char* e = std::getenv("QSIM_NOISE_KEEP_BUFFERS");
        return e ? std::atoi(e) : -1;
    }();
    if (keep == 1) return;
    if (keep != 0) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            free_b = 0;
        }
        if (free_b >= (sizeof(double2) << s->n) + kAltMarginBytes) return;
    }
    QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    if (s->noise_stream) QSIM_HIPCHK(hipStreamSynchronize(s->noise_stream));
    if (s->noise_codes) (void)hipFree(s->noise_codes);
    s->noise_codes = nullptr;
    s->noise_codes_cap = 0;
    if (s->noise_lists) (void)hipFree(s->noise_lists);
    s->noise_lists = nullptr;
    s->noise_lists_cap = 0;
    if (!s->relayout) release_alt(s);
}

// One fused plan on the state: relayout passes alternate between the state's two buffers.
static void launch_plan(qsim_state* s, const Plan& plan, Timer* tm, const JitModule* jm) {
    FusedRange range;
    bool relayout = false;
    for (const FusedPass& p : plan.passes) relayout = relayout || p.relayout;
    if (relayout) {
        // (choose_first_layout only takes relayout plans once the buffer exists)
        if (!ensure_alt(s)) fail(QSIM_ERR_DEVICE, "out of device memory for the relayout buffer");
        range.alt = s->alt;
    }
    double2* r = launch_fused(s->d, s->n, 1, plan, (const TileOp*)s->ops.ptr, (const Stage*)s->stages.ptr,
                              s->stream, tm, jm, nullptr, range);
    if (r == s->d) return;
    if (s->pinned) {  // keep the amplitudes where the handed-out pointer points
        QSIM_HIPCHK(hipMemcpyAsync(s->d, r, sizeof(double2) << s->n, hipMemcpyDeviceToDevice, s->stream));
        return;
    }
    s->alt = s->d;
    s->d = r;
}

// jit = false: the pass interpreter only (a one-off network — the layout restore — would wait
// longer for its compile than its passes take).
static void run_fused(qsim_state* s, const std::vector<Op>& ops, bool jit = true) {
    PlanCache::Entry& pe = s->plans.get(ops, s->n, s->stream);
    const Plan& plan = pe.plan;
    const JitModule* jm = jit ? jit_for(pe.jit, plan, s->n) : nullptr;
    s->ops.upload(plan.ops.data(), plan.ops.size() * sizeof(TileOp), s->stream);
    s->stages.upload(plan.stages.data(), plan.stages.size() * sizeof(Stage), s->stream);
    launch_plan(s, plan, &s->timer, jm);
    s->last_passes = (int)plan.passes.size();
    s->last_jit_passes = 0;
    if (jm)
        for (hipFunction_t f : jm->fn) s->last_jit_passes += f != nullptr;
}

// Undo the relabeling: a fused network of physical SWAPs that brings logical qubit q back to
// position q (exact data movement), then the identity map.  Every entry that reads or writes
// amplitudes by index calls this first.
static void canonicalize(qsim_state* s) {
    if (s->perm.empty()) return;
    const int n = s->n;
    // One gate-free relayout pass (relayout.hip) from 16 qubits: every amplitude stored at its
    // identity-layout position in a single HBM round trip (QSIM_RESTORE_ONE_PASS=0: the SWAP
    // network below, a few passes).
    static const bool one_pass = [] {
        const char* e = std::getenv("QSIM_RESTORE_ONE_PASS");
        return e == nullptr || std::atoi(e) != 0;
    }();
    // (it writes out of place: without room for the second buffer, the in-place SWAP network)
    if (one_pass && n >= 16 && n - 12 <= 32 && ensure_alt(s)) {
        const Plan plan = plan_permutation_pass(n, s->perm);
        s->stages.upload(plan.stages.data(), plan.stages.size() * sizeof(Stage), s->stream);
        launch_plan(s, plan, &s->timer, nullptr);
        s->perm.clear();  // (last_passes keeps describing the last circuit run)
        if (!s->relayout) release_alt(s);  // (only relayout plans keep the second buffer)
        return;
    }
    std::vector<int> p = s->perm, inv(n);
    for (int q = 0; q < n; ++q) inv[p[q]] = q;
    std::vector<Op> swaps;
    for (int q = 0; q < n; ++q) {
        if (p[q] == q) continue;
        const int b = p[q], r = inv[q];  // logical q sits at b, logical r at position q
        qsim_gate g{};
        g.type = QSIM_GATE_SWAP;
        g.nqubits = 2;
        g.qubits[0] = q;
        g.qubits[1] = b;
        swaps.push_back(lower_gate(g, n));
        swaps.back().src = (int)swaps.size() - 1;
        p[r] = b;
        inv[b] = r;
        p[q] = q;
        inv[q] = q;
    }
    s->perm.clear();
    if (!swaps.empty()) run_fused(s, swaps, false);
}
// Before an entry that overwrites every amplitude: the labels are dropped, not restored.
static void drop_layout(qsim_state* s) {
    if (s->relayout) {  // (a relayout plan's second buffer: as canonicalize would leave it)
        canonicalize(s);
    }
    s->perm.clear();
    s->basis = false;
}
// Before an entry that reads amplitudes by index (touch: and writes them).
static void prep(qsim_state* s, bool touch) {
    canonicalize(s);
    if (touch) s->basis = false;
}
// One timed candidate of the first-run layout choice: a tile height and the labels chosen under
// it, with the circuit lowered under those labels and its plan at that height.
struct LayoutCandidate {
    int h = kTileHDefault;
    std::vector<int> perm;  // empty: identity
    std::vector<Op> ops;
    Plan plan;
    bool relayout = false;  // a relayout plan (relayout.hip)
};
// Time every candidate with its own circuit-specialised kernels on this device (each candidate's
// whole plan under its own tile height, the faster of two runs, the basis state restored after
// each) and return the fastest: the cost model ranks layouts from probes of other boxes, real
// pass times differ by a few per cent between devices, and whether 13-qubit tiles (fewer passes,
// slower streaming) beat 12-qubit ones depends on the circuit.  The plans stay cached
// (compiled).
static size_t calibrate_candidates(qsim_state* s, std::vector<LayoutCandidate>& cands) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    QSIM_HIPCHK(hipEventCreate(&e0));
    QSIM_HIPCHK(hipEventCreate(&e1));
    size_t best = 0;
    float best_ms = 3.0e38f;
    try {
        for (size_t k = 0; k < cands.size(); ++k) {
            LayoutCandidate& c = cands[k];
            const TileHeightScope scope(c.h, tile_rb_for(s->n, c.h));
            s->plans.put(c.ops, s->n, c.plan, s->stream);
            PlanCache::Entry& pe = s->plans.get(c.ops, s->n, s->stream);
            const JitModule* jm = jit_for(pe.jit, pe.plan, s->n);
            s->ops.upload(pe.plan.ops.data(), pe.plan.ops.size() * sizeof(TileOp), s->stream);
            s->stages.upload(pe.plan.stages.data(), pe.plan.stages.size() * sizeof(Stage), s->stream);
            float ms = 3.0e38f;
            const int reps = s->n < 26 ? 5 : 2;  // (short runs: more repetitions against noise)
            for (int rep = 0; rep < reps; ++rep) {
                QSIM_HIPCHK(hipEventRecord(e0, s->stream));
                launch_plan(s, pe.plan, nullptr, jm);
                QSIM_HIPCHK(hipEventRecord(e1, s->stream));
                QSIM_HIPCHK(hipEventSynchronize(e1));
                float t = 0.0f;
                QSIM_HIPCHK(hipEventElapsedTime(&t, e0, e1));
                ms = std::min(ms, t);
            }
            launch_init_basis(s->d, s->n, 1, s->basis_idx, s->stream);  // the state as it was
            static const bool dbg = std::getenv("QSIM_RELABEL_DEBUG") != nullptr;
            if (dbg)
                std::fprintf(stderr, "[calibrate] candidate %zu (h=%d, %zu passes): %.3f ms per run\n", k, c.h,
                             pe.plan.passes.size(), ms);
            if (ms < best_ms) {
                best = k;
                best_ms = ms;
            }
        }
    } catch (...) {
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        // a candidate may have run partway: put the basis state back (best effort) or, if even
        // that fails, stop treating the amplitudes as that basis state (no relabeling later)
        try {
            launch_init_basis(s->d, s->n, 1, s->basis_idx, s->stream);
            QSIM_HIPCHK(hipStreamSynchronize(s->stream));
        } catch (...) {
            s->basis = false;
        }
        throw;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    return best;
}

// The labels (s->perm) and, with cross-height calibration, the tile height (s->tile_h) for the
// first fused run of a basis state.  Candidates: the layout model's choice and its next
// alternatives at the state's default height; with cross-height calibration also at the other
// height (13-qubit tiles with the 13-qubit cost factor 1.25, which steers the labels toward
// mixed plans, and with factor 1) — every candidate timed on the device, the fastest kept.
static void choose_first_layout(qsim_state* s, const qsim_gate* gates, size_t count) {
    const int n = s->n;
    const size_t bytes = count * sizeof(qsim_gate);
    auto lower_under = [&](const std::vector<int>& pi) {
        std::vector<Op> ops;
        ops.reserve(count);
        for (size_t i = 0; i < count; ++i) {
            qsim_gate m = gates[i];
            for (int j = 0; j < m.nqubits && j < 3; ++j) m.qubits[j] = pi[m.qubits[j]];
            ops.push_back(lower_gate(m, n));
            ops.back().src = (int)i;
        }
        return ops;
    };
    static const size_t alts = [] {  // QSIM_RELABEL_CALIBRATE_CANDIDATES (default 3) per height
        const char* e = std::getenv("QSIM_RELABEL_CALIBRATE_CANDIDATES");
        return (size_t)std::max(1, e ? std::atoi(e) : 3) - 1;
    }();
    const bool heights = calibrate_heights(n) && s->tile_h < 0;
    const int th = s->tile_h >= 0 ? s->tile_h : tile_height_for(n);
    auto memo_put = [&](const std::vector<int>& perm) {
        const TileHeightScope scope(th);  // (a single-height decision is keyed by its height)
        layout_memo_put(n, 0, gates, bytes, perm, heights ? s->tile_h : -1);
    };
    // Relayout plans permute qubit labels, so they follow the relabeling mode (not its size
    // threshold), and they need the second buffer: without room for it, fixed layouts only.
    const bool relayout = relayout_enabled(n) && relabel_mode_on() && !tile_height_is_set() && ensure_alt(s);
    struct AltRelease {  // a first run that does not end on a relayout plan keeps one buffer
        qsim_state* s;
        ~AltRelease() {
            if (!s->relayout) try {
                    release_alt(s);
                } catch (...) {
                }
        }
    } alt_release{s};
    const bool timing = relabel_calibrate(n);
    {
        // a relayout choice made before for this circuit (by timing, or by pass count when
        // candidates are not timed: memoised apart)
        std::vector<int> memo;
        int mh = -1;
        if (relayout && layout_memo_get(n, 2, gates, bytes, memo, timing ? &mh : nullptr) &&
            !(memo.empty() && relayout_forced())) {
            if (memo.empty()) return;  // (decided: no relayout plan, and no relabeling below)
            std::vector<RelayoutChoice> vs;
            plan_relayout_variants(n, lower_under, SIZE_MAX, vs);
            for (RelayoutChoice& rc : vs) {
                if (rc.perm != memo) continue;
                const TileHeightScope scope(6, tile_rb_for(n, 6));
                s->plans.put(rc.ops, n, std::move(rc.plan), s->stream);
                s->perm = memo;
                s->tile_h = 6;
                s->relayout = true;
                s->calibrated = timing;
                return;
            }
        }
    }
    {
        std::vector<int> memo;
        int mh = -1;
        const TileHeightScope scope(th);
        // (a forced relayout plan does not take a fixed-layout decision made before)
        if (!relayout_forced() && layout_memo_get(n, 0, gates, bytes, memo, heights ? &mh : nullptr)) {
            s->perm = memo;  // decided before for this circuit (its plan: the plan cache)
            if (heights) s->tile_h = mh;
            s->calibrated = heights;  // (a cross-height decision is always a timed one)
            return;
        }
    }
    struct Gen {
        int h;
        double t13;
        size_t alts;
    };
    std::vector<Gen> gens{{th, layout_t13(), relabel_calibrate(n) ? alts : 0}};
    if (heights) {
        if (th == 7) gens.push_back({6, 1.0, alts});
        else gens.insert(gens.end(), {{7, 1.25, alts}, {7, 1.0, 0}});
    }
    std::vector<LayoutCandidate> cands;
    auto add = [&](int h, std::vector<int> perm, std::vector<Op> ops, Plan plan, bool rl = false) {
        for (const LayoutCandidate& c : cands)
            if (c.h == h && c.perm == perm && c.relayout == rl) return;  // the same candidate twice
        cands.push_back(LayoutCandidate{h, std::move(perm), std::move(ops), std::move(plan), rl});
    };
    // Relayout plan (12-qubit tiles, every pass stores under the next pass's layout): a
    // candidate like the others when candidates are timed, else taken when it needs fewer passes
    // than the fixed-layout choice.
    // (planned on a worker thread while the fixed-layout candidates are chosen)
    RelayoutChoice rc;  // the best predicted variant (timing compares all of rcs)
    std::vector<RelayoutChoice> rcs;
    bool have_rc = false;
    struct Joiner {
        std::thread t;
        void join() {
            if (t.joinable()) t.join();
        }
        ~Joiner() { join(); }
    } rc_worker;
    if (relayout)
        rc_worker.t = std::thread([&] {
            try {
                const TileHeightScope scope(6, tile_rb_for(n, 6));
                have_rc = plan_relayout_variants(n, lower_under, SIZE_MAX, rcs) > 0;
                if (have_rc) rc = rcs.front();
            } catch (...) {
                have_rc = false;  // (no relayout candidate)
            }
        });
    const bool force_rc = relayout_forced();  // (tests: QSIM_RELAYOUT=2 / qsim_set_relayout(2))
    auto take_relayout = [&]() {
        {
            const TileHeightScope scope(6, tile_rb_for(n, 6));
            s->plans.put(rc.ops, n, std::move(rc.plan), s->stream);
        }
        s->perm = rc.perm;
        s->tile_h = 6;
        s->relayout = true;
        layout_memo_put(n, 2, gates, bytes, s->perm, timing ? 6 : -1);
    };
    if (!relabel_enabled(n)) {
        // relayout only (states below the relabeling threshold): taken when it needs fewer
        // passes than the circuit's plan under the identity labels
        if (!relayout) return;  // (no room for the second buffer: nothing to decide, no memo)
        rc_worker.join();
        std::vector<int> id(n);
        for (int q = 0; q < n; ++q) id[q] = q;
        std::vector<Op> ops0 = lower_under(id);
        Plan p0;
        {
            const TileHeightScope scope(th, tile_rb_for(n, th));
            p0 = plan_fused(ops0, n, th);
        }
        // with inline compilation (the bench's mode) the identity-label plan and the relayout
        // variants are timed on the device, as at the first run of larger states
        static const bool time_small = [] {
            const char* e = std::getenv("QSIM_RELAYOUT_TIME_SMALL");
            return e == nullptr || std::atoi(e) != 0;
        }();
        if (have_rc && !force_rc && time_small && jit_mode() == 2 && calibrate_mode_on()) {
            add(th, {}, ops0, p0);
            for (const RelayoutChoice& v : rcs)
                if (v.plan.passes.size() <= p0.passes.size()) add(6, v.perm, v.ops, v.plan, true);
            if (cands.size() > 1) {
                LayoutCandidate& w = cands[calibrate_candidates(s, cands)];
                s->calibrated = true;
                if (w.relayout) {
                    rc.perm = w.perm;
                    rc.ops = w.ops;
                    rc.plan = w.plan;
                    take_relayout();
                } else {
                    layout_memo_put(n, 2, gates, bytes, {}, -1);
                }
                return;
            }
            cands.clear();
        }
        if (have_rc && (force_rc || rc.plan.passes.size() < p0.passes.size())) {
            take_relayout();
        } else {
            layout_memo_put(n, 2, gates, bytes, {}, -1);
        }
        return;
    }
    if (force_rc) {  // (tests: a relayout plan whenever one exists)
        rc_worker.join();
        if (have_rc) {
            take_relayout();
            return;
        }
    }
    // The relayout planner keeps running on its worker while the fixed-layout candidates are
    // chosen below; it is joined where its result is first needed.
    for (const Gen& g : gens) {
        const TileHeightScope scope(g.h, tile_rb_for(n, g.h));
        const LayoutT13Scope t13(g.t13);
        LayoutChoice lc = choose_layout(n, lower_under, relabel_tries(), g.alts);
        if (lc.perm.empty()) {  // the identity is this height's choice
            rc_worker.join();
            if (!heights && !(have_rc && timing)) {  // (nothing to time)
                if (have_rc && rc.plan.passes.size() < lc.passes_before) {
                    take_relayout();
                    return;
                }
                memo_put({});
                return;
            }
            std::vector<int> id(n);
            for (int q = 0; q < n; ++q) id[q] = q;
            std::vector<Op> ops = lower_under(id);
            Plan plan = plan_fused(ops, n, g.h);
            add(g.h, {}, std::move(ops), std::move(plan));
        } else {
            add(g.h, std::move(lc.perm), std::move(lc.ops), std::move(lc.plan));
        }
        for (LayoutChoice::Alt& a : lc.alts) add(g.h, std::move(a.perm), std::move(a.ops), std::move(a.plan));
    }
    rc_worker.join();
    if (have_rc) {
        if (timing) {
            for (const RelayoutChoice& v : rcs) add(6, v.perm, v.ops, v.plan, true);
        } else if (rc.plan.passes.size() < cands[0].plan.passes.size()) {
            take_relayout();
            return;
        }
    }
    size_t best = 0;
    if (cands.size() > 1) {
        best = calibrate_candidates(s, cands);  // (their plans stay cached, compiled)
    } else {
        const TileHeightScope scope(cands[0].h, tile_rb_for(n, cands[0].h));
        if (!cands[0].perm.empty()) s->plans.put(cands[0].ops, n, cands[0].plan, s->stream);
    }
    LayoutCandidate& w = cands[best];
    s->calibrated = cands.size() > 1;
    if (w.relayout) {  // (re-put: the timing loop may have evicted it)
        rc.perm = w.perm;
        rc.ops = w.ops;
        rc.plan = w.plan;
        take_relayout();
        return;
    }
    if (heights) s->tile_h = w.h;
    s->perm = std::move(w.perm);
    memo_put(s->perm);
}

// An op with every index bit moved through pi (bit b -> position pi[b]).
static Op permute_op(Op o, const std::vector<int>& pi) {
    o.t0 = pi[o.t0];
    if (o.t1 >= 0) o.t1 = pi[o.t1];
    uint64_t m = 0;
    for (uint64_t c = o.cmask; c; c &= c - 1) m |= 1ull << pi[__builtin_ctzll(c)];
    o.cmask = m;
    return o;
}
// Density-matrix relabeling: the 2n index bits of rho under a permutation that plans the lowered
// circuit (density.hip dm_lower) into fewer passes — the state-vector search (relabel.hip
// choose_layout: seeded random labelings, the fewest-pass ones annealed on the layout cost
// model) over bit positions rather than qubits, so row and column bits move independently.
// QSIM_DM_RELABEL_TRIES labelings (default 48, about 1 s of host planning at 14 qubits; 256 when
// the candidates are timed on the device — more fewest-pass candidates to time: 14q 9.19k ->
// 9.52k gates/s); 0 turns it off.
// Below 24 index bits (rho of <= 11 qubits: ~1 ms passes) a quarter of that (the search
// is paid on the first run of every new circuit structure).
static int dm_relabel_tries(int nbits, bool timed = false) {
    static const int v = [] {
        const char* e = std::getenv("QSIM_DM_RELABEL_TRIES");
        return e ? std::max(0, std::atoi(e)) : -1;
    }();
    if (v >= 0) return v;
    const int full = timed ? 256 : 48;
    return nbits >= 24 ? full : full / 4;
}
// The DM relabeling follows the state-vector relabel policy (qsim_set_relabel / QSIM_RELABEL: mode
// 0 turns it off) with its own size floor in index bits (QSIM_DM_RELABEL_MIN_BITS, default 16:
// rho of 8 qubits).
static bool dm_relabel_enabled(int nbits) {
    static const int min_bits = [] {
        const char* e = std::getenv("QSIM_DM_RELABEL_MIN_BITS");
        return e ? std::max(2, std::atoi(e)) : 16;
    }();
    return relabel_mode_on() && nbits >= min_bits && dm_relabel_tries(nbits) > 0;
}
static LayoutChoice dm_choose_layout(int nbits, const std::vector<Op>& ops, size_t want_alts = 0) {
    auto lower = [&](const std::vector<int>& pi) {
        std::vector<Op> out;
        out.reserve(ops.size());
        for (const Op& o : ops) out.push_back(permute_op(o, pi));
        return out;
    };
    // QSIM_DM_STAGE_US (default 1000, layout-cost units per register stage; 0: cost alone): the
    // round-5 timed candidates at 14 qubits ran ~0.1 ms longer per stage and per 1 000 units of
    // predicted cost (profiles/r05/dm_relabel/sweep, stage counts from QSIM_DM_CAND_DEBUG)
    static const double stage_us = [] {
        const char* e = std::getenv("QSIM_DM_STAGE_US");
        return e ? std::max(0.0, std::atof(e)) : 1000.0;
    }();
    return choose_layout(nbits, lower, dm_relabel_tries(nbits, want_alts > 0), want_alts, stage_us);
}

static qsim_gate map_gate(const qsim_state* s, const qsim_gate& g) {
    qsim_gate m = g;
    if (!s->perm.empty())
        for (int j = 0; j < g.nqubits && j < 3; ++j)
            if (g.qubits[j] >= 0 && g.qubits[j] < s->n) m.qubits[j] = s->perm[g.qubits[j]];
    return m;
}

extern "C" {

const char* qsim_last_error(void) { return g_last_error.c_str(); }

int qsim_state_last_run(qsim_state* s, int* passes, int* jit_passes) {
    return guarded([&] {
        check_state(s);
        if (passes) *passes = s->last_passes;
        if (jit_passes) *jit_passes = s->last_jit_passes;
    });
}
int qsim_abi_version(void) { return QSIM_ABI_VERSION; }

int qsim_state_layout_info(qsim_state* s, int* tile_h, int* calibrated, int* relabeled) {
    return guarded([&] {
        check_state(s);
        if (tile_h) *tile_h = s->tile_h >= 0 ? s->tile_h : tile_height_for(s->n);
        if (calibrated) *calibrated = s->calibrated ? 1 : 0;
        if (relabeled) *relabeled = s->perm.empty() ? 0 : 1;
    });
}

int qsim_state_relayout(qsim_state* s, int* relayout) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(relayout, QSIM_ERR_INVALID_ARGUMENT, "null out");
        *relayout = s->relayout ? 1 : 0;
    });
}

int qsim_state_restore_layout(qsim_state* s) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        canonicalize(s);
    });
}

int qsim_set_tile_height(int h) {
    return guarded([&] { tile_height_configure(h); });
}

int qsim_set_tile_ctrl_out(int mode) {
    return guarded([&] { tile_ctrl_out_configure(mode); });
}

int qsim_set_tile_rb7(int rb) {
    return guarded([&] { tile_rb7_configure(rb); });
}

int qsim_set_calibrate(int mode, int min_qubits) {
    return guarded([&] { calibrate_configure(mode, min_qubits); });
}

int qsim_set_device(int device) {
    return guarded([&] {
        int c = 0;
        QSIM_HIPCHK(hipGetDeviceCount(&c));
        if (device < 0 || device >= c) fail(QSIM_ERR_INVALID_ARGUMENT, "device index out of range");
        QSIM_HIPCHK(hipSetDevice(device));
    });
}

int qsim_device_count(int* count) {
    return guarded([&] {
        QSIM_REQUIRE(count, QSIM_ERR_INVALID_ARGUMENT, "null count");
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        if (e != hipSuccess) c = 0;
        *count = c;
    });
}

int qsim_device_info(int device, char* name, size_t name_len, int* cu_count, size_t* total_mem) {
    return guarded([&] {
        hipDeviceProp_t p;
        QSIM_HIPCHK(hipGetDeviceProperties(&p, device));
        if (name && name_len) {
            std::strncpy(name, p.name, name_len - 1);
            name[name_len - 1] = 0;
        }
        if (cu_count) *cu_count = p.multiProcessorCount;
        if (total_mem) *total_mem = p.totalGlobalMem;
    });
}

int qsim_state_create_on(int device, int n_qubits, qsim_state** out) {
    return guarded([&] {
        QSIM_REQUIRE(out, QSIM_ERR_INVALID_ARGUMENT, "null out");
        *out = nullptr;
        // StateVector ctor validation (src/StateVector.cu:135-141, Constants.hpp:68-69)
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > QSIM_MAX_QUBITS_SINGLE)
            fail(QSIM_ERR_INVALID_ARGUMENT, "Number of qubits must be between " +
                                                std::to_string(QSIM_MIN_QUBITS) + " and " +
                                                std::to_string(QSIM_MAX_QUBITS_SINGLE));
        DeviceGuard g(device);
        auto s = std::make_unique<qsim_state>();
        s->n = n_qubits;
        s->device = device;
        QSIM_HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        s->timer.stream = s->stream;
        // QSIM_STATE_OFFSET_KB (experiments): the amplitudes start that far into their allocation
        static const size_t off = [] {
            const char* e = std::getenv("QSIM_STATE_OFFSET_KB");
            return e ? (size_t)std::max(0ll, std::atoll(e)) * 1024 : (size_t)0;
        }();
        static const int contiguous = [] {  // QSIM_STATE_CONTIGUOUS (experiments)
            const char* e = std::getenv("QSIM_STATE_CONTIGUOUS");
            return e ? std::atoi(e) : 0;
        }();
        const size_t sbytes = ((sizeof(double2)) << n_qubits) + off;
        if (!contiguous || hipExtMallocWithFlags(&s->base, sbytes, hipDeviceMallocContiguous) != hipSuccess) {
            (void)hipGetLastError();
            s->base = nullptr;
            QSIM_HIPCHK(hipMalloc(&s->base, sbytes));
        }
        s->d = reinterpret_cast<double2*>(reinterpret_cast<char*>(s->base) + off);
        s->base_d = s->d;
        QSIM_HIPCHK(hipMalloc((void**)&s->d_partials, 4096 * sizeof(double)));
        QSIM_HIPCHK(hipMalloc((void**)&s->d_result, sizeof(double)));
        launch_init_basis(s->d, s->n, 1, 0, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
        *out = s.release();
    });
}

int qsim_state_create(int n_qubits, qsim_state** out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return qsim_state_create_on(dev, n_qubits, out);
}

int qsim_state_destroy(qsim_state* s) {
    return guarded([&] {
        if (!s) return;
        DeviceGuard g(s->device);
        delete s;
    });
}

int qsim_state_num_qubits(const qsim_state* s, int* n) {
    return guarded([&] {
        check_state(s);
        *n = s->n;
    });
}

int qsim_state_device_ptr(qsim_state* s, void** dptr) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        prep(s, true);  // the caller may read or write through the pointer
        s->pinned = true;  // (relayout runs copy their result back to this buffer)
        *dptr = s->d;
    });
}

int qsim_state_stream(qsim_state* s, void** stream) {
    return guarded([&] {
        check_state(s);
        *stream = (void*)s->stream;
    });
}

int qsim_state_init_zero(qsim_state* s) {
    return guarded([&] {
        check_state(s);
        DeviceGuard g(s->device);
        launch_init_basis(s->d, s->n, 1, 0, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
        s->perm.clear();
        s->basis = true;
        s->basis_idx = 0;
        s->tile_h = -1;  // (the next first run chooses again: memo)
        s->calibrated = false;
        s->relayout = false;
    });
}

int qsim_state_init_basis(qsim_state* s, uint64_t idx) {
    return guarded([&] {
        check_state(s);
        if (idx >= (1ull << s->n)) fail(QSIM_ERR_INVALID_ARGUMENT, "Basis index out of range");
        DeviceGuard g(s->device);
        launch_init_basis(s->d, s->n, 1, idx, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
        s->perm.clear();
        s->basis = true;
        s->basis_idx = idx;
        s->tile_h = -1;
        s->calibrated = false;
        s->relayout = false;
    });
}

int qsim_state_sync(qsim_state* s) {
    return guarded([&] {
        check_state(s);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_apply_gate(qsim_state* s, const qsim_gate* g) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(g, QSIM_ERR_INVALID_ARGUMENT, "null gate");
        DeviceGuard dg(s->device);
        validate_gate(*g, s->n);
        const Op op = lower_gate(map_gate(s, *g), s->n);
        s->basis = false;
        launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
    });
}

int qsim_run(qsim_state* s, const qsim_gate* gates, size_t count, int flags) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        DeviceGuard dg(s->device);
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], s->n);
        auto lower_all = [&]() {
            std::vector<Op> ops;
            ops.reserve(count);
            for (size_t i = 0; i < count; ++i) {
                ops.push_back(lower_gate(map_gate(s, gates[i]), s->n));
                ops.back().src = (int)i;
            }
            return ops;
        };
        // First run on a basis state: choose the qubit labels (and, with cross-height calibration,
        // the tile height) for fewer passes and faster pass layouts (relabel.hip: choose_layout).
        // A state whose raw device pointer was handed out (devicePtr) is never relabeled: the
        // pointer must always see the canonical amplitudes (reference include/StateVector.cuh:
        // devicePtr() is the state itself), and a relabeled run would leave them qubit-permuted
        // there until the next index-based reader.  So pinned states run the identity layout in
        // place (no relayout plan, no second buffer, no copy-back).
        if ((flags & QSIM_RUN_FUSED) && !s->pinned && s->basis && s->perm.empty() && count > 0 &&
            (relabel_enabled(s->n) || (relayout_enabled(s->n) && relabel_mode_on() && !tile_height_is_set()))) {
            choose_first_layout(s, gates, count);
            if (!s->perm.empty() && s->basis_idx) {  // relabel the basis state itself
                uint64_t k = 0;
                for (int q = 0; q < s->n; ++q)
                    if ((s->basis_idx >> q) & 1ull) k |= 1ull << s->perm[q];
                launch_init_basis(s->d, s->n, 1, k, s->stream);
            }
        }
        const int th = s->tile_h >= 0 ? s->tile_h : tile_height_for(s->n);
        const TileHeightScope tile_h(th, tile_rb_for(s->n, th));  // plans of this run
        const std::vector<Op> ops = lower_all();
        s->basis = false;
        if (flags & QSIM_RUN_FUSED) {
            run_fused(s, ops);
        } else {
            for (const Op& op : ops) launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
        }
    });
}

int qsim_apply_matrix1q(qsim_state* s, int target, const double m[8], const int* controls,
                        int n_controls) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(m, QSIM_ERR_INVALID_ARGUMENT, "null matrix");
        if (target < 0 || target >= s->n)
            fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(target) + " out of range");
        Op op;
        op.kind = K_M1;
        op.sub = S_GEN;
        op.t0 = target;
        for (int i = 0; i < 8; ++i) op.m[i] = m[i];
        for (int i = 0; i < n_controls; ++i) {
            const int c = controls[i];
            if (c < 0 || c >= s->n)
                fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(c) + " out of range");
            if (c == target || ((op.cmask >> c) & 1ull))
                fail(QSIM_ERR_INVALID_ARGUMENT, "control qubits must be distinct from target");
            op.cmask |= 1ull << c;
        }
        DeviceGuard dg(s->device);
        prep(s, true);
        launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
    });
}

int qsim_apply_matrix2q(qsim_state* s, int q0, int q1, const double m[32], const int* controls,
                        int n_controls) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(m, QSIM_ERR_INVALID_ARGUMENT, "null matrix");
        QSIM_REQUIRE(controls || n_controls == 0, QSIM_ERR_INVALID_ARGUMENT, "null controls");
        for (int q : {q0, q1})
            if (q < 0 || q >= s->n) fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(q) + " out of range");
        if (q0 == q1) fail(QSIM_ERR_INVALID_ARGUMENT, "Two-qubit gate requires distinct qubits");
        uint64_t cm = 0;
        for (int i = 0; i < n_controls; ++i) {
            const int c = controls[i];
            if (c < 0 || c >= s->n) fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(c) + " out of range");
            if (c == q0 || c == q1 || ((cm >> c) & 1ull))
                fail(QSIM_ERR_INVALID_ARGUMENT, "control qubits must be distinct from the targets");
            cm |= 1ull << c;
        }
        DeviceGuard dg(s->device);
        prep(s, true);
        launch_matrix2q(s->d, s->n, q0, q1, m, cm, s->stream, &s->timer);
    });
}

int qsim_apply_matrix(qsim_state* s, const int* targets, int k, const double* m,
                      const int* controls, int n_controls) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(m && targets, QSIM_ERR_INVALID_ARGUMENT, "null matrix or targets");
        QSIM_REQUIRE(controls || n_controls == 0, QSIM_ERR_INVALID_ARGUMENT, "null controls");
        if (k < 1 || k > 8) fail(QSIM_ERR_INVALID_ARGUMENT, "matrix must act on 1 to 8 qubits");
        uint64_t used = 0, cm = 0;
        for (int j = 0; j < k; ++j) {
            const int q = targets[j];
            if (q < 0 || q >= s->n) fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(q) + " out of range");
            if ((used >> q) & 1ull) fail(QSIM_ERR_INVALID_ARGUMENT, "target qubits must be distinct");
            used |= 1ull << q;
        }
        for (int i = 0; i < n_controls; ++i) {
            const int c = controls[i];
            if (c < 0 || c >= s->n) fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(c) + " out of range");
            if ((used >> c) & 1ull)
                fail(QSIM_ERR_INVALID_ARGUMENT, "control qubits must be distinct from the targets");
            used |= 1ull << c;
            cm |= 1ull << c;
        }
        DeviceGuard dg(s->device);
        prep(s, true);
        const int dim = 1 << k;
        std::vector<double> mt(2 * (size_t)dim * dim);  // transpose: mt[c][r] = M[r][c]
        for (int r = 0; r < dim; ++r)
            for (int c = 0; c < dim; ++c) {
                mt[2 * ((size_t)c * dim + r)] = m[2 * ((size_t)r * dim + c)];
                mt[2 * ((size_t)c * dim + r) + 1] = m[2 * ((size_t)r * dim + c) + 1];
            }
        double2* d_mt = (double2*)s->scratch.get(mt.size() * sizeof(double), s->stream);
        QSIM_HIPCHK(hipMemcpyAsync(d_mt, mt.data(), mt.size() * sizeof(double), hipMemcpyHostToDevice,
                                   s->stream));
        launch_matrixk(s->d, s->n, targets, k, d_mt, cm, s->stream, &s->timer);
        // the matrix lives in the state's scratch: wait before the next user may reuse it
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_apply_hadamard_optimized(void* dstate, int n_qubits, int target, void* stream) {
    qsim_gate g{};
    g.type = QSIM_GATE_H;
    g.nqubits = 1;
    g.qubits[0] = target;
    return qsim_apply_gate_raw(dstate, n_qubits, &g, stream);
}

int qsim_apply_cnot_optimized(void* dstate, int n_qubits, int control, int target, void* stream) {
    qsim_gate g{};
    g.type = QSIM_GATE_CNOT;
    g.nqubits = 2;
    g.qubits[0] = control;
    g.qubits[1] = target;
    return qsim_apply_gate_raw(dstate, n_qubits, &g, stream);
}

int qsim_apply_matrix1q_raw(void* dstate, int n_qubits, int target, const double m[8], void* stream) {
    return guarded([&] {
        QSIM_REQUIRE(dstate && m, QSIM_ERR_INVALID_ARGUMENT, "null argument");
        if (n_qubits < 1 || n_qubits > QSIM_MAX_QUBITS_SINGLE)
            fail(QSIM_ERR_INVALID_ARGUMENT, "Number of qubits must be between 1 and 30");
        if (target < 0 || target >= n_qubits)
            fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(target) + " out of range");
        Op op;
        op.kind = K_M1;
        op.sub = S_GEN;
        op.t0 = target;
        for (int i = 0; i < 8; ++i) op.m[i] = m[i];
        launch_op((double2*)dstate, n_qubits, 1, op, (hipStream_t)stream, nullptr);
    });
}

int qsim_apply_diagonal_layer(qsim_state* s, const double* gp, uint64_t active) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(gp || active == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate_params");
        if (s->n < 64 && (active >> s->n)) fail(QSIM_ERR_OUT_OF_RANGE, "active mask names a qubit >= n");
        std::vector<Op> ops;
        for (int q = 0; q < s->n; ++q) {
            if (!((active >> q) & 1ull)) continue;
            Op o;
            o.kind = K_DIAG;
            o.sub = S_GEN;
            o.t0 = q;
            o.m[0] = gp[8 * q + 0];
            o.m[1] = gp[8 * q + 1];
            o.m[2] = gp[8 * q + 6];
            o.m[3] = gp[8 * q + 7];
            o.d0_one = o.m[0] == 1.0 && o.m[1] == 0.0;
            o.src = (int)ops.size();
            ops.push_back(o);
        }
        DeviceGuard dg(s->device);
        prep(s, true);
        if (!ops.empty()) run_fused(s, ops);
    });
}

int qsim_plan_fused(int n_qubits, const qsim_gate* gates, size_t count, int hmax, int32_t* order,
                    int32_t* pass_of, int32_t* n_passes) {
    return guarded([&] {
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > 40) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        if (hmax < 0 || hmax > kTileHMax) fail(QSIM_ERR_INVALID_ARGUMENT, "hmax out of range");
        std::vector<Op> ops;
        for (size_t i = 0; i < count; ++i) {
            ops.push_back(lower_gate(gates[i], n_qubits));
            ops.back().src = (int)i;
        }
        const Plan plan = plan_fused(ops, n_qubits, hmax);
        size_t k = 0;
        int32_t tile = 0;
        for (const FusedPass& p : plan.passes) {
            if (p.single >= 0) {
                if (order) order[k] = plan.singles[p.single].src;
                if (pass_of) pass_of[k] = -1;
                ++k;
                continue;
            }
            auto emit = [&](int o) {
                if (plan.order[o] < 0) return;  // 2nd/3rd controlled-X of a lowered SWAP
                if (order) order[k] = plan.order[o];
                if (pass_of) pass_of[k] = tile;
                ++k;
            };
            if (p.stage_end > p.stage_begin) {
                for (int s = p.stage_begin; s < p.stage_end; ++s)
                    for (int o = plan.stages[s].op_begin; o < plan.stages[s].op_end; ++o) emit(o);
            } else {
                for (int o = p.op_begin; o < p.op_end; ++o) emit(o);
            }
            ++tile;
        }
        if (n_passes) *n_passes = tile;
    });
}

int qsim_set_jit(int mode, int min_qubits) {
    return guarded([&] {
        if (mode > 2) fail(QSIM_ERR_INVALID_ARGUMENT, "jit mode must be 0 (off), 1 (background) or 2 (inline)");
        jit_configure(mode, min_qubits);
    });
}

int qsim_set_relabel(int mode, int min_qubits) {
    return guarded([&] {
        if (mode > 1) fail(QSIM_ERR_INVALID_ARGUMENT, "relabel mode must be 0 (off) or 1 (on)");
        relabel_configure(mode, min_qubits);
    });
}

int qsim_state_perm(qsim_state* s, int32_t* perm) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(perm, QSIM_ERR_INVALID_ARGUMENT, "null perm");
        for (int q = 0; q < s->n; ++q) perm[q] = s->perm.empty() ? q : s->perm[q];
    });
}

int qsim_plan_relabel(int n_qubits, const qsim_gate* gates, size_t count, int32_t* perm,
                      double* cost_before_us, double* cost_after_us) {
    return guarded([&] {
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > 40) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], n_qubits);
        auto lower_under = [&](const std::vector<int>& pi) {
            std::vector<Op> ops;
            for (size_t i = 0; i < count; ++i) {
                qsim_gate m = gates[i];
                for (int j = 0; j < m.nqubits && j < 3; ++j) m.qubits[j] = pi[m.qubits[j]];
                ops.push_back(lower_gate(m, n_qubits));
                ops.back().src = (int)i;
            }
            return ops;
        };
        const LayoutChoice lc = choose_layout(n_qubits, lower_under, relabel_tries());
        if (perm)
            for (int q = 0; q < n_qubits; ++q) perm[q] = lc.perm.empty() ? q : lc.perm[q];
        if (cost_before_us) *cost_before_us = lc.cost_before;
        if (cost_after_us) *cost_after_us = lc.cost_after;
    });
}

int qsim_jit_shutdown(void) {
    return guarded([&] { jit_shutdown(); });
}

int qsim_jit_source(int n_qubits, const qsim_gate* gates, size_t count, char* buf, size_t cap,
                    size_t* len) {
    return guarded([&] {
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > 40) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        std::vector<Op> ops;
        for (size_t i = 0; i < count; ++i) {
            ops.push_back(lower_gate(gates[i], n_qubits));
            ops.back().src = (int)i;
        }
        const std::string src = jit_source(plan_fused(ops, n_qubits));
        if (len) *len = src.size();
        if (buf && cap) {
            const size_t m = std::min(cap - 1, src.size());
            std::memcpy(buf, src.data(), m);
            buf[m] = 0;
        }
    });
}

int qsim_jit_build(int n_qubits, const qsim_gate* gates, size_t count, size_t* code_bytes) {
    return guarded([&] {
        size_t len = 0;
        const int rc = qsim_jit_source(n_qubits, gates, count, nullptr, 0, &len);
        if (rc != QSIM_OK) fail(rc, qsim_last_error());
        std::string src(len + 1, '\0');
        qsim_jit_source(n_qubits, gates, count, &src[0], len + 1, &len);
        src.resize(len);
        std::vector<char> code;
        std::string log;
        if (!src.empty() && !jit_compile(src, code, log)) fail(QSIM_ERR_RUNTIME, "hipRTC: " + log);
        if (code_bytes) *code_bytes = code.size();
    });
}

int qsim_jit_build_relayout(int n_qubits, const qsim_gate* gates, size_t count, size_t* code_bytes) {
    return guarded([&] {
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > 40) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        for (size_t i = 0; i < count; ++i) validate_gate(gates[i], n_qubits);
        auto lower = [&](const std::vector<int>& pi) {
            std::vector<Op> ops;
            for (size_t i = 0; i < count; ++i) {
                qsim_gate m = gates[i];
                for (int j = 0; j < m.nqubits && j < 3; ++j) m.qubits[j] = pi[m.qubits[j]];
                ops.push_back(lower_gate(m, n_qubits));
                ops.back().src = (int)i;
            }
            return ops;
        };
        RelayoutChoice rc;
        if (!plan_relayout(n_qubits, lower, SIZE_MAX, rc)) fail(QSIM_ERR_RUNTIME, "no relayout plan");
        const std::string src = jit_source(rc.plan);
        std::vector<char> code;
        std::string log;
        if (!src.empty() && !jit_compile(src, code, log)) fail(QSIM_ERR_RUNTIME, "hipRTC: " + log);
        if (code_bytes) *code_bytes = code.size();
    });
}

int qsim_apply_gate_raw(void* dstate, int n_qubits, const qsim_gate* g, void* stream) {
    return guarded([&] {
        QSIM_REQUIRE(dstate && g, QSIM_ERR_INVALID_ARGUMENT, "null argument");
        if (n_qubits < QSIM_MIN_QUBITS || n_qubits > 40)
            fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        const Op op = lower_gate(*g, n_qubits);
        launch_op((double2*)dstate, n_qubits, 1, op, (hipStream_t)stream, nullptr);
    });
}

int qsim_state_to_host(qsim_state* s, double* dst) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(dst, QSIM_ERR_INVALID_ARGUMENT, "null destination");
        DeviceGuard dg(s->device);
        prep(s, false);
        QSIM_HIPCHK(hipMemcpyAsync(dst, s->d, sizeof(double2) << s->n, hipMemcpyDeviceToHost,
                                   s->stream));
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_state_from_host(qsim_state* s, const double* src) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(src, QSIM_ERR_INVALID_ARGUMENT, "null source");
        DeviceGuard dg(s->device);
        s->perm.clear();  // overwritten in logical order
        s->basis = false;
        QSIM_HIPCHK(hipMemcpyAsync(s->d, src, sizeof(double2) << s->n, hipMemcpyHostToDevice,
                                   s->stream));
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_state_probabilities(qsim_state* s, double* dst) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(dst, QSIM_ERR_INVALID_ARGUMENT, "null destination");
        DeviceGuard dg(s->device);
        prep(s, false);
        const uint64_t N = 1ull << s->n;
        double* d_p = (double*)s->scratch.get(N * sizeof(double), s->stream);
        launch_probabilities(s->d, N, d_p, s->stream);
        QSIM_HIPCHK(hipMemcpyAsync(dst, d_p, N * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_state_total_probability(qsim_state* s, double* out) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(out, QSIM_ERR_INVALID_ARGUMENT, "null out");
        DeviceGuard dg(s->device);
        *out = reduce_norm(s->d, s->n, -1, s->d_partials, s->d_result, s->stream);
    });
}

int qsim_state_prob_bit_zero(qsim_state* s, int bit, double* out) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(out, QSIM_ERR_INVALID_ARGUMENT, "null out");
        if (bit < 0 || bit >= s->n) fail(QSIM_ERR_INVALID_ARGUMENT, "bit out of range");
        DeviceGuard dg(s->device);
        prep(s, false);
        *out = reduce_norm(s->d, s->n, bit, s->d_partials, s->d_result, s->stream);
    });
}

int qsim_state_max_abs_diff(qsim_state* a, qsim_state* b, double* out) {
    return guarded([&] {
        check_state(a);
        check_state(b);
        QSIM_REQUIRE(out, QSIM_ERR_INVALID_ARGUMENT, "null out");
        if (a->n != b->n) fail(QSIM_ERR_INVALID_ARGUMENT, "states have different qubit counts");
        if (a->device != b->device) fail(QSIM_ERR_INVALID_ARGUMENT, "states live on different devices");
        DeviceGuard dg(a->device);
        prep(a, false);  // both in the identity layout
        prep(b, false);
        QSIM_HIPCHK(hipStreamSynchronize(a->stream));  // a's writes done; b's stream orders the rest
        *out = a == b ? 0.0 : reduce_max_abs_diff(a->d, b->d, a->n, b->d_partials, b->d_result, b->stream);
    });
}

int qsim_state_memory_bytes(qsim_state* s, uint64_t* bytes) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(bytes, QSIM_ERR_INVALID_ARGUMENT, "null out");
        const uint64_t amps = sizeof(double2) << s->n;
        *bytes = amps + (s->alt_base ? amps : 0) + 4096 * sizeof(double) + sizeof(double) + s->scratch.cap +
                 s->ops.cap + s->stages.cap + 2 * s->noise_codes_cap + 2 * s->noise_lists_cap;
    });
}

int qsim_state_collapse(qsim_state* s, int bit, int result, double scale) {
    return guarded([&] {
        check_state(s);
        if (bit < 0 || bit >= s->n) fail(QSIM_ERR_INVALID_ARGUMENT, "bit out of range");
        if (result != 0 && result != 1) fail(QSIM_ERR_INVALID_ARGUMENT, "result must be 0 or 1");
        DeviceGuard dg(s->device);
        prep(s, true);
        launch_collapse(s->d, s->n, bit, result, scale, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_state_sample(qsim_state* s, const double* uniforms, int shots, int64_t* out) {
    return guarded([&] {
        check_state(s);
        if (shots <= 0) fail(QSIM_ERR_INVALID_ARGUMENT, "n_shots must be positive");
        QSIM_REQUIRE(uniforms && out, QSIM_ERR_INVALID_ARGUMENT, "null buffer");
        DeviceGuard dg(s->device);
        prep(s, false);
        sample_indices(s->d, s->n, 1, uniforms, shots, out, s->stream, s->scratch);
    });
}

int qsim_noise_apply(qsim_state* s, int type, int qubit, double probability, uint64_t seed,
                     uint64_t counter) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        prep(s, true);
        launch_noise(s->d, s->n, type, qubit, probability, seed, counter, s->stream, &s->timer);
    });
}

int qsim_noisy_run(qsim_state* s, const qsim_gate* gates, size_t count,
                   const qsim_noise_channel* channels, size_t n_channels, uint64_t seed,
                   uint64_t* counter, int flags) {
    return guarded([&] {
        check_state(s);
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        QSIM_REQUIRE(channels || n_channels == 0, QSIM_ERR_INVALID_ARGUMENT, "null channel list");
        QSIM_REQUIRE(counter, QSIM_ERR_INVALID_ARGUMENT, "null counter");
        DeviceGuard dg(s->device);
        prep(s, true);
        std::vector<Op> ops;
        for (size_t i = 0; i < count; ++i) {
            ops.push_back(lower_gate(gates[i], s->n));
            ops.back().src = (int)i;
        }
        for (size_t c = 0; c < n_channels; ++c) {
            if (channels[c].type < 0 || channels[c].type > 5)
                fail(QSIM_ERR_INVALID_ARGUMENT, "unknown noise type");
            if (channels[c].qubit < 0 || channels[c].qubit >= s->n)
                fail(QSIM_ERR_OUT_OF_RANGE, "Qubit index " + std::to_string(channels[c].qubit) + " out of range");
        }
        if (n_channels == 0) {
            if (flags & QSIM_RUN_FUSED) run_fused(s, ops);
            else for (const Op& op : ops) launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
            return;
        }
        std::vector<NoiseChan> chans;
        for (size_t c = 0; c < n_channels; ++c)
            chans.push_back(NoiseChan{channels[c].type, channels[c].qubit, channels[c].probability});
        // where the amplitudes are now: a pinned state's handed-out pointer (prep() leaves the
        // amplitudes of a pinned state in the buffer that was handed out, which may be either one)
        double2* const home = s->d;
        // QSIM_NOISY_TILE=1 (from 12 qubits, flip-only models): the in-tile path (noise.hip
        // launch_gate_noise_run: the gate and the channel prefix whose qubits lie in its tile in one
        // LDS pass, their flips from lists built one step ahead on noise_stream, the rest pushed one
        // launch per channel) — the same draws, so the same states as the pulled and pushed paths.
        // Opt-in: at 26 qubits with 26 channels the 14-15 per-channel suffix launches (0.04 ms
        // each) outweigh the pull pass, 904 vs 1 024 gates/s.
        {
            const char* te = std::getenv("QSIM_NOISY_TILE");  // (read per run: tests switch it)
            bool tile = te != nullptr && std::atoi(te) != 0 && s->n >= 12;
            for (const NoiseChan& ch : chans) tile = tile && (ch.type == 0 || ch.type >= 3);
            for (const Op& op : ops) tile = tile && gate_noise_tile_supported(s->n, &op);
            if (tile) {
                const size_t lb = gate_noise_lists_bytes(s->n, 1, chans);
                GnLists L{};
                const bool lists = lb && ensure_noise_lists(s, lb);
                if (lists) {
                    L.buf[0] = s->noise_lists;
                    L.buf[1] = s->noise_lists + s->noise_lists_cap;
                    L.set_bytes = s->noise_lists_cap;
                    L.ms = s->noise_stream;
                    L.built[0] = s->nev_map[0];
                    L.built[1] = s->nev_map[1];
                    L.used[0] = s->nev_pull[0];
                    L.used[1] = s->nev_pull[1];
                    L.start = s->nev_start;
                }
                launch_gate_noise_run(s->d, s->n, 1, 0, ops, chans, seed, *counter, s->stream, &s->timer,
                                      lists ? &L : nullptr);
                trim_noise_buffers(s);
                return;
            }
        }
        if (pull_noise_supported(s->n, chans, true) && ensure_noise_buffers(s, chans.size())) {
            // Flip channels only: the noise after gate i is applied by gate i+1's pass (out of
            // place), the noise after the last gate by one identity pass (noise.hip); the same
            // draws as the per-channel passes below, so the same state.
            // The words of step i (set i & 1) are built on noise_stream while the pass of step
            // i - 1 runs; the pass of step i waits for them, the words of step i + 2 for that pass
            // (QSIM_NOISE_MAP_OVERLAP=0: one stream).
            const char* oe = std::getenv("QSIM_NOISE_MAP_OVERLAP");
            const bool overlap = oe == nullptr || std::atoi(oe) != 0;
            const size_t G = ops.size();
            const uint64_t c0 = *counter;
            *counter += (uint64_t)G * n_channels;
            auto words = [&](size_t i) { return (void*)(s->noise_codes + (i & 1) * s->noise_codes_cap); };
            // QSIM_NOISE_MAP_FUSED=1 (opt-in): step i's pass also builds step i + 1's words (its
            // hash-and-log walks meant to fill its own memory stalls; noise.hip k_pull_gate<...,
            // MAP>), one stream.  Measured slower at 26 qubits: 1.22 ms per fused pass against
            // 0.70 + 0.24 ms apart, 815 vs 1 063 gates/s (the walks and their LDS cost the pass its
            // occupancy), so the default is the word map as a kernel of its own, beside the pass
            // (overlap) or before it.
            const char* fe = std::getenv("QSIM_NOISE_MAP_FUSED");
            if (fe != nullptr && std::atoi(fe) != 0 && G) {
                launch_noise_map(s->n, 1, 0, chans, seed, c0, words(0), s->stream, &s->timer);
                launch_op(s->d, s->n, 1, ops[0], s->stream, &s->timer);
                for (size_t i = 0; i < G; ++i) {
                    double2* dst = s->alt;
                    const PullMapNext nx{0, seed, c0 + (i + 1) * n_channels, words(i + 1)};
                    launch_pull_gate(s->d, dst, s->n, 1, chans, i + 1 < G ? &ops[i + 1] : nullptr, words(i), s->stream,
                                     &s->timer, i + 1 < G ? &nx : nullptr);
                    s->alt = s->d;
                    s->d = dst;
                }
                if (s->pinned && s->d != home) {
                    QSIM_HIPCHK(hipMemcpyAsync(home, s->d, sizeof(double2) << s->n, hipMemcpyDeviceToDevice,
                                               s->stream));
                    s->alt = s->d;
                    s->d = home;
                }
                trim_noise_buffers(s);
                return;
            }
            hipStream_t ms = overlap ? s->noise_stream : s->stream;
            auto map = [&](size_t i) {
                if (overlap && i >= 2) QSIM_HIPCHK(hipStreamWaitEvent(ms, s->nev_pull[i & 1], 0));
                launch_noise_map(s->n, 1, 0, chans, seed, c0 + i * n_channels, words(i), ms, &s->timer);
                if (overlap) QSIM_HIPCHK(hipEventRecord(s->nev_map[i & 1], ms));
            };
            if (overlap) {  // (the previous run's passes may still read both sets)
                QSIM_HIPCHK(hipEventRecord(s->nev_start, s->stream));
                QSIM_HIPCHK(hipStreamWaitEvent(ms, s->nev_start, 0));
                for (size_t i = 0; i < std::min<size_t>(G, 2); ++i) map(i);
            }
            if (G) launch_op(s->d, s->n, 1, ops[0], s->stream, &s->timer);
            for (size_t i = 0; i < G; ++i) {
                if (overlap) QSIM_HIPCHK(hipStreamWaitEvent(s->stream, s->nev_map[i & 1], 0));
                else map(i);
                double2* dst = s->alt;
                launch_pull_gate(s->d, dst, s->n, 1, chans, i + 1 < G ? &ops[i + 1] : nullptr, words(i), s->stream,
                                 &s->timer);
                s->alt = s->d;
                s->d = dst;
                if (overlap && i + 2 < G) {
                    QSIM_HIPCHK(hipEventRecord(s->nev_pull[i & 1], s->stream));
                    map(i + 2);
                }
            }
            if (s->pinned && s->d != home) {  // keep the amplitudes where the handed-out pointer points
                QSIM_HIPCHK(hipMemcpyAsync(home, s->d, sizeof(double2) << s->n, hipMemcpyDeviceToDevice,
                                           s->stream));
                s->alt = s->d;
                s->d = home;
            }
            // The second buffer and the code words stay for the next run (qsim_state_memory_bytes
            // counts them) only while the device keeps room for another state of this size beside
            // them; otherwise they are freed now, so a later StateVector does not fail where the
            // reference's single-buffer one would not.
            trim_noise_buffers(s);
            return;
        }
        for (const Op& op : ops) {
            launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
            for (size_t c = 0; c < n_channels; ++c)
                launch_noise(s->d, s->n, channels[c].type, channels[c].qubit, channels[c].probability,
                             seed, (*counter)++, s->stream, &s->timer);
        }
    });
}

static void check_dm(const qsim_state* s, int n) {
    check_state(s);
    if (n < 1 || n > QSIM_DM_MAX_QUBITS)
        fail(QSIM_ERR_INVALID_ARGUMENT, "Density matrix supports 1-" + std::to_string(QSIM_DM_MAX_QUBITS) + " qubits");
    if (s->n != 2 * n) fail(QSIM_ERR_INVALID_ARGUMENT, "density matrix state must have 2n qubits");
}

int qsim_dm_run(qsim_state* s, int n, const qsim_gate* gates, size_t count,
                const qsim_noise_channel* channels, size_t n_channels, int flags) {
    return guarded([&] {
        check_dm(s, n);
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        QSIM_REQUIRE(channels || n_channels == 0, QSIM_ERR_INVALID_ARGUMENT, "null channel list");
        DeviceGuard dg(s->device);
        std::vector<Op> ops;
        dm_lower(n, gates, count, channels, n_channels, ops, (flags & QSIM_DM_REFERENCE_Y) != 0);
        // the state-vector size rule for the 2n index bits (13-qubit tiles for 26-28 bits: DM 13-14
        // qubits; W-HC + depolarizing at 14 qubits 6.87 k -> 7.35 k gates/s, 8 -> 7 passes)
        const int th = tile_height_for(s->n);
        const TileHeightScope tile_h(th, tile_rb_for(s->n, th));
        // First fused run on |0><0| (a reset rho: basis index 0, which every labeling leaves at 0):
        // choose the index-bit labels (dm_choose_layout; W-HC + depolarizing 14q: 7 -> 6 passes),
        // memoised per (circuit, channels, flags).  Later runs keep the labels and map their ops
        // through them; readers restore the identity first (prep).  A pinned state (handed-out
        // device pointer) is never relabeled.
        const bool fresh = (flags & QSIM_RUN_FUSED) && !s->pinned && s->basis && s->basis_idx == 0 &&
                           s->perm.empty() && count > 0 && dm_relabel_enabled(s->n);
        if (fresh) {
            // memo key: the circuit's STRUCTURE (gate types and qubits, channel types and qubits,
            // flags) — not rotation angles or probabilities, so a parameter sweep (reset + run with
            // new angles) reuses the labels instead of searching again; any labels are exact, the
            // structure is what they were chosen for
            std::vector<int32_t> key;
            key.reserve(4 * count + 2 * n_channels + 2);
            for (size_t i = 0; i < count; ++i) {
                key.push_back(gates[i].type);
                for (int j = 0; j < 3; ++j) key.push_back(j < gates[i].nqubits ? gates[i].qubits[j] : -1);
            }
            for (size_t i = 0; i < n_channels; ++i) {
                key.push_back(channels[i].type);
                key.push_back(channels[i].qubit);
            }
            key.push_back((int32_t)count);
            key.push_back(flags);
            std::vector<int> memo;
            if (layout_memo_get(s->n, 3, key.data(), key.size() * sizeof(int32_t), memo, nullptr)) {
                s->perm = memo;
            } else {
                // with layout calibration (inline compilation, >= 26 index bits by default) the
                // fewest-pass candidates are timed on the device, as a state vector's are: the
                // cost model prices run lengths, not the register stages that DM passes spend
                // most of their time in (QSIM_DM_RELABEL_CANDIDATES, default 8; 14q: the 6-pass
                // candidates run 10.4-11.9 ms)
                static const size_t alts = [] {
                    const char* e = std::getenv("QSIM_DM_RELABEL_CANDIDATES");
                    return (size_t)std::max(1, e ? std::atoi(e) : 8) - 1;
                }();
                LayoutChoice lc = dm_choose_layout(s->n, ops, relabel_calibrate(s->n) ? alts : 0);
                if (!lc.perm.empty() && !lc.alts.empty()) {
                    std::vector<LayoutCandidate> cands;
                    cands.push_back(LayoutCandidate{th, lc.perm, std::move(lc.ops), std::move(lc.plan), false});
                    for (LayoutChoice::Alt& a : lc.alts)
                        cands.push_back(LayoutCandidate{th, a.perm, std::move(a.ops), std::move(a.plan), false});
                    s->perm = cands[calibrate_candidates(s, cands)].perm;  // (every plan stays cached)
                    s->calibrated = true;
                } else if (!lc.perm.empty()) {
                    s->plans.put(lc.ops, s->n, std::move(lc.plan), s->stream);
                    s->perm = lc.perm;
                }
                layout_memo_put(s->n, 3, key.data(), key.size() * sizeof(int32_t), s->perm, -1);
            }
        } else if (s->pinned || s->relayout) {
            prep(s, true);  // (identity labels; a relayout-plan layout is the state vector's own)
        }
        s->basis = false;
        if (!s->perm.empty())
            for (Op& o : ops) o = permute_op(o, s->perm);
        if (flags & QSIM_RUN_FUSED) run_fused(s, ops);
        else for (const Op& op : ops) launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
    });
}

int qsim_dm_plan_info(int n, const qsim_gate* gates, size_t count, const qsim_noise_channel* channels,
                      size_t n_channels, int flags, int32_t* info, size_t cap, size_t* n_passes) {
    return guarded([&] {
        if (n < 1 || n > QSIM_DM_MAX_QUBITS) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        QSIM_REQUIRE(channels || n_channels == 0, QSIM_ERR_INVALID_ARGUMENT, "null channel list");
        std::vector<Op> ops;
        dm_lower(n, gates, count, channels, n_channels, ops, (flags & QSIM_DM_REFERENCE_Y) != 0);
        const int th = tile_height_for(2 * n);
        const TileHeightScope tile_h(th, tile_rb_for(2 * n, th));
        Plan plan;
        LayoutChoice lc;
        if (flags & QSIM_DM_PLAN_RELABELED) {
            // (QSIM_DM_CAND_DEBUG: every candidate the timed first run would time, in its order:
            // passes, register stages per pass, layout cost)
            static const bool dbg = std::getenv("QSIM_DM_CAND_DEBUG") != nullptr;
            static const size_t nalt = [] {
                const char* e = std::getenv("QSIM_DM_CAND_DEBUG");
                return e ? (size_t)std::max(1, std::atoi(e)) : (size_t)1;
            }();
            lc = dm_choose_layout(2 * n, ops, dbg ? nalt - 1 : 0);
            if (dbg && !lc.perm.empty()) {
                auto show = [&](size_t k, const Plan& pl) {
                    int st = 0;
                    std::string per;
                    for (const FusedPass& fp : pl.passes) {
                        st += fp.stage_end - fp.stage_begin;
                        per += " " + std::to_string(fp.stage_end - fp.stage_begin);
                    }
                    std::fprintf(stderr, "[dmcand] %zu passes %zu stages %d (%s ) cost %.1f\n", k, pl.passes.size(), st,
                                 per.c_str(), plan_layout_cost_us(pl));
                };
                show(0, lc.plan);
                for (size_t a = 0; a < lc.alts.size(); ++a) show(a + 1, lc.alts[a].plan);
            }
        }
        if (!lc.perm.empty()) plan = std::move(lc.plan);
        else plan = plan_fused(ops, 2 * n);  // (as qsim_dm_run's run_fused plans it)
        for (size_t p = 0; p < plan.passes.size() && p < cap && info; ++p) {
            const FusedPass& fp = plan.passes[p];
            int nops = 0;
            for (int st = fp.stage_begin; st < fp.stage_end; ++st) nops += plan.stages[st].op_end - plan.stages[st].op_begin;
            if (fp.stage_end == fp.stage_begin) nops = fp.op_end - fp.op_begin;
            info[4 * p] = fp.single >= 0 ? -1 : fp.h;
            info[4 * p + 1] = nops;
            info[4 * p + 2] = fp.stage_end - fp.stage_begin;
            info[4 * p + 3] = fp.r0;
        }
        if (n_passes) *n_passes = plan.passes.size();
    });
}

int qsim_dm_jit_source(int n, const qsim_gate* gates, size_t count, const qsim_noise_channel* channels,
                       size_t n_channels, int flags, char* buf, size_t cap, size_t* len) {
    return guarded([&] {
        if (n < 1 || n > QSIM_DM_MAX_QUBITS) fail(QSIM_ERR_INVALID_ARGUMENT, "bad qubit count");
        QSIM_REQUIRE(gates || count == 0, QSIM_ERR_INVALID_ARGUMENT, "null gate list");
        QSIM_REQUIRE(channels || n_channels == 0, QSIM_ERR_INVALID_ARGUMENT, "null channel list");
        std::vector<Op> ops;
        dm_lower(n, gates, count, channels, n_channels, ops, (flags & QSIM_DM_REFERENCE_Y) != 0);
        const int th = tile_height_for(2 * n);
        const TileHeightScope tile_h(th, tile_rb_for(2 * n, th));
        const std::string src = jit_source(plan_fused(ops, 2 * n));
        if (len) *len = src.size();
        if (buf && cap) {
            const size_t m = std::min(cap - 1, src.size());
            std::memcpy(buf, src.data(), m);
            buf[m] = 0;
        }
    });
}

int qsim_dm_apply_channel(qsim_state* s, int n, int type, int qubit, double p) {
    return guarded([&] {
        check_dm(s, n);
        DeviceGuard dg(s->device);
        prep(s, true);
        std::vector<Op> ops;
        dm_lower_channel(n, type, qubit, p, ops);
        for (const Op& op : ops) launch_op(s->d, s->n, 1, op, s->stream, &s->timer);
    });
}

int qsim_dm_diagonal(qsim_state* s, int n, double* dst) {
    return guarded([&] {
        check_dm(s, n);
        QSIM_REQUIRE(dst, QSIM_ERR_INVALID_ARGUMENT, "null destination");
        DeviceGuard dg(s->device);
        prep(s, false);
        double* d_p = (double*)s->scratch.get(sizeof(double) << n, s->stream);
        launch_dm_diag(s->d, n, d_p, s->stream);
        QSIM_HIPCHK(hipMemcpyAsync(dst, d_p, sizeof(double) << n, hipMemcpyDeviceToHost, s->stream));
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_dm_init_pure(qsim_state* s, int n, const double* psi) {
    return guarded([&] {
        check_dm(s, n);
        QSIM_REQUIRE(psi, QSIM_ERR_INVALID_ARGUMENT, "null state");
        DeviceGuard dg(s->device);
        drop_layout(s);
        double2* d_psi = (double2*)s->scratch.get(sizeof(double2) << n, s->stream);
        QSIM_HIPCHK(hipMemcpyAsync(d_psi, psi, sizeof(double2) << n, hipMemcpyHostToDevice, s->stream));
        launch_dm_init(s->d, d_psi, n, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_dm_init_maximally_mixed(qsim_state* s, int n) {
    return guarded([&] {
        check_dm(s, n);
        DeviceGuard dg(s->device);
        drop_layout(s);
        launch_dm_init(s->d, nullptr, n, s->stream);
        QSIM_HIPCHK(hipStreamSynchronize(s->stream));
    });
}

int qsim_state_profile(qsim_state* s, int enable) {
    return guarded([&] {
        check_state(s);
        s->timer.enabled = enable != 0;
        s->timer.stream = s->stream;
    });
}

int qsim_state_profile_count(qsim_state* s, int* n) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        s->timer.resolve();
        *n = (int)s->timer.stats.size();
    });
}

int qsim_state_profile_get(qsim_state* s, int i, char* name, size_t name_len, double* total_ms,
                           int64_t* launches, double* alg_bytes) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        s->timer.resolve();
        if (i < 0 || i >= (int)s->timer.stats.size()) fail(QSIM_ERR_OUT_OF_RANGE, "bad index");
        const auto& st = s->timer.stats[i];
        if (name && name_len) {
            std::strncpy(name, st.name.c_str(), name_len - 1);
            name[name_len - 1] = 0;
        }
        if (total_ms) *total_ms = st.ms;
        if (launches) *launches = st.launches;
        if (alg_bytes) *alg_bytes = st.bytes;
    });
}

int qsim_state_profile_reset(qsim_state* s) {
    return guarded([&] {
        check_state(s);
        DeviceGuard dg(s->device);
        s->timer.reset();
    });
}

}  // extern "C"
