// engine.hpp — internal declarations shared by the HIP translation units of libqsim_hip.so.
//
// Nothing here crosses the C ABI (include/qsim_hip.h).  Host code lowers each reference
// GateOp (include/Circuit.hpp:64-84) to an `Op`: a (multi-)controlled 2x2 unitary on one
// target, a (multi-)controlled diagonal, or a SWAP.  The kernels only know those three kinds.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "qsim_hip.h"

namespace qsim_hip {

// ---------------------------------------------------------------------------------------
// Errors (mapped to QSIM_ERR_* at the ABI boundary)
// ---------------------------------------------------------------------------------------
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] inline void fail(int code, const std::string& m) { throw Error(code, m); }
// Thread-local message returned by qsim_last_error() (capi.hip).
void set_last_error(const char* msg);

#define QSIM_HIPCHK(call)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            ::qsim_hip::fail(QSIM_ERR_DEVICE, std::string("HIP error: ") +                  \
                                                  hipGetErrorString(e_) + " at " __FILE__ ":" + \
                                                  std::to_string(__LINE__));                \
    } while (0)

// ---------------------------------------------------------------------------------------
// Lowered operations
// ---------------------------------------------------------------------------------------
enum Kind : int { K_M1 = 0, K_DIAG = 1, K_SWAP = 2 };

// Sub-kinds select exact reference arithmetic where the reference kernel has a closed form
// (src/Gates.cu:31-175), so per-gate results are bitwise those formulas.
enum Sub : int {
    S_GEN = 0,  // general complex 2x2 / general diagonal
    S_X = 1,    // swap                                   (Gates.cu:31-44)
    S_Y = 2,    // (im1,-re1),(-im0,re0)                  (Gates.cu:46-63)
    S_H = 3,    // (a0+-a1)*0.7071067811865476            (Gates.cu:79-104)
    S_NEG = 4,  // d1 = -1   (Z, CZ)                      (Gates.cu:65-77, 283-296)
    S_I = 5,    // d1 = +i   (S)                          (Gates.cu:106-119)
    S_MI = 6,   // d1 = -i   (Sdag)                       (Gates.cu:143-155)
    S_T = 7,    // d1 = (1+i)/sqrt2  as (re-im, re+im)*c  (Gates.cu:121-141)
    S_TDG = 8   // d1 = (1-i)/sqrt2  as (re+im, im-re)*c  (Gates.cu:157-175)
};

constexpr double kInvSqrt2 = 0.7071067811865476;  // literal used by src/Gates.cu:88

struct Op {
    int kind = K_M1;
    int sub = S_GEN;
    int t0 = 0, t1 = -1;   // target (t1: second SWAP qubit)
    uint64_t cmask = 0;    // control qubits, all must read 1
    bool d0_one = false;   // DIAG: d0 == 1 exactly -> only the |1> half is touched
    double m[8] = {0};     // M1: a,b,c,d ; DIAG: d0,d1 (re,im interleaved)
    int src = -1;          // index of the circuit gate this op came from
    int ncontrols() const { return __builtin_popcountll(cmask); }
};

// Lower one reference gate (validated) to an Op.  Throws Error on bad input.
Op lower_gate(const qsim_gate& g, int n_qubits);
// Validate a gate against n qubits with the reference's rules (src/Circuit.cpp:16-55).
void validate_gate(const qsim_gate& g, int n_qubits);
// Algorithmic HBM bytes of one op over `amps` amplitudes.
double op_alg_bytes(const Op& op, double amps);
const char* gate_name(int type);

// ---------------------------------------------------------------------------------------
// Kernel launch interface (gates.hip)
// ---------------------------------------------------------------------------------------
struct Timer;  // per-launch HIP-event attribution (capi.hip)

// Apply one op to `batch` contiguous trajectories of 2^n amplitudes each.
void launch_op(double2* st, int n, uint64_t batch, const Op& op, hipStream_t s, Timer* tm);

// General 2^k x 2^k matrix (k <= 8) on `targets` (matrix-index bit j = targets[j]), d_mt the
// device copy of the transposed matrix, controlled on cmask.
void launch_matrixk(double2* st, int n, const int* targets, int k, const double2* d_mt,
                    uint64_t cmask, hipStream_t s, Timer* tm);
// General 4x4 on qubits (q0, q1) (m row-major over (b1 << 1) | b0, re/im interleaved), controlled.
void launch_matrix2q(double2* st, int n, int q0, int q1, const double* m, uint64_t cmask,
                     hipStream_t s, Timer* tm);

// Fused tile passes (fused.hip).
struct FusedPass {
    int single = -1;       // >= 0: not a tile pass but one per-gate op, Plan::singles[single]
    int h = 0;             // tile = 64 << h amplitudes (tile bits 0 .. 5 + h)
    int r0 = 6;            // tile bits 0 .. r0-1 are qubits 0 .. r0-1 (2^r0-amplitude HBM runs)
    int hpos[10] = {0};    // ascending physical qubits of tile bits r0 .. 5 + h (all >= r0)
    int rb = 4;            // staged: register bits per stage (threads per workgroup = 64 << h >> rb)
    int op_begin = 0, op_end = 0;  // range in the pass-op buffer (unstaged kernel)
    int stage_begin = 0, stage_end = 0;  // range in Plan::stages (staged kernel, h >= 4)
    int hu_count = 0;      // unnormalized H butterflies in the pass: store scales by 2^(-k/2)
    // Algorithmic HBM bytes per amplitude of the pass: min(32, sum of its gates' SURVEY §8(d)
    // bytes) — a pass of one CNOT is charged 16, not the 32 a full read+write would move.
    double alg_bpa = 32.0;
    // Relayout pass (plan_relayout, relayout.hip): the tile is loaded under this pass's layout
    // (r0 / hpos above) but stored under the next pass's: tile bit x goes to physical position
    // st_pos[x], tile-id bit i (the i-th non-tile position of the load layout, ascending) to
    // st_tid[i].  The last stage's lanes are the tile bits with the lowest store positions
    // (Stage::tmap), so the store still moves whole runs.
    int relayout = 0;
    int st_pos[13] = {0};
    int st_tid[32] = {0};
    int n_tid = 0;
};
struct TileOp {            // an Op re-expressed in tile-index bits
    int kind, sub, b0, b1;
    uint32_t cmask;
    int d0_one;
    int p0;                // staged kernel: register-bit position of the target (-1: thread bit)
    uint32_t cm_reg;       // staged kernel: controls among the stage bits, in register-bit space
    uint32_t cm_thr;       // staged kernel: controls among the other tile bits (tile space)
    // Pauli-frame fields (batched noisy runs, batched.hip): the op's circuit step, its target
    // qubit, and per control (<= 2) its qubit, register position in its stage (-1: thread bit)
    // and tile bit.
    int step, tq;
    int cq[2], cpos[2], cb[2];
    int _pad;
    // Tile-constant controls (tile_ctrl_out): physical positions outside the tile the op is
    // controlled on — the tile's non-tile bits are fixed, so the op runs on a whole tile or not
    // at all (a uniform branch on the tile's base address, no tile slot used).
    uint64_t cm_out;
    double m[8];
};
// A stage of a staged tile pass: every thread holds the 2^rb amplitudes spanned by `fix` (the
// stage's tile bits) in registers; ops in [op_begin, op_end) act on them with no LDS traffic.
// Register r of a stage holds tile element jb | offs(r), offs(r) = r spread over fix[].  Both
// address maps are XOR-linear in the element index, so their per-register parts are
// precomputed here and the kernel combines them with the thread part by one OR / XOR.
// LDS layout between two stages: element j lives at slot sigma(j) = j ^ sum_i parity(j & trow[i])
// << i (trow[i] only holds tile bits above i: triangular, so sigma is a bijection).  The planner
// picks trow per stage transition so that both the writes of the stage before (ds_write_b128:
// 8 groups of 8 lanes, slot mod 8) and the reads of the stage after (ds_read_b128: 4 groups of
// 16 lanes, slot mod 16) are bank-conflict-free (MI355X_MICROARCH.md §LDS); the fixed
// j ^ ((j >> 4) & 15) is 2-way conflicted whenever a stage's lanes span bits 0-3 and 4-7 unevenly.
struct Stage {
    uint64_t goff[16];     // HBM amplitude offset of offs(r) (its bits >= 6 spread over hpos)
    uint32_t lds[16];      // LDS byte offset 16 * sigma_in(offs(r)): this stage's reads
    uint32_t lds_w[16];    // LDS byte offset 16 * sigma_out(offs(r)): this stage's writes
    uint32_t trow_in[4], trow_out[4];  // the two layouts' sigma rows (see above)
    int fix[4];            // ascending stage tile bits
    int op_begin, op_end;
    // Thread bit i of the stage's element index jb sits at tile bit tmap[i] (the non-register
    // tile bits, ascending — the zero insertion at fix[] — except in the last stage of a
    // relayout pass, where they are ordered by store position).  tscatter != 0: use tmap.
    int tmap[10];
    int tscatter;
    int _pad;
};
// sigma of a layout (host and device)
__host__ __device__ __forceinline__ uint32_t lds_sigma(uint32_t j, const uint32_t* trow) {
    uint32_t s = j;
#pragma unroll
    for (int i = 0; i < 4; ++i) s ^= (uint32_t)(__builtin_popcount(j & trow[i]) & 1) << i;
    return s;
}
struct Plan {
    std::vector<FusedPass> passes;
    std::vector<TileOp> ops;
    std::vector<int> order;  // source gate index of each entry of `ops` (execution order)
    std::vector<Stage> stages;
    std::vector<Op> singles;  // ops run by the per-gate kernels (gate wider than the tile, n < 6)
    size_t fused_gate_count = 0;
    size_t tile_passes = 0;
};
constexpr int kTileHMax = 7;  // 64 << 7 = 8192 amplitudes = 128 KiB of LDS per workgroup
constexpr int kTileHDefault = 6;  // 12-qubit tiles unless QSIM_TILE_HMAX / qsim_set_tile_hmax
constexpr int kHposMax = 10;  // tile bits above the run: 6 + h - r0 <= 9
// Register bits per thread of a staged pass: 16 amplitudes per thread; 256 threads per workgroup
// up to h = 6, 512 at h = 7 (one 128 KiB workgroup per CU, the same 8 waves per CU).
constexpr int stage_rb(int h) { return h >= 6 ? 4 : h - 2; }
constexpr int stage_threads(int h) { return (64 << h) >> stage_rb(h); }
constexpr int kTileR0 = 6;    // contiguous run bits of a staged tile (QSIM_TILE_R0 in 4..6)
// hmax < 0: the process default (kTileHDefault, or QSIM_TILE_HMAX up to kTileHMax).
// avoid: qubits no tile may contain (ops never act on them; only tile padding is affected).
// avoid_first: the same for the plan's FIRST pass only (the sharded engine: the pivots of the
// remap before a step steer its leading pass, those of the remap after it every pass).
Plan plan_fused(const std::vector<Op>& ops, int n, int hmax = -1, uint64_t avoid = 0, uint64_t avoid_first = 0);
// Rebuild the last pass of `plan` (staged) as a relayout pass that stores load position p at
// tau[p] (a permutation of 0..n-1; the sharded engine's fused remap pack / unpack).
void relayout_last_pass(Plan& plan, int n, const int* tau);
// One tile pass appended to a plan (fused.hip; plan_fused and the relayout planner use it).
// bit_of[q] < 0: op qubit q is not a tile qubit (a tile-constant control); phys_of (null: the
// identity) gives such a control's physical position under the pass's load layout.
void append_tile_pass(Plan& plan, const std::vector<Op>& ops, int n, int h, int r0, const int* hpos,
                      const int* bit_of, const int* st_pos, const int* st_tid, const int* phys_of = nullptr);
// Tile-constant controls (QSIM_TILE_CTRL_OUT, default 1; qsim_set_tile_ctrl_out): a control
// qubit need not be a tile qubit — planners then only require an op's targets in the tile.
// Off for the calling thread inside a CtrlOutOff scope (batched Pauli-frame plans).
bool tile_ctrl_out();
void tile_ctrl_out_configure(int mode);
struct CtrlOutOff {
    CtrlOutOff();
    ~CtrlOutOff();
    CtrlOutOff(const CtrlOutOff&) = delete;
    CtrlOutOff& operator=(const CtrlOutOff&) = delete;
  private:
    bool prev_;
};
// Relayout plans (relayout.hip): every pass stores its tile under the next pass's layout, so
// each pass may choose all of its tile qubits except the four of the contiguous run, which come
// from the pass before (the last pass restores the first layout, so re-runs need no restore).
// `lower` maps the circuit through a logical -> physical permutation exactly as the caller will.
// Returns false when no relayout plan beats `max_passes` passes.
struct RelayoutChoice {
    std::vector<int> perm;  // the first (and last) layout, logical -> physical
    std::vector<Op> ops;    // the circuit lowered under perm
    Plan plan;
    double cost_us = 0.0;   // predicted (layout model)
};
bool plan_relayout(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                   size_t max_passes, RelayoutChoice& out);
// Up to QSIM_RELAYOUT_VARIANTS (default 3) closed tile sequences of the fewest passes, each with
// QSIM_RELAYOUT_LAYOUT_VARIANTS (default 2) position choices: relayout choices, best predicted first — the candidates a timed first run compares; memoised.
size_t plan_relayout_variants(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                              size_t max_passes, std::vector<RelayoutChoice>& out);
bool relayout_enabled(int n);  // QSIM_RELAYOUT (default 1), QSIM_RELAYOUT_MIN_QUBITS (default 20)
void relayout_configure(int mode, int min_qubits);  // qsim_set_relayout; < 0 leaves a setting
// A single gate-free relayout pass taking logical qubit q from physical perm[q] to q (n >= 12).
Plan plan_permutation_pass(int n, const std::vector<int>& perm);
bool relayout_forced();  // mode 2: a relayout plan whenever one exists (tests)
int tile_height_default();             // the h that hmax < 0 means (scope, setting, env, 6)
int tile_height_for(int n);            // a single-GPU state's height (the setting, or by size)
bool tile_height_is_set();             // qsim_set_tile_height or QSIM_TILE_HMAX in force
void tile_height_configure(int h);     // qsim_set_tile_height: h < 0 restores the env default
int tile_rb_default(int heff);         // register bits per stage of a staged pass of height heff
int tile_rb7();                        // register bits per stage of 13-qubit tiles (4, or 3)
void tile_rb7_configure(int rb);       // qsim_set_tile_rb7: 3 or 4; else back to QSIM_TILE_RB7
int tile_rb_for(int n, int h);         // a single-GPU state's stage width (-1: stage_rb(h))
// Plans made by this thread while the scope lives default to height h and, for 12-qubit tiles,
// rb register bits per stage (qsim_run of a state).
struct TileHeightScope {
    explicit TileHeightScope(int h, int rb = -1);
    ~TileHeightScope();
    TileHeightScope(const TileHeightScope&) = delete;
    TileHeightScope& operator=(const TileHeightScope&) = delete;
  private:
    int prev_, prev_rb_;
};
// Layout-aware qubit relabeling (relabel.hip): predicted cost of a tile (qubit mask) in
// microseconds, the tiles of a plan's staged passes, and the permutation (logical -> physical)
// minimising the predicted cost of `tiles` (empty: keep the identity, < min_gain better).
bool relabel_enabled(int n);                        // policy (QSIM_RELABEL*, qsim_set_relabel)
bool relabel_mode_on();  // the mode alone (QSIM_RELABEL / qsim_set_relabel != 0), whatever the size
void relabel_configure(int mode, int min_qubits);   // < 0 leaves a setting unchanged
double layout_cost_us(uint64_t tile);
std::vector<uint64_t> plan_tiles(const Plan& plan);
double plan_layout_cost_us(const Plan& plan);
std::vector<int> choose_relabel(const std::vector<uint64_t>& tiles, int n, double* before, double* after,
                                double min_gain = 0.03);
// The layout for a whole circuit: labels chosen for fewer passes first, then the cheapest pass
// layouts (relabel.hip).  perm empty: keep the identity.  ops / plan: the circuit under perm as
// the caller's `lower` produced it, and its plan (for the caller's plan cache).
struct LayoutChoice {
    std::vector<int> perm;
    std::vector<Op> ops;
    Plan plan;
    size_t passes_before = 0;
    double cost_before = 0.0, cost_after = 0.0;
    // want_alts > 0: the next acceptable candidates (same pass count), predicted-cost order
    struct Alt {
        std::vector<int> perm;
        std::vector<Op> ops;
        Plan plan;
    };
    std::vector<Alt> alts;
};
// stage_us > 0: the fewest-pass candidates are ranked by their plans' layout cost plus stage_us per
// register stage (density-matrix passes spend their time in their stages) instead of by the
// annealed layout cost alone.
LayoutChoice choose_layout(int n, const std::function<std::vector<Op>(const std::vector<int>&)>& lower,
                           int tries, size_t want_alts = 0, double stage_us = 0.0);
// QSIM_RELABEL_CALIBRATE (default 1) / QSIM_RELABEL_CALIBRATE_MIN_QUBITS (default 26): with
// inline compilation (QSIM_JIT=2) the first run of a basis state times the model's choice and
// its alternatives with their circuit-specialised kernels and keeps the fastest (capi.hip).
bool relabel_calibrate(int n);
void calibrate_configure(int mode, int min_qubits);  // negative: unchanged
bool calibrate_mode_on();  // the calibration mode alone (QSIM_RELABEL_CALIBRATE / qsim_set_calibrate)
int relabel_tries();  // QSIM_RELABEL_TRIES (default 7): random labelings planned per choice
// Process-wide memo of layout choices per circuit (kind: 0 state, 1 batched with its run flags).
// h != null / h >= 0: a decision that also chose the tile height (cross-height calibration).
// On-disk cache across processes (cache.hip; QSIM_CACHE=0 off, QSIM_CACHE_DIR): hipRTC code objects
// keyed by their source and options, layout decisions keyed like the in-process memo.
std::string cache_dir();
uint64_t cache_hash(const void* p, size_t n, uint64_t seed);
bool jit_cache_load(const std::string& src, const std::string& opts, std::vector<char>& code);
void jit_cache_store(const std::string& src, const std::string& opts, const std::vector<char>& code);
bool layout_cache_load(int n, int kind, const void* key, size_t bytes, std::vector<int>& perm, int* h);
void layout_cache_store(int n, int kind, const void* key, size_t bytes, int h, const std::vector<int>& perm);
bool layout_memo_get(int n, int kind, const void* gates, size_t bytes, std::vector<int>& perm, int* h = nullptr);
void layout_memo_put(int n, int kind, const void* gates, size_t bytes, const std::vector<int>& perm, int h = -1);
bool calibrate_heights(int n);  // QSIM_CALIBRATE_HEIGHTS (capi.hip: choose_first_layout)
// Factor on the predicted cost of a 13-qubit tile (QSIM_LAYOUT_T13, default 1); a scope sets it
// for the calling thread (and choose_layout hands it to its worker threads).
double layout_t13();
struct LayoutT13Scope {
    explicit LayoutT13Scope(double f);
    ~LayoutT13Scope();
    LayoutT13Scope(const LayoutT13Scope&) = delete;
    LayoutT13Scope& operator=(const LayoutT13Scope&) = delete;
  private:
    double prev_;
};
// Circuit-specialised pass kernels (jit.hip): hipRTC code object of one plan on one device.
struct JitJob;
struct JitModule {
    hipModule_t mod = nullptr;
    std::vector<hipFunction_t> fn;  // per plan pass; null = run by the interpreter
    ~JitModule();
};
struct JitState {
    std::shared_ptr<JitJob> job;
    std::unique_ptr<JitModule> mod;
    bool failed = false;
};
int jit_mode();        // 0 off, 1 background compile (default), 2 compile on first use
bool jit_pass_pipelined(const FusedPass& p);  // persistent software-pipelined pass kernel (jit.hip)
int jit_min_qubits();  // smaller states never JIT (QSIM_JIT_MIN_QUBITS, default 20)
void jit_configure(int mode, int min_qubits);  // < 0 leaves a setting unchanged
void jit_shutdown();  // stop the background compiler (queued jobs dropped, running one joined)
std::string jit_source(const Plan& plan);      // empty when the plan has no staged pass
bool jit_compile(const std::string& src, std::vector<char>& code, std::string& log);
// The loaded module for `plan`, or null while it compiles / when JIT does not apply.
const JitModule* jit_for(JitState& js, const Plan& plan, int n);

// The last few plans of one engine object (LRU): re-running a circuit (the benchmark loop,
// repeated trajectories, two circuits alternating on one state) skips the host planning and,
// once compiled, runs the specialised kernels.
struct PlanCache {
    struct Entry {
        int n = -1, h = -1;  // h: the tile height the plan was made for
        int ctrl_out = -1;   // tile_ctrl_out() when it was planned
        uint64_t avoid = 0, avoid_first = 0;
        std::vector<Op> key;
        Plan plan;
        JitState jit;
        uint64_t used = 0;
    };
    static constexpr size_t kEntries = 16;  // (first-run calibration keeps its candidates)
    std::vector<std::unique_ptr<Entry>> entries;
    uint64_t clock = 0;
    // stream: where the owner runs this cache's plans (drained before a plan is evicted)
    Entry& get(const std::vector<Op>& ops, int n_qubits, hipStream_t stream, uint64_t avoid = 0,
               uint64_t avoid_first = 0);
    // insert a plan computed elsewhere under `ops` (relabeling plans its candidates itself)
    void put(std::vector<Op> ops, int n_qubits, Plan plan, hipStream_t stream);
};
// Which part of a plan to launch: passes [first, last) over the sub-space whose qubits in
// fix_mask read fix_val (fix_mask = 0: the whole state).  Sub-space launches need staged passes.
struct FusedRange {
    size_t first = 0, last = SIZE_MAX;
    uint64_t fix_mask = 0, fix_val = 0;
    // relayout passes write out of place (a tile's store addresses are other tiles' load
    // addresses): they alternate between the state and `alt` (same size)
    double2* alt = nullptr;
};
// frames != null: batched noisy run under per-trajectory Pauli frames (FArgs::frames).
// Returns the buffer that holds the result (st, or range.alt after an odd number of relayout
// passes).
double2* launch_fused(double2* st, int n, uint64_t batch, const Plan& plan, const TileOp* d_ops,
                  const Stage* d_stages, hipStream_t s, Timer* tm, const JitModule* jm = nullptr,
                  const uint64_t* frames = nullptr, const FusedRange& range = FusedRange());

// Single-trajectory Monte-Carlo noise (noise.hip): one per-pair pass of channel `type`
// (reference NoiseType numbering) on `qubit`, uniforms from the hash of (seed, counter, pair);
// traj0: global trajectory index of trajectory 0 (the pair index hashed is the global one).
void launch_noise(double2* st, int n, int type, int qubit, double p, uint64_t seed,
                  uint64_t counter, hipStream_t s, Timer* tm, uint64_t batch = 1, uint64_t traj0 = 0);
// Every channel that follows one gate, passes counter, counter + 1, ... (counter is advanced):
// flip channels over a large batch run in one launch (work-group per unit of trajectories),
// otherwise one launch_noise per channel.  Same draws and results either way.
struct NoiseChan {
    int type, qubit;
    double p;
};
void launch_noise_after_gate(double2* st, int n, const std::vector<NoiseChan>& chans, uint64_t seed,
                             uint64_t& counter, hipStream_t s, Timer* tm, uint64_t batch, uint64_t traj0);
// Gate + in-tile noise (noise.hip): the gate and the prefix of `chans` whose qubits lie in its
// 4096-amplitude tile in one LDS pass, the rest by the push kernel; counter advances by
// chans.size().  Same states as launch_op + launch_noise_after_gate.  op == null: no gate.
bool gate_noise_tile_supported(int n, const Op* op);
void launch_gate_noise_step(double2* st, int n, uint64_t batch, uint64_t traj0, const Op* op,
                            const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t& counter, hipStream_t s,
                            Timer* tm);
// A whole run of gate steps (ops[i].kind < 0: no gate) through the tile kernel, each step's
// prefix flip lists built by k_gn_lists on L->ms (two sets, event-ordered) during the step before;
// L == null or gate_noise_lists_bytes == 0: the tile kernels walk the blocks themselves.  Every
// op must pass gate_noise_tile_supported.  counter advances by ops.size() x chans.size().
struct GnLists {
    void* buf[2];
    size_t set_bytes;  // of one set (>= gate_noise_lists_bytes)
    hipStream_t ms;
    hipEvent_t built[2], used[2], start;
};
size_t gate_noise_lists_bytes(int n, uint64_t batch, const std::vector<NoiseChan>& chans);
void launch_gate_noise_run(double2* st, int n, uint64_t batch, uint64_t traj0, const std::vector<Op>& ops,
                           const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t& counter, hipStream_t s,
                           Timer* tm, const GnLists* L);
// Pulled noise (noise.hip): the noise step after one gate (channels `chans`, passes counter0,
// counter0 + 1, ...; the push kernels' draws) applied by the NEXT gate's pass: dst = U (P src)
// out of place, op == null: the identity (the last step of a run).  words: >=
// pull_noise_codes_bytes (one code word per amplitude).  Supported when n >= 9, every channel
// flips (depolarizing / X / Y / Z) and at most 32 can fire; QSIM_NOISE_PULL=0 / 1 overrides the
// caller's default (NoisySimulator: on; BatchedSimulator: off — measured).
bool pull_noise_supported(int n, const std::vector<NoiseChan>& chans, bool default_on);
size_t pull_noise_codes_bytes(int n, uint64_t batch, size_t nch);
void launch_pull_noise_step(const double2* src, double2* dst, int n, uint64_t batch, uint64_t traj0,
                            const std::vector<NoiseChan>& chans, uint64_t seed, uint64_t counter0,
                            const Op* op, void* words, hipStream_t s, Timer* tm);
// Its two halves, for callers that build the next step's words on another stream while this
// step's pass runs (the map reads no amplitudes).
void launch_noise_map(int n, uint64_t batch, uint64_t traj0, const std::vector<NoiseChan>& chans, uint64_t seed,
                      uint64_t counter0, void* words, hipStream_t s, Timer* tm);
// next (optional): this pass also builds the NEXT step's code words (counter0: its first pass
// counter) — the word map fused into the pull pass (QSIM_NOISE_MAP_FUSED).
struct PullMapNext {
    uint64_t traj0, seed, counter0;
    void* words;
};
void launch_pull_gate(const double2* src, double2* dst, int n, uint64_t batch, const std::vector<NoiseChan>& chans,
                      const Op* op, const void* words, hipStream_t s, Timer* tm, const PullMapNext* next = nullptr);

// Density matrices as 2n-index-bit states (density.hip).
void dm_lower(int n, const qsim_gate* gates, size_t count, const qsim_noise_channel* ch,
              size_t nch, std::vector<Op>& out, bool reference_y = false);
void dm_lower_channel(int n, int type, int qubit, double p, std::vector<Op>& out);
void launch_dm_diag(const double2* rho, int n, double* out, hipStream_t s);
void launch_dm_init(double2* rho, const double2* psi, int n, hipStream_t s);

// Reductions / readout helpers (reduce.hip)
void launch_init_basis(double2* st, int n, uint64_t batch, uint64_t basis, hipStream_t s);
void launch_probabilities(const double2* st, uint64_t count, double* out, hipStream_t s);
// sum over |a_i|^2 for i with ((i >> bit) & 1) == 0 (bit < 0: all), deterministic 2-pass.
double reduce_norm(const double2* st, int n, int bit, double* d_partials, double* d_result,
                   hipStream_t s);
void launch_collapse(double2* st, int n, int bit, int result, double scale, hipStream_t s);
// max over the 2^n amplitudes of the larger per-component |a - b| (d_partials: >= 2048 doubles).
double reduce_max_abs_diff(const double2* a, const double2* b, int n, double* d_partials, double* d_result,
                           hipStream_t s);
struct Scratch;
void launch_histogram(const int64_t* d_idx, uint64_t count, uint64_t N, unsigned long long* d_hist,
                      hipStream_t s);
void sample_indices(const double2* st, int n, uint64_t batch, const double* uniforms, int shots,
                    int64_t* out, hipStream_t s, Scratch& scratch);
// Average of |a|^2 over `batch` trajectories into out[2^n] (device).
void launch_avg_probabilities(const double2* st, int n, uint64_t batch, double* out,
                              hipStream_t s);

// ---------------------------------------------------------------------------------------
// Timing (capi.hip): per-launch HIP events grouped by kernel name.
// ---------------------------------------------------------------------------------------
struct Timer {
    struct Pending { int slot; hipEvent_t a, b; double bytes; };
    struct Stat { std::string name; double ms = 0; int64_t launches = 0; double bytes = 0; };
    bool enabled = false;
    std::vector<Stat> stats;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    hipStream_t stream = nullptr;
    int slot_of(const char* name);
    void begin(const char* name, double bytes, hipEvent_t* a_out, int* slot_out);
    void end(int slot, hipEvent_t a, double bytes);
    // ext mode: two events for a launch to time itself; finish() queues them for resolve()
    void begin_ext(const char* name, hipEvent_t* a_out, hipEvent_t* b_out, int* slot_out);
    void finish(int slot, hipEvent_t a, hipEvent_t b, double bytes);
    void resolve();   // synchronizes on outstanding events
    void reset();
    ~Timer();
};
// Device copy of a small host descriptor array (fused plans).  Uploads only when the bytes
// change (a re-run of the same circuit re-uses the resident plan); the host shadow stays alive
// until the async copy that reads it has completed.
struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    std::vector<unsigned char> shadow;
    hipEvent_t copied = nullptr;
    void upload(const void* src, size_t bytes, hipStream_t s);
    ~DevBuf();
};

// Grow-only device scratch of one engine object (readback / sampling temporaries).  Every user
// synchronises its stream before returning, so the next user may reuse the memory; growing
// waits for the stream before the old block is freed.  (Plain hipMalloc memory: the
// stream-ordered pool is not used for buffers that pageable host copies read or write.)
struct Scratch {
    void* ptr = nullptr;
    size_t cap = 0;
    void* get(size_t bytes, hipStream_t s);
    ~Scratch();
};

// RAII scope used around each launch.  Record mode: events recorded on the stream before and
// after the launch (two marker packets, ~8 us of serialisation per launch — 35 % of a 20-qubit
// circuit).  Ext mode (ext = true): the two events are handed to the launch itself through
// start() / stop() (hipExtLaunchKernel / hipExtModuleLaunchKernel), which time the dispatch
// packet with no extra packets; the launch site must pass them.
struct TimedLaunch {
    Timer* tm; int slot = -1; hipEvent_t a = nullptr, b = nullptr; double bytes; bool ext = false;
    hipStream_t stream;  // the end event goes on the stream the begin event went on
    TimedLaunch(Timer* t, const char* name, double b, hipStream_t s, bool ext = false);
    hipEvent_t start() const { return a; }  // null when profiling is off
    hipEvent_t stop() const { return b; }
    ~TimedLaunch();
};

}  // namespace qsim_hip
