/*
 * qsim_hip.h — C ABI of the MI355X (gfx950) state-vector engine.
 *
 * This is the drop-in boundary between host code (the C++17 API in
 * include/qsim/ headers, the Python ctypes mirror, or any FFI) and the
 * hand-written HIP kernels.  Plain C types only: opaque handles, pointers,
 * sizes, int status codes.  No HIP, torch or C++ types cross it.
 *
 * Amplitude layout: 2^n interleaved {double re, double im} (16 B each),
 * index bit q == qubit q (LSB-first; reference src/Gates.cu:19-25 and
 * tests/test_gates.cu:258-273 pin this convention).
 *
 * Every entry point returns QSIM_OK (0) or a QSIM_ERR_* code; the message of
 * the last failure on the calling thread is in qsim_last_error().
 *
 * Reference interfaces replaced (file:line in rylanmalarchick/cuda-quantum-simulator):
 *   StateVector ctor/alloc/init      include/StateVector.cuh:66-86, src/StateVector.cu:130-202
 *   Gates.cuh __global__ kernels     include/Gates.cuh:58-101 (launched per gate)
 *   Simulator::run / applyGate       include/Simulator.hpp:53-85, src/Simulator.cu:28-154
 *   toHost / getProbabilities        src/StateVector.cu:204-233
 *   measure (prob + collapse)        src/StateVector.cu:260-314
 *   sample                           src/Simulator.cu:164-185, src/StateVector.cu:316-342
 *   OptimizedGates applyGate1Q_opt   include/OptimizedGates.cuh:91-93
 *   BatchedSimulator                 include/NoiseModel.cuh:231-297, src/NoiseModel.cu:653-972
 *   DensityMatrix(Simulator)         include/DensityMatrix.cuh:63-224, src/DensityMatrix.cu
 *   NoisySimulator noise kernels     include/NoiseModel.cuh:139-214, src/NoiseModel.cu:115-577
 */
#ifndef QSIM_HIP_H
#define QSIM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QSIM_ABI_VERSION 2

/* ---- status codes (mapped to the reference's exception types by the C++ layer) ---- */
enum {
    QSIM_OK = 0,
    QSIM_ERR_INVALID_ARGUMENT = 1, /* std::invalid_argument (src/StateVector.cu:135-141, :261-266) */
    QSIM_ERR_OUT_OF_RANGE = 2,     /* std::out_of_range (src/Circuit.cpp:26-31, src/NoiseModel.cu:917-919) */
    QSIM_ERR_RUNTIME = 3,          /* std::runtime_error (zero-probability measure, unknown gate) */
    QSIM_ERR_DEVICE = 4            /* std::runtime_error from a HIP/RCCL failure (CUDA_CHECK analogue) */
};

/* ---- gate types: numbering == reference enum class GateType (include/Circuit.hpp:42-59) ---- */
enum {
    QSIM_GATE_X = 0, QSIM_GATE_Y = 1, QSIM_GATE_Z = 2, QSIM_GATE_H = 3,
    QSIM_GATE_S = 4, QSIM_GATE_T = 5, QSIM_GATE_SDAG = 6, QSIM_GATE_TDAG = 7,
    QSIM_GATE_RX = 8, QSIM_GATE_RY = 9, QSIM_GATE_RZ = 10,
    QSIM_GATE_CNOT = 11, QSIM_GATE_CZ = 12, QSIM_GATE_CRY = 13, QSIM_GATE_CRZ = 14,
    QSIM_GATE_SWAP = 15, QSIM_GATE_TOFFOLI = 16,
    QSIM_GATE_COUNT = 17
};

/* One circuit operation, same meaning as the reference GateOp (include/Circuit.hpp:64-84):
 * qubits = [target] | [control, target] | [q1, q2] (SWAP) | [c1, c2, target]. */
typedef struct qsim_gate {
    int32_t type;      /* QSIM_GATE_* */
    int32_t nqubits;   /* 1, 2 or 3 */
    int32_t qubits[3];
    int32_t _pad;
    double  parameter; /* angle in radians for Rx/Ry/Rz/CRY/CRZ, else ignored */
} qsim_gate;

/* Execution flags for qsim_run / qsim_batch_run. */
enum {
    QSIM_RUN_PER_GATE = 0,   /* one kernel launch per gate (reference Simulator::run shape) */
    QSIM_RUN_FUSED = 1       /* host planner groups gates into LDS-tiled fused passes */
};

typedef struct qsim_state qsim_state; /* one 2^n state vector on one GPU + its HIP stream */
typedef struct qsim_batch qsim_batch; /* B trajectories of 2^n amplitudes (BatchedSimulator) */

/* ---- library ---- */
const char* qsim_last_error(void);
int qsim_abi_version(void);
int qsim_device_count(int* count);
/* Device of the calling thread's next objects (hipSetDevice; the reference always uses the
 * default device).  One process per GPU selects its LOCAL_RANK with this. */
int qsim_set_device(int device);
/* Name/bandwidth facts of the current device (for bench reports). name_len includes NUL. */
int qsim_device_info(int device, char* name, size_t name_len, int* cu_count, size_t* total_mem);

/* ---- state vector lifecycle (StateVector.cuh:66-86) ---- */
/* 1 <= n_qubits <= QSIM_MAX_QUBITS_SINGLE (30, Constants.hpp:68), else QSIM_ERR_INVALID_ARGUMENT.
 * The new state is |0...0> (src/StateVector.cu:130-143). */
int qsim_state_create(int n_qubits, qsim_state** out);
int qsim_state_create_on(int device, int n_qubits, qsim_state** out);
int qsim_state_destroy(qsim_state* s);
int qsim_state_num_qubits(const qsim_state* s, int* n);
/* Raw device address of amplitude 0 (StateVector::devicePtr, StateVector.cuh:89-90). */
int qsim_state_device_ptr(qsim_state* s, void** dptr);
/* hipStream_t of the state, as an opaque pointer. */
int qsim_state_stream(qsim_state* s, void** stream);
int qsim_state_init_zero(qsim_state* s);                      /* initializeZero */
int qsim_state_init_basis(qsim_state* s, uint64_t basis_idx);  /* initializeBasis; >= 2^n -> INVALID_ARGUMENT */
int qsim_state_sync(qsim_state* s);

/* ---- gate application ---- */
/* Validate + apply one gate (Simulator::applyGate, src/Simulator.cu:38-46).  Asynchronous. */
int qsim_apply_gate(qsim_state* s, const qsim_gate* g);
/* Whole circuit (Simulator::run, src/Simulator.cu:28-36).  flags = QSIM_RUN_*.  Asynchronous. */
int qsim_run(qsim_state* s, const qsim_gate* gates, size_t count, int flags);
/* General 2x2 unitary [[a,b],[c,d]] on `target`, m = {a.re,a.im,b.re,b.im,c.re,c.im,d.re,d.im}
 * (applyGate1Q_opt, include/OptimizedGates.cuh:91-93), optionally controlled on `controls`. */
int qsim_apply_matrix1q(qsim_state* s, int target, const double m[8],
                        const int* controls, int n_controls);
/* General 4x4 matrix on (q0, q1), m = 32 doubles, row-major over the index (bit q1 << 1) | bit q0,
 * optionally controlled (the k = 2 applyMatrix of SURVEY §8(f) rank 3).  Asynchronous. */
int qsim_apply_matrix2q(qsim_state* s, int q0, int q1, const double m[32], const int* controls,
                        int n_controls);
/* General 2^k x 2^k complex matrix on k <= 8 target qubits (generalises
 * applyGate1Q_opt, src/OptimizedGates.cu:165-183, and cuStateVec's applyMatrix used by
 * benchmarks/benchmark_custatevec.cu:131-135): m row-major, re/im interleaved, matrix-index bit j
 * = bit targets[j] of the amplitude index; applied on the control == 1 subspace of `controls`.
 * Asynchronous; synchronises before returning (the matrix is staged in device scratch). */
int qsim_apply_matrix(qsim_state* s, const int* targets, int k, const double* m,
                      const int* controls, int n_controls);
/* Named dispatchers of the reference (src/OptimizedGates.cu:388-413, declared in
 * include/OptimizedGates.cuh:161-166) on a raw device pointer and stream, routed to this build's
 * per-gate kernels; applyGate1Q_opt's general 2x2 as qsim_apply_matrix1q_raw. */
int qsim_apply_hadamard_optimized(void* dstate, int n_qubits, int target, void* stream);
int qsim_apply_cnot_optimized(void* dstate, int n_qubits, int control, int target, void* stream);
int qsim_apply_matrix1q_raw(void* dstate, int n_qubits, int target, const double m[8], void* stream);
/* applyFusedSingleQubitLayer (src/OptimizedGates.cu:344-382): for every qubit q in `active`,
 * amplitudes with bit q = 0 are scaled by gate_params[q*4+0] and those with bit q = 1 by
 * gate_params[q*4+3] (complex, re/im interleaved: 8 doubles per qubit).  Runs as fused passes. */
int qsim_apply_diagonal_layer(qsim_state* s, const double* gate_params, uint64_t active);
/* Host-only introspection of the fused-pass planner (no device needed).  Writes, for each gate
 * in execution order, its index in `gates` (order[count]) and its pass number (pass_of[count],
 * -1 for gates executed per-gate), and the number of passes.  Gates are only reordered past
 * gates on disjoint qubits. */
int qsim_plan_fused(int n_qubits, const qsim_gate* gates, size_t count, int hmax,
                    int32_t* order, int32_t* pass_of, int32_t* n_passes);
/* Circuit-specialised pass kernels (hipRTC, no reference counterpart: the reference launches one
 * fixed kernel per gate, src/Simulator.cu:38-154).  mode 0 = off, 1 = compile in the background
 * on a plan's first run and switch to the compiled kernels when ready (default), 2 = compile on
 * the first run before launching; states below min_qubits always use the pass interpreter.
 * A negative argument leaves that setting unchanged (env defaults: QSIM_JIT, QSIM_JIT_MIN_QUBITS). */
int qsim_set_jit(int mode, int min_qubits);
/* Stop the background compiler: queued compiles are dropped (their plans stay on the
 * interpreter) and the one in progress is waited for.  Called at exit (the Python package
 * registers it with atexit; the library registers it after its first compile) so no compile runs
 * while the compiler's static state is destroyed; later background requests are refused. */
int qsim_jit_shutdown(void);
/* Layout-aware qubit relabeling (no reference counterpart; relabel.hip).  A fused pass's speed
 * depends on the physical qubit positions its tile spans (the memory system's address mapping).
 * On the first fused qsim_run of a state that holds a computational basis state (after create /
 * init), the engine may choose a logical -> physical qubit permutation for the circuit's plan and
 * keep running the state under it; every entry that reads or writes amplitudes by index first
 * restores the identity layout with a fused SWAP network, so results are unchanged.  mode 0 off,
 * 1 on (default, QSIM_RELABEL); states below min_qubits (default 26, QSIM_RELABEL_MIN_QUBITS)
 * are never relabeled; negative arguments leave a setting unchanged. */
int qsim_set_relabel(int mode, int min_qubits);
int qsim_state_perm(qsim_state* s, int32_t* perm);  /* current logical -> physical map, n entries */
/* First-run layout decision of a state (no reference counterpart): the tile height its fused
 * runs plan at, whether the layout was chosen by timing candidates on the device (layout and
 * cross-height calibration), whether the qubits are currently relabeled. */
int qsim_state_layout_info(qsim_state* s, int* tile_h, int* calibrated, int* relabeled);
/* Bring a relabeled state back to the identity qubit layout now (the fused SWAP network every
 * index-based reader runs first); a no-op when it is not relabeled. */
int qsim_state_restore_layout(qsim_state* s);
/* Whether the state's first fused run chose a relayout plan (no reference counterpart): every
 * 12-qubit tile pass stores its tile under the next pass's qubit layout, so each pass picks all
 * of its tile qubits except the four of the contiguous run (fewer passes); the last pass restores
 * the first layout.  QSIM_RELAYOUT=0 disables them (QSIM_RELAYOUT_MIN_QUBITS, default 20).
 * Relayout passes write out of place into a second 2^n buffer: a first run only considers them
 * when the device has room for it (otherwise the fixed-layout plan runs in place), and the buffer
 * is freed again unless the run keeps a relayout plan (qsim_state_memory_bytes). */
int qsim_state_relayout(qsim_state* s, int* relayout);
/* Relayout plans on (mode 1: when they need fewer passes, or win the device timing with
 * calibration) / off (0) / forced (2: whenever one exists — tests) for first runs from now on, for
 * states of at least min_qubits qubits; they permute qubit labels, so relabeling mode 0
 * (qsim_set_relabel / QSIM_RELABEL=0) turns them off too, whatever the state's size; negative
 * arguments leave a setting unchanged. */
int qsim_set_relayout(int mode, int min_qubits);
/* Host-only: compile the relayout plan's pass kernels with hipRTC for gfx950 (no GPU needed);
 * code_bytes: the code object's size.  QSIM_ERR_RUNTIME when there is no relayout plan. */
int qsim_jit_build_relayout(int n_qubits, const qsim_gate* gates, size_t count, size_t* code_bytes);
/* Host-only check of the planners' index math (tests; no GPU): plan the circuit (mode 0: the
 * fixed-layout planner under the identity labels; 1: the relayout planner) and execute the plan
 * on the host exactly as the staged pass kernels address the state (register stages, LDS slots,
 * store layouts).  amps: 2^n interleaved re/im in logical qubit order, updated in place.
 * perm (n entries, may be null): the layout the plan starts and ends in (logical -> physical);
 * passes: the plan's pass count.  QSIM_ERR_RUNTIME when mode 1 finds no relayout plan.
 * mode 2: the one-pass identity-layout restore instead (gates unused): amps holds the state in
 * the physical order of layout perm (input), and is returned in logical order. */
int qsim_plan_exec_host(int n_qubits, const qsim_gate* gates, size_t count, int mode, double* amps,
                        int32_t* perm, int* passes);
/* Host-only: the relayout plan of a circuit (what qsim_run would consider): its first/last layout
 * (perm, n entries, may be null), pass count and predicted time in microseconds (layout model);
 * *passes = 0 when none exists. */
int qsim_plan_relayout(int n_qubits, const qsim_gate* gates, size_t count, int32_t* perm, int* passes,
                       double* predicted_us);
/* Layout calibration (with QSIM_JIT = 2, from min_qubits; defaults QSIM_RELABEL_CALIBRATE = 1,
 * QSIM_RELABEL_CALIBRATE_MIN_QUBITS = 26): the first run of a basis state times the layout
 * model's choice and two alternatives with their compiled pass kernels (the basis state is
 * restored after each) and keeps the fastest.  Negative arguments leave a setting unchanged. */
int qsim_set_calibrate(int mode, int min_qubits);
/* Tile height of fused passes planned from now on (no reference counterpart): a tile spans 6 + h
 * qubits (64 << h amplitudes in LDS).  h = 6 (12 qubits, 64 KiB, two workgroups per CU) is the
 * default; h = 7 (13 qubits, 128 KiB, one 512-thread workgroup per CU, persistent pipelined
 * kernels) needs fewer passes on some circuits but streams slower.  h < 0 restores
 * the default (QSIM_TILE_HMAX); plans already cached for a circuit keep their height. */
int qsim_set_tile_height(int h);
/* Tile-constant controls (no reference counterpart; default on, QSIM_TILE_CTRL_OUT): the fused
 * planners require only an op's TARGETS to be tile qubits; a control outside the tile is fixed for
 * the whole tile, so the op runs on the tiles where it reads 1 (a uniform branch on the tile's
 * base address) — a CNOT costs one tile slot, not two.  mode 0 off, 1 on, negative: unchanged;
 * plans made from now on.  Batched Pauli-frame passes always keep every control a tile qubit. */
int qsim_set_tile_ctrl_out(int mode);
/* Register bits per stage of 13-qubit tiles: 4 (16 amplitudes per thread, 512-thread workgroups,
 * the default) or 3 (8 per thread, 1024 threads); anything else restores QSIM_TILE_RB7. */
int qsim_set_tile_rb7(int rb);
/* Host-only: the permutation the engine would choose for this circuit (identity when none pays)
 * and the predicted pass-layout cost (microseconds, summed over the plan's passes) before/after. */
int qsim_plan_relabel(int n_qubits, const qsim_gate* gates, size_t count, int32_t* perm,
                      double* cost_before_us, double* cost_after_us);
/* Host-only: the generated source of a circuit's plan (len = its size; buf gets up to cap-1
 * bytes + NUL), and a hipRTC compile of it for gfx950 (code_bytes = code-object size). */
int qsim_jit_source(int n_qubits, const qsim_gate* gates, size_t count, char* buf, size_t cap,
                    size_t* len);
int qsim_jit_build(int n_qubits, const qsim_gate* gates, size_t count, size_t* code_bytes);
/* Kernel-level entry on a raw device pointer (the reference's Gates.cuh kernels, launched by
 * tests/test_statevector.cu:151-159).  stream may be NULL (the null stream). */
int qsim_apply_gate_raw(void* dstate, int n_qubits, const qsim_gate* g, void* stream);

/* ---- readout (each synchronizes the state's stream) ---- */
int qsim_state_to_host(qsim_state* s, double* dst);            /* 2*2^n doubles */
int qsim_state_from_host(qsim_state* s, const double* src);    /* 2*2^n doubles */
int qsim_state_probabilities(qsim_state* s, double* dst);      /* 2^n doubles, |a_i|^2 */
int qsim_state_total_probability(qsim_state* s, double* out);  /* device wave64 reduction */
/* P(index bit `bit` == 0), device reduction (qubitProbabilityKernel src/StateVector.cu:83-99
 * + host sum :280-287).  `bit` is an index bit: the C++ layer maps the reference's
 * big-endian measure(q) to bit n-1-q. */
int qsim_state_prob_bit_zero(qsim_state* s, int bit, double* out);
/* Zero amplitudes whose `bit` != result, scale the rest (collapseStateKernel :105-124). */
int qsim_state_collapse(qsim_state* s, int bit, int result, double scale);
/* Draw `shots` basis indices from |a|^2 with uniforms u[i] in [0,1) supplied by the caller
 * (host RNG keeps the reference's mt19937 stream): device CDF + binary search. */
int qsim_state_sample(qsim_state* s, const double* uniforms, int shots, int64_t* out);
/* max_i max(|Re a_i - Re b_i|, |Im a_i - Im b_i|) of two states of the same size on the same
 * device, both read in the identity qubit layout, computed on the device (no reference
 * counterpart: tests/test_gpu_cpu_equivalence.cu:26 compares per component on the host, which at
 * 30 qubits would copy 32 GiB).  NaN when any difference is NaN. */
int qsim_state_max_abs_diff(qsim_state* a, qsim_state* b, double* out);
/* Device bytes the state owns now: the 2^n x 16 B amplitudes, the second buffer a relayout plan
 * writes into (same size; allocated on a first run only when the device has room for it, freed
 * when the run does not keep a relayout plan), reduction and plan buffers, readout scratch. */
int qsim_state_memory_bytes(qsim_state* s, uint64_t* bytes);

/* ---- timing (bench / profiling) ---- */
/* Enable per-launch HIP-event timing on the state's stream; kernels are attributed by name. */
int qsim_state_profile(qsim_state* s, int enable);
/* Number of distinct kernel names timed so far, and per-name stats (ms totals, launch counts). */
int qsim_state_profile_count(qsim_state* s, int* n);
int qsim_state_profile_get(qsim_state* s, int i, char* name, size_t name_len,
                           double* total_ms, int64_t* launches, double* alg_bytes);
int qsim_state_profile_reset(qsim_state* s);
/* Introspection of the last fused qsim_run on this state: tile passes planned and how many ran
 * as circuit-specialised (hipRTC) kernels rather than the pass interpreter. */
int qsim_state_last_run(qsim_state* s, int* passes, int* jit_passes);

/* ---- batched trajectories (BatchedSimulator, include/NoiseModel.cuh:231-297) ---- */
/* Noise channel on one qubit, NoiseType numbering == reference enum (NoiseModel.cuh:49-56). */
typedef struct qsim_noise_channel {
    int32_t type;   /* 0 Depolarizing, 1 AmplitudeDamping, 2 PhaseDamping, 3 BitFlip, 4 PhaseFlip, 5 BitPhaseFlip */
    int32_t qubit;
    double  probability;
} qsim_noise_channel;

int qsim_batch_create(int n_qubits, int batch_size, qsim_batch** out);
int qsim_batch_destroy(qsim_batch* b);
int qsim_batch_reset(qsim_batch* b);
int qsim_batch_set_seed(qsim_batch* b, uint64_t seed);
/* Trajectory sharding (SURVEY §8(e) "BatchedSimulator shards trivially by trajectory"; no
 * reference counterpart — the reference runs every trajectory on one GPU): this object's B
 * trajectories are trajectories [first, first + B) of a larger ensemble.  Noise draws are keyed
 * by the global trajectory index (both noise processes), so G objects with offsets 0, B, 2B, ...
 * and the same seed hold exactly the trajectories one object of G*B trajectories would. */
int qsim_batch_set_trajectory_offset(qsim_batch* b, uint64_t first);
/* Apply the circuit to every trajectory; after each gate apply every channel (reference
 * BatchedSimulator::run, src/NoiseModel.cu:815-831).  Gate semantics follow
 * src/NoiseModel.cu:717-801 when flags has QSIM_BATCH_REFERENCE_GATESET, else the full gate set.
 * For n >= 10 the gates run as fused tile passes with the noise carried as per-trajectory Pauli
 * frames (same draws, same trajectories); QSIM_BATCH_PER_GATE forces one kernel per gate plus
 * one Pauli pass per noisy step (the reference's structure). */
enum { QSIM_BATCH_FULL_GATESET = 0, QSIM_BATCH_REFERENCE_GATESET = 1, QSIM_BATCH_PER_GATE = 2,
       QSIM_BATCH_REFERENCE_NOISE = 4 };
/* QSIM_BATCH_REFERENCE_NOISE: the reference's noise process instead of the physical channel —
 * after every gate, one pass per Depolarizing channel entry (other types are ignored, as the
 * reference's batched mode does) over all B x 2^(n-1) amplitude pairs; each pair draws its own
 * uniform (float, compared with the double probability) and below p picks X/Y/Z at float
 * thresholds 1/3, 2/3 with a second draw, applied to that pair only
 * (applyBatchedDepolarizingKernel, src/NoiseModel.cu:834-892).  The draws come from the counter
 * hash of qsim_noise_apply keyed by (seed, pass counter, global pair index t*2^(n-1) + pair). */
int qsim_batch_run(qsim_batch* b, const qsim_gate* gates, size_t count,
                   const qsim_noise_channel* channels, size_t n_channels, int flags);
int qsim_batch_avg_probabilities(qsim_batch* b, double* dst);           /* 2^n */
int qsim_batch_traj_probabilities(qsim_batch* b, int traj, double* dst);  /* 2^n */
int qsim_batch_traj_state(qsim_batch* b, int traj, double* dst);          /* 2*2^n */
/* BatchedSimulator::sample (src/NoiseModel.cu:938-957) on the device: uniforms and out are
 * trajectory-major, B x shots (shot s of trajectory t at t*shots + s — the reference's draw
 * order); out = lower_bound of the uniform over the trajectory's CDF, 2^n when past its end. */
int qsim_batch_sample(qsim_batch* b, const double* uniforms, int shots, int64_t* out);
/* BatchedSimulator::getHistogram (src/NoiseModel.cu:959-972): counts of the sampled outcomes
 * over every trajectory and shot, out-of-range outcomes skipped; hist has 2^n entries. */
int qsim_batch_histogram(qsim_batch* b, const double* uniforms, int shots, int64_t* hist);
int qsim_batch_device_ptr(qsim_batch* b, void** dptr);
int qsim_batch_sync(qsim_batch* b);
/* Last fused batched run: tile passes and how many ran as circuit-specialised kernels. */
int qsim_batch_last_run(qsim_batch* b, int* passes, int* jit_passes);
int qsim_batch_profile(qsim_batch* b, int enable);
int qsim_batch_profile_count(qsim_batch* b, int* n);
int qsim_batch_profile_get(qsim_batch* b, int i, char* name, size_t name_len,
                           double* total_ms, int64_t* launches, double* alg_bytes);

/* ---- single-trajectory Monte-Carlo noise (NoisySimulator, include/NoiseModel.cuh:139-214) ----
 * One noise pass on `qubit` with the reference kernels' per-pair semantics
 * (applyBitFlipKernel ... applyPhaseDampingKernel, src/NoiseModel.cu:115-314): every amplitude
 * pair draws from a counter hash of (seed, counter, pair index).  Asynchronous. */
int qsim_noise_apply(qsim_state* s, int type, int qubit, double probability, uint64_t seed,
                     uint64_t counter);
/* Flips applied so far by range-checked noise launches (QSIM_NOISE_CHECK=1: the one-launch
 * reference noise kernel counts every access outside its work-group's pairs on the device and
 * fails the call if there is one; tests read this to see the check had work to do). */
int qsim_noise_check_flips(uint64_t* flips);
/* Tests: `draws` geometric gaps of a flip channel of probability p (keyed by `key`) taken the
 * engine's way (single precision first, the double log where that cannot decide) against
 * floor(ln u / ln(1 - P)) in double, both capped at one 256-pair block (a walk only needs to know
 * a gap is past its block): *mismatches (0 expected) and *fallbacks. */
int qsim_noise_gap_check(double p, uint64_t draws, uint64_t key, uint64_t* mismatches, uint64_t* fallbacks);
/* On-disk cache across processes of the first-run costs (no reference counterpart: the reference
 * compiles its kernels ahead of time and does no layout search): circuit-specialised pass kernels
 * (hipRTC code objects) and layout decisions, in QSIM_CACHE_DIR (default $XDG_CACHE_HOME/qsim_amd
 * or $HOME/.cache/qsim_amd; QSIM_CACHE=0 off).  Counters of this process: entries loaded / written. */
int qsim_cache_stats(uint64_t* jit_hits, uint64_t* jit_stores, uint64_t* layout_hits, uint64_t* layout_stores);
/* Tests: the same comparison on TARGETED draws — for every gap boundary m in [0, 256] (u_m =
 * exp(m ln(1 - P))) and both ends of the interval of doubles that round to the float nearest u_m,
 * 2 x half consecutive u values around each; *draws = how many were checked. */
int qsim_noise_gap_check_edges(double p, uint64_t half, uint64_t* mismatches, uint64_t* fallbacks,
                               uint64_t* draws);
/* NoisySimulator::run (src/NoiseModel.cu:369-382): each gate, then every channel entry in order,
 * one noise pass each; *counter advances by one per pass.  With no channel entries the circuit
 * runs as fused passes (flags = QSIM_RUN_*), else one kernel per gate (the noise interleaves). */
int qsim_noisy_run(qsim_state* s, const qsim_gate* gates, size_t count,
                   const qsim_noise_channel* channels, size_t n_channels, uint64_t seed,
                   uint64_t* counter, int flags);

/* ---- density matrices (DensityMatrix / DensityMatrixSimulator, include/DensityMatrix.cuh:63-224)
 * rho of n qubits (1 <= n <= QSIM_DM_MAX_QUBITS) lives in a qsim_state created with 2n qubits:
 * amplitude k = i * 2^n + j holds rho[i][j] (the reference's row-major layout,
 * src/DensityMatrix.cu:29-30); purity = qsim_state_total_probability, the matrix =
 * qsim_state_to_host, measurement collapse = qsim_state_collapse on bits q + n and q. */
#define QSIM_DM_MAX_QUBITS 15
/* DensityMatrixSimulator::run (src/DensityMatrix.cu:201-212): each gate as U rho U^dag, then for
 * each of its qubits every channel entry on that qubit or with qubit = -1 (a global channel).
 * CRY/CRZ/Toffoli -> QSIM_ERR_RUNTIME (:264-266).  flags = QSIM_RUN_* | QSIM_DM_REFERENCE_Y.
 * Asynchronous. */
/* QSIM_DM_REFERENCE_Y: Y acts as the reference's dmApplyY, rho -> -Y rho Y^dag
 * (src/DensityMatrix.cu:507-546: its phases are those of Y rho Y^dag times -1, so the trace
 * changes sign); default: Y rho Y^dag. */
#define QSIM_DM_REFERENCE_Y 8
int qsim_dm_run(qsim_state* rho, int n_qubits, const qsim_gate* gates, size_t count,
                const qsim_noise_channel* channels, size_t n_channels, int flags);
/* Host-only: the fused plan qsim_dm_run (QSIM_RUN_FUSED) would run for this circuit, four ints
 * per pass: tile height h (tile = 64 << h elements; -1: a per-gate step), ops, register stages,
 * contiguous run bits r0.  With QSIM_DM_PLAN_RELABELED in flags: the plan under the index-bit
 * labels a first run on |0><0| chooses. */
#define QSIM_DM_PLAN_RELABELED 0x100
int qsim_dm_plan_info(int n_qubits, const qsim_gate* gates, size_t count, const qsim_noise_channel* channels,
                      size_t n_channels, int flags, int32_t* info, size_t cap, size_t* n_passes);
/* Host-only: the circuit-specialised kernel source of that plan (as qsim_jit_source). */
int qsim_dm_jit_source(int n_qubits, const qsim_gate* gates, size_t count, const qsim_noise_channel* channels,
                       size_t n_channels, int flags, char* buf, size_t cap, size_t* len);
/* One channel (applyDepolarizing ... applyBitPhaseFlip, :298-356) on `qubit`. */
int qsim_dm_apply_channel(qsim_state* rho, int n_qubits, int type, int qubit, double p);
int qsim_dm_diagonal(qsim_state* rho, int n_qubits, double* dst);          /* 2^n: Re rho_ii */
int qsim_dm_init_pure(qsim_state* rho, int n_qubits, const double* psi);   /* rho = |psi><psi| */
int qsim_dm_init_maximally_mixed(qsim_state* rho, int n_qubits);          /* rho = I / 2^n */

/* ---- multi-GPU: state sharded by its high physical qubits, one process per GPU, RCCL ----
 * (the reference is single-GPU, README.md:361-367).  World size W = 2^g ranks;
 * rank r holds the 2^(n-g) amplitudes whose top g PHYSICAL index bits equal r.  A logical->
 * physical qubit map is kept on every rank: SWAP gates only relabel it, gates whose target sits
 * on a global (rank) bit trigger an all-to-all qubit remap over RCCL. */
typedef struct qsim_dist qsim_dist;
#define QSIM_DIST_UNIQUE_ID_BYTES 128
#define QSIM_MAX_QUBITS_DIST 36
/* Lowered operation record (host planner output, see qsim_dist_plan). kind: 0 controlled 2x2
 * (m = a,b,c,d), 1 controlled diagonal (m = d0,d1), 2 swap(t0,t1); qubits are PHYSICAL local
 * positions of the rank the plan was made for. */
typedef struct qsim_op {
    int32_t kind, sub, t0, t1;
    uint64_t cmask;
    int32_t d0_one, src;
    double m[8];
} qsim_op;
/* One plan step: kind 0 = ops[op_begin, op_end) on the local shard; kind 1 = exchange that
 * swaps global physical positions gpos[i] with local positions lpos[i], i < k.  Overlapped
 * remaps: an exchange with pivots (pmask != 0: up to 4 local physical positions; pivot = the
 * lowest, -1 if none) runs as 2^m part-exchanges, one per value of the pivot bits.  An ops step
 * with role bit 1 runs the trailing passes of its fused plan that avoid the pivots of the
 * exchange after it per part (each part's transfer then overlaps the later parts' passes); role
 * bit 2: its leading passes that avoid the pivots of the exchange before it run per part as each
 * part lands.  The step is planned as one fused plan either way (ops steps report pivot -1). */
typedef struct qsim_dist_step {
    int32_t kind, k;
    int32_t op_begin, op_end;
    int32_t gpos[8], lpos[8];
    int32_t pivot, role;
    uint64_t pmask;
    uint64_t coarse; /* exchange: pivots the step before's coarse passes leave untouched (0: none) */
} qsim_dist_step;

int qsim_dist_unique_id(void* id_out);  /* ncclGetUniqueId, on rank 0 */
int qsim_dist_create(int n_qubits, int rank, int world, const void* unique_id, int device,
                     qsim_dist** out);
/* Virtual ranks: all `world` shards in this process on one GPU, exchanged by device copies
 * (same planner and pack/unpack kernels, no RCCL) — for testing the sharded path on one GPU. */
int qsim_dist_create_virtual(int n_qubits, int world, int device, qsim_dist** out);
/* Attach a world-1 RCCL communicator (unique id from qsim_dist_unique_id) to a virtual object:
 * its slab moves then run as ncclSend / ncclRecv pairs to rank 0 itself in the same groups, and
 * its all-reduces through RCCL — the multi-rank call sequence (non-blocking init, groups,
 * settle, watchdog) on one GPU (tests). */
int qsim_dist_virtual_rccl(qsim_dist* d, const void* unique_id);
/* Exchanges of the last qsim_dist_run (summed over this process's shards) whose pack and unpack
 * ran inside the local passes: the last pass before the remap stored its tiles straight into the
 * send buffer's slab layout and the step after it planned in that layout, loading from the receive
 * buffer, its last pass storing back to the standard positions (no k_exchange_copy). */
int qsim_dist_fused_remaps(qsim_dist* d, int* remaps);
/* Host-staged transport (no RCCL): one shard per process like qsim_dist_create, but every
 * point-to-point transfer is handed to `fn` as host buffers.  A post sends `bytes` from `send` to
 * rank `peer` and receives `bytes` from `peer` into `recv` (either may be NULL for a one-sided
 * post); posts pair up as grouped ncclSend / ncclRecv do: the k-th post of rank r naming q
 * with the k-th post of q naming r.  `fn` returns 0 on success.  Used to run several rank
 * processes on one GPU (tests); no counterpart in the reference (single-GPU, README.md:361-367). */
typedef struct qsim_dist_post {
    int32_t peer, _pad;
    uint64_t bytes;
    const void* send;
    void* recv;
} qsim_dist_post;
typedef int (*qsim_dist_transport_fn)(void* ctx, const qsim_dist_post* posts, size_t count);
int qsim_dist_create_hosted(int n_qubits, int rank, int world, int device, qsim_dist_transport_fn fn,
                            void* ctx, qsim_dist** out);
int qsim_dist_destroy(qsim_dist* d);
int qsim_dist_run(qsim_dist* d, const qsim_gate* gates, size_t count, int flags);
int qsim_dist_sync(qsim_dist* d);
/* Collective: qsim_dist_sync, then a one-value all-reduce on the communicator, so every rank
 * returns within the collective's latency of the others (the per-step timing barrier of the
 * N > 1 bench; no reference counterpart: the reference is single-GPU, README.md:361-367). */
int qsim_dist_barrier(qsim_dist* d);
int qsim_dist_overlapped(qsim_dist* d, int* remaps); /* remaps of the last run that overlapped local work */
/* Runs of this object whose first step merged the previous run's carried last step (the
 * EXPERIMENTAL cross-run overlap, QSIM_DIST_CARRY=1, off by default; read per run). */
int qsim_dist_carried_runs(qsim_dist* d, int* runs);
int qsim_dist_remap_bytes(qsim_dist* d, double* sent); /* bytes this rank sent in its last run's remaps */
int qsim_dist_reset(qsim_dist* d);                         /* |0..0>, identity qubit map */
int qsim_dist_perm(qsim_dist* d, int32_t* perm);            /* logical -> physical, n entries */
/* This rank's 2*2^(n-g) doubles (virtual mode: all shards in rank order, 2*2^n doubles). */
int qsim_dist_local_state(qsim_dist* d, double* dst);
/* Full state in LOGICAL index order on rank 0 (collective; dst may be NULL on other ranks). */
int qsim_dist_gather_state(qsim_dist* d, double* dst);
int qsim_dist_total_probability(qsim_dist* d, double* out); /* collective */
int qsim_dist_prob_bit_zero(qsim_dist* d, int logical_bit, double* out);  /* collective */
int qsim_dist_profile(qsim_dist* d, int enable);
int qsim_dist_profile_count(qsim_dist* d, int* n);
int qsim_dist_profile_get(qsim_dist* d, int i, char* name, size_t name_len, double* total_ms,
                          int64_t* launches, double* alg_bytes);
/* Host-only planner (no GPU, no RCCL): the exact step list qsim_dist_run executes on `rank`
 * starting from qubit map perm_inout (updated).  Call with caps = 0 to size the output. */
int qsim_dist_plan(int n_qubits, int world, int rank, const qsim_gate* gates, size_t count,
                   int32_t* perm_inout, qsim_dist_step* steps, size_t step_cap, size_t* n_steps,
                   qsim_op* ops, size_t op_cap, size_t* n_ops);

/* Host-only: per step of that plan, as qsim_dist_run would plan it, three ints: fused passes
 * (-1 for an exchange step), leading passes that run per half as the exchange before lands, and
 * trailing passes that run per half before the exchange after (the overlapped work);
 * `cap` counts steps.  perm_inout updated as by qsim_dist_plan. */
int qsim_dist_plan_passes(int n_qubits, int world, int rank, const qsim_gate* gates, size_t count,
                          int32_t* perm_inout, int32_t* passes, size_t cap, size_t* n_steps);
/* As qsim_dist_plan_passes, with the cross-run overlap of qsim_dist_run: *carry_inout (in) the
 * pivots of the previous run's last remap still in flight when this run starts (0: none; the first
 * step's leading passes that avoid them run per part), (out) the pivots this run carries into the
 * next (its last step runs wholly per part and is merged into the next run's first step). */
int qsim_dist_plan_passes_carry(int n, int world, int rank, const qsim_gate* gates, size_t count,
                                int32_t* perm_inout, uint64_t* carry_inout, int32_t* passes, size_t cap,
                                size_t* n_steps);
/* As qsim_dist_plan_passes_carry with five ints per step: passes, head, tail, then the coarse
 * passes (those just ahead of the tail that run per coarse part, DStep::coarse / qsim_dist_step
 * .coarse of the exchange after) and the number of coarse pivot bits. */
int qsim_dist_plan_passes_coarse(int n, int world, int rank, const qsim_gate* gates, size_t count,
                                 int32_t* perm_inout, uint64_t* carry_inout, int32_t* passes, size_t cap,
                                 size_t* n_steps);

/* Host-only: forget the process-wide memo of remap pivots (planning is then redone from scratch,
 * as in a fresh rank process). */
int qsim_dist_plan_memo_clear(void);
/* Host-only: the slab layout the pack / unpack kernels use for exchange step `step` on `rank`.
 * part < 0: the whole remap; part j: part j of an overlapped remap (its pivot bits hold j).
 * my_c: the slab that stays; peer_of[c], c < 2^k: the rank slab c goes to and comes from;
 * index[c * chunk + e] (e < chunk = 2^(L - k - m), m = pivots of a part, 0 for part < 0): the
 * local amplitude index of element e of slab c.  index_cap counts entries (2^(L - m) needed). */
int qsim_dist_slab_map(int n_qubits, int world, int rank, const qsim_dist_step* step, int part,
                       int32_t* my_c, int32_t* peer_of, uint64_t* index, size_t index_cap);

#define QSIM_MAX_QUBITS_SINGLE 30
#define QSIM_MIN_QUBITS 1

#ifdef __cplusplus
}
#endif
#endif /* QSIM_HIP_H */
