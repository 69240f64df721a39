"""ctypes bindings of the C ABI (include/qsim_hip.h, include/qsim_circuits.h).

The HIP engine (lib/libqsim_hip.so) is REQUIRED: there is no CPU fallback anywhere in this
package.  If the shared object is missing or cannot be loaded, import fails loudly.
"""
from __future__ import annotations

import atexit
import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_int, c_int32, c_int64,
                    c_size_t, c_uint, c_uint64, c_void_p)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
HIP_LIB_PATH = os.path.join(LIB_DIR, "libqsim_hip.so")
API_LIB_PATH = os.path.join(LIB_DIR, "libqsim.so")

QSIM_OK = 0
QSIM_ERR_INVALID_ARGUMENT = 1
QSIM_ERR_OUT_OF_RANGE = 2
QSIM_ERR_RUNTIME = 3
QSIM_ERR_DEVICE = 4

QSIM_RUN_PER_GATE = 0
QSIM_RUN_FUSED = 1
QSIM_DM_REFERENCE_Y = 8  # qsim_dm_run flag
QSIM_BATCH_FULL_GATESET = 0
QSIM_BATCH_REFERENCE_GATESET = 1
QSIM_BATCH_PER_GATE = 2
QSIM_BATCH_REFERENCE_NOISE = 4

QSIM_CIRCUIT_BELL = 0
QSIM_CIRCUIT_GHZ = 1
QSIM_CIRCUIT_RANDOM = 2
QSIM_CIRCUIT_RANDOM_HC = 3
QSIM_CIRCUIT_SCALING = 4


class qsim_gate(Structure):
    _fields_ = [("type", c_int32), ("nqubits", c_int32), ("qubits", c_int32 * 3),
                ("_pad", c_int32), ("parameter", c_double)]


class qsim_noise_channel(Structure):
    _fields_ = [("type", c_int32), ("qubit", c_int32), ("probability", c_double)]


def _load(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"qsim_amd: native library {path} is missing; build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


hip = _load(HIP_LIB_PATH)
api = _load(API_LIB_PATH)

_P = c_void_p


def _sig(lib, name, argtypes, restype=c_int):
    f = getattr(lib, name)
    f.argtypes = argtypes
    f.restype = restype
    return f


# ---- engine (libqsim_hip.so)
_sig(hip, "qsim_last_error", [], c_char_p)
_sig(hip, "qsim_abi_version", [])
_sig(hip, "qsim_device_count", [POINTER(c_int)])
_sig(hip, "qsim_set_device", [c_int])
_sig(hip, "qsim_device_info", [c_int, c_char_p, c_size_t, POINTER(c_int), POINTER(c_size_t)])
_sig(hip, "qsim_state_create", [c_int, POINTER(_P)])
_sig(hip, "qsim_state_create_on", [c_int, c_int, POINTER(_P)])
_sig(hip, "qsim_state_destroy", [_P])
_sig(hip, "qsim_state_num_qubits", [_P, POINTER(c_int)])
_sig(hip, "qsim_state_device_ptr", [_P, POINTER(_P)])
_sig(hip, "qsim_state_stream", [_P, POINTER(_P)])
_sig(hip, "qsim_state_init_zero", [_P])
_sig(hip, "qsim_state_init_basis", [_P, c_uint64])
_sig(hip, "qsim_state_sync", [_P])
_sig(hip, "qsim_apply_gate", [_P, POINTER(qsim_gate)])
_sig(hip, "qsim_run", [_P, POINTER(qsim_gate), c_size_t, c_int])
_sig(hip, "qsim_apply_matrix1q", [_P, c_int, POINTER(c_double), POINTER(c_int), c_int])
_sig(hip, "qsim_apply_matrix2q", [_P, c_int, c_int, POINTER(c_double), POINTER(c_int), c_int])
_sig(hip, "qsim_apply_matrix", [_P, POINTER(c_int), c_int, POINTER(c_double), POINTER(c_int), c_int])
_sig(hip, "qsim_apply_hadamard_optimized", [_P, c_int, c_int, _P])
_sig(hip, "qsim_apply_cnot_optimized", [_P, c_int, c_int, c_int, _P])
_sig(hip, "qsim_apply_matrix1q_raw", [_P, c_int, c_int, POINTER(c_double), _P])
_sig(hip, "qsim_apply_diagonal_layer", [_P, POINTER(c_double), c_uint64])
_sig(hip, "qsim_apply_gate_raw", [_P, c_int, POINTER(qsim_gate), _P])
_sig(hip, "qsim_plan_fused", [c_int, POINTER(qsim_gate), c_size_t, c_int, _P, _P,
                              POINTER(c_int32)])
_sig(hip, "qsim_set_jit", [c_int, c_int])
_sig(hip, "qsim_jit_shutdown", [])
_sig(hip, "qsim_set_relabel", [c_int, c_int])
_sig(hip, "qsim_state_perm", [_P, POINTER(c_int32)])
_sig(hip, "qsim_state_layout_info", [_P, POINTER(c_int), POINTER(c_int), POINTER(c_int)])
_sig(hip, "qsim_state_restore_layout", [_P])
_sig(hip, "qsim_state_relayout", [_P, POINTER(c_int)])
_sig(hip, "qsim_set_relayout", [c_int, c_int])
_sig(hip, "qsim_jit_build_relayout", [c_int, POINTER(qsim_gate), c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_plan_relayout", [c_int, POINTER(qsim_gate), c_size_t, POINTER(c_int32), POINTER(c_int),
                                 POINTER(c_double)])
_sig(hip, "qsim_plan_exec_host", [c_int, POINTER(qsim_gate), c_size_t, c_int, _P, POINTER(c_int32),
                                  POINTER(c_int)])
_sig(hip, "qsim_set_calibrate", [c_int, c_int])
_sig(hip, "qsim_set_tile_height", [c_int])
_sig(hip, "qsim_set_tile_rb7", [c_int])
_sig(hip, "qsim_set_tile_ctrl_out", [c_int])
_sig(hip, "qsim_plan_relabel", [c_int, _P, c_size_t, POINTER(c_int32), POINTER(c_double), POINTER(c_double)])
# Stop the background pass compiler before interpreter / library teardown (a hipRTC compile that
# is still running while the compiler's statics are destroyed aborts the process).
atexit.register(hip.qsim_jit_shutdown)
_sig(hip, "qsim_jit_source", [c_int, POINTER(qsim_gate), c_size_t, c_char_p, c_size_t,
                              POINTER(c_size_t)])
_sig(hip, "qsim_jit_build", [c_int, POINTER(qsim_gate), c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_state_to_host", [_P, _P])
_sig(hip, "qsim_state_from_host", [_P, _P])
_sig(hip, "qsim_state_probabilities", [_P, _P])
_sig(hip, "qsim_state_total_probability", [_P, POINTER(c_double)])
_sig(hip, "qsim_state_prob_bit_zero", [_P, c_int, POINTER(c_double)])
_sig(hip, "qsim_state_collapse", [_P, c_int, c_int, c_double])
_sig(hip, "qsim_state_sample", [_P, _P, c_int, _P])
_sig(hip, "qsim_state_max_abs_diff", [_P, _P, POINTER(c_double)])
_sig(hip, "qsim_state_memory_bytes", [_P, POINTER(c_uint64)])
_sig(hip, "qsim_state_profile", [_P, c_int])
_sig(hip, "qsim_state_profile_count", [_P, POINTER(c_int)])
_sig(hip, "qsim_state_profile_get", [_P, c_int, c_char_p, c_size_t, POINTER(c_double),
                                     POINTER(c_int64), POINTER(c_double)])
_sig(hip, "qsim_state_profile_reset", [_P])
_sig(hip, "qsim_batch_create", [c_int, c_int, POINTER(_P)])
_sig(hip, "qsim_batch_destroy", [_P])
_sig(hip, "qsim_batch_reset", [_P])
_sig(hip, "qsim_batch_set_seed", [_P, c_uint64])
_sig(hip, "qsim_batch_set_trajectory_offset", [_P, c_uint64])
_sig(hip, "qsim_batch_run", [_P, POINTER(qsim_gate), c_size_t, POINTER(qsim_noise_channel),
                             c_size_t, c_int])
_sig(hip, "qsim_batch_avg_probabilities", [_P, _P])
_sig(hip, "qsim_batch_traj_probabilities", [_P, c_int, _P])
_sig(hip, "qsim_batch_traj_state", [_P, c_int, _P])
_sig(hip, "qsim_batch_sample", [_P, _P, c_int, _P])
_sig(hip, "qsim_state_last_run", [_P, _P, _P])
_sig(hip, "qsim_batch_last_run", [_P, _P, _P])
_sig(hip, "qsim_batch_histogram", [_P, _P, c_int, _P])
_sig(hip, "qsim_batch_device_ptr", [_P, POINTER(_P)])
_sig(hip, "qsim_batch_sync", [_P])
_sig(hip, "qsim_batch_profile", [_P, c_int])
_sig(hip, "qsim_batch_profile_count", [_P, POINTER(c_int)])
_sig(hip, "qsim_batch_profile_get", [_P, c_int, c_char_p, c_size_t, POINTER(c_double),
                                     POINTER(c_int64), POINTER(c_double)])

_sig(hip, "qsim_noise_apply", [_P, c_int, c_int, c_double, c_uint64, c_uint64])
_sig(hip, "qsim_noise_check_flips", [POINTER(c_uint64)])
_sig(hip, "qsim_noise_gap_check", [c_double, c_uint64, c_uint64, POINTER(c_uint64), POINTER(c_uint64)])
_sig(hip, "qsim_cache_stats", [POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)])
_sig(hip, "qsim_noise_gap_check_edges", [c_double, c_uint64, POINTER(c_uint64), POINTER(c_uint64),
                                         POINTER(c_uint64)])
_sig(hip, "qsim_noisy_run", [_P, POINTER(qsim_gate), c_size_t, POINTER(qsim_noise_channel), c_size_t,
                             c_uint64, POINTER(c_uint64), c_int])

_sig(hip, "qsim_dm_plan_info", [c_int, POINTER(qsim_gate), c_size_t, POINTER(qsim_noise_channel), c_size_t,
                                  c_int, POINTER(c_int32), c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_dm_jit_source", [c_int, POINTER(qsim_gate), c_size_t, POINTER(qsim_noise_channel), c_size_t,
                                   c_int, c_char_p, c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_dm_run", [_P, c_int, POINTER(qsim_gate), c_size_t, POINTER(qsim_noise_channel),
                          c_size_t, c_int])
_sig(hip, "qsim_dm_apply_channel", [_P, c_int, c_int, c_int, c_double])
_sig(hip, "qsim_dm_diagonal", [_P, c_int, _P])
_sig(hip, "qsim_dm_init_pure", [_P, c_int, _P])
_sig(hip, "qsim_dm_init_maximally_mixed", [_P, c_int])

# ---- multi-GPU (sharded) state
class qsim_op(Structure):
    _fields_ = [("kind", c_int32), ("sub", c_int32), ("t0", c_int32), ("t1", c_int32),
                ("cmask", c_uint64), ("d0_one", c_int32), ("src", c_int32),
                ("m", c_double * 8)]


class qsim_dist_step(Structure):
    _fields_ = [("kind", c_int32), ("k", c_int32), ("op_begin", c_int32), ("op_end", c_int32),
                ("gpos", c_int32 * 8), ("lpos", c_int32 * 8), ("pivot", c_int32), ("role", c_int32),
                ("pmask", c_uint64), ("coarse", c_uint64)]


class qsim_dist_post(Structure):
    _fields_ = [("peer", c_int32), ("_pad", c_int32), ("bytes", c_uint64), ("send", c_void_p),
                ("recv", c_void_p)]


qsim_dist_transport_fn = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(qsim_dist_post), c_size_t)

_sig(hip, "qsim_dist_unique_id", [_P])
_sig(hip, "qsim_dist_create", [c_int, c_int, c_int, _P, c_int, POINTER(_P)])
_sig(hip, "qsim_dist_create_virtual", [c_int, c_int, c_int, POINTER(_P)])
_sig(hip, "qsim_dist_create_hosted", [c_int, c_int, c_int, c_int, qsim_dist_transport_fn, _P,
                                      POINTER(_P)])
_sig(hip, "qsim_dist_virtual_rccl", [_P, c_char_p])
_sig(hip, "qsim_dist_destroy", [_P])
_sig(hip, "qsim_dist_run", [_P, POINTER(qsim_gate), c_size_t, c_int])
_sig(hip, "qsim_dist_sync", [_P])
_sig(hip, "qsim_dist_barrier", [_P])
_sig(hip, "qsim_dist_overlapped", [_P, POINTER(c_int)])
_sig(hip, "qsim_dist_fused_remaps", [_P, POINTER(c_int)])
_sig(hip, "qsim_dist_carried_runs", [_P, POINTER(c_int)])
_sig(hip, "qsim_dist_remap_bytes", [_P, POINTER(c_double)])
_sig(hip, "qsim_dist_plan_memo_clear", [])
_sig(hip, "qsim_dist_slab_map", [c_int, c_int, c_int, POINTER(qsim_dist_step), c_int, POINTER(c_int32),
                                 POINTER(c_int32), POINTER(c_uint64), c_size_t])
_sig(hip, "qsim_dist_reset", [_P])
_sig(hip, "qsim_dist_perm", [_P, POINTER(c_int32)])
_sig(hip, "qsim_dist_local_state", [_P, _P])
_sig(hip, "qsim_dist_gather_state", [_P, _P])
_sig(hip, "qsim_dist_total_probability", [_P, POINTER(c_double)])
_sig(hip, "qsim_dist_prob_bit_zero", [_P, c_int, POINTER(c_double)])
_sig(hip, "qsim_dist_profile", [_P, c_int])
_sig(hip, "qsim_dist_profile_count", [_P, POINTER(c_int)])
_sig(hip, "qsim_dist_profile_get", [_P, c_int, c_char_p, c_size_t, POINTER(c_double),
                                    POINTER(c_int64), POINTER(c_double)])
_sig(hip, "qsim_dist_plan", [c_int, c_int, c_int, POINTER(qsim_gate), c_size_t, POINTER(c_int32),
                             POINTER(qsim_dist_step), c_size_t, POINTER(c_size_t),
                             POINTER(qsim_op), c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_dist_plan_passes", [c_int, c_int, c_int, POINTER(qsim_gate), c_size_t,
                                    POINTER(c_int32), POINTER(c_int32), c_size_t, POINTER(c_size_t)])
_sig(hip, "qsim_dist_plan_passes_carry", [c_int, c_int, c_int, POINTER(qsim_gate), c_size_t,
                                          POINTER(c_int32), POINTER(c_uint64), POINTER(c_int32), c_size_t,
                                          POINTER(c_size_t)])

# ---- C++ API library (libqsim.so): circuit factories
_sig(hip, "qsim_dist_plan_passes_coarse", [c_int, c_int, c_int, POINTER(qsim_gate), c_size_t,
                                          POINTER(c_int32), POINTER(c_uint64), POINTER(c_int32), c_size_t,
                                          POINTER(c_size_t)])

# ---- C++ API library (libqsim.so): circuit factories
_sig(api, "qsim_circuit_make", [c_int, c_int, c_int, c_uint, POINTER(qsim_gate), c_size_t,
                                POINTER(c_size_t)])
_sig(api, "qsim_circuit_depth", [c_int, POINTER(qsim_gate), c_size_t, POINTER(c_size_t)])
_sig(api, "qsim_circuits_last_error", [], c_char_p)


def raise_for(rc: int, msg_fn=None) -> None:
    """Map a QSIM_ERR_* code to the reference's exception classes (Python analogues)."""
    if rc == QSIM_OK:
        return
    msg = (msg_fn or hip.qsim_last_error)()
    msg = msg.decode() if isinstance(msg, bytes) else str(msg)
    if rc == QSIM_ERR_INVALID_ARGUMENT:
        raise ValueError(msg)            # std::invalid_argument
    if rc == QSIM_ERR_OUT_OF_RANGE:
        raise IndexError(msg)            # std::out_of_range
    raise RuntimeError(msg)              # std::runtime_error (incl. device errors)


def check(rc: int) -> None:
    raise_for(rc)


def check_circ(rc: int) -> None:
    raise_for(rc, api.qsim_circuits_last_error)


def loaded_paths():
    return [HIP_LIB_PATH, API_LIB_PATH]
