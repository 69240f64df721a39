"""Host-side view of the engine's fused-pass planner (qsim_plan_fused, include/qsim_hip.h)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .circuit import Circuit


def plan_fused(circuit: Circuit, hmax: int = 6):
    """Return (order, pass_of, n_passes): execution order of the circuit's gates (indices into
    circuit.getGates()), the pass each runs in (-1 = per-gate), and the number of fused passes."""
    arr, cnt = circuit.to_abi()
    order = np.zeros(max(1, cnt), np.int32)
    pass_of = np.zeros(max(1, cnt), np.int32)
    npass = ctypes.c_int32(0)
    _lib.check(_lib.hip.qsim_plan_fused(circuit.getNumQubits(), arr, cnt, hmax,
                                        order.ctypes.data_as(ctypes.c_void_p),
                                        pass_of.ctypes.data_as(ctypes.c_void_p),
                                        ctypes.byref(npass)))
    return order[:cnt], pass_of[:cnt], npass.value


def set_jit(mode: int = -1, min_qubits: int = -1) -> None:
    """Circuit-specialised pass kernels: mode 0 off, 1 background compile (default), 2 compile
    on a plan's first run; states below `min_qubits` use the pass interpreter (qsim_set_jit)."""
    _lib.check(_lib.hip.qsim_set_jit(mode, min_qubits))


def jit_source(circuit: Circuit) -> str:
    """The HIP source the engine generates for this circuit's fused plan ('' if no staged pass)."""
    arr, cnt = circuit.to_abi()
    n = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_jit_source(circuit.getNumQubits(), arr, cnt, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value + 1)
    _lib.check(_lib.hip.qsim_jit_source(circuit.getNumQubits(), arr, cnt, buf, n.value + 1,
                                        ctypes.byref(n)))
    return buf.value.decode()


def jit_build(circuit: Circuit) -> int:
    """Compile the circuit's generated pass kernels with hipRTC for gfx950 (no GPU needed);
    returns the code-object size in bytes (0 when nothing is specialised)."""
    arr, cnt = circuit.to_abi()
    n = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_jit_build(circuit.getNumQubits(), arr, cnt, ctypes.byref(n)))
    return n.value


def set_relabel(mode: int = -1, min_qubits: int = -1) -> None:
    """Layout-aware qubit relabeling of fused runs (qsim_set_relabel): mode 0 off, 1 on; states
    below `min_qubits` are never relabeled; negative arguments leave a setting unchanged."""
    _lib.check(_lib.hip.qsim_set_relabel(mode, min_qubits))


def set_relayout(mode: int = -1, min_qubits: int = -1) -> None:
    """Relayout plans (every pass stores its tile under the next pass's qubit layout) for first
    runs of states from `min_qubits` on (qsim_set_relayout): mode 0 off, 1 on (when they need
    fewer passes or win the device timing), 2 forced (tests); negative arguments leave a setting
    unchanged."""
    _lib.check(_lib.hip.qsim_set_relayout(mode, min_qubits))


def set_calibrate(mode: int = -1, min_qubits: int = -1) -> None:
    """Time the layout model's top candidates on the device at a basis state's first run and
    keep the fastest (qsim_set_calibrate; needs set_jit(2)): mode 0 off, 1 on."""
    _lib.check(_lib.hip.qsim_set_calibrate(mode, min_qubits))


def set_tile_height(h: int = -1) -> None:
    """Tile height of fused passes planned from now on (qsim_set_tile_height): tiles of 6 + h
    qubits, h in 0..7 (default 6); h < 0 restores the default."""
    _lib.check(_lib.hip.qsim_set_tile_height(h))


def set_tile_rb7(rb: int = -1) -> None:
    """Register bits per stage of 13-qubit tiles (4: 512-thread workgroups, default; 3: 1024
    threads with 8 amplitudes each); -1 restores QSIM_TILE_RB7."""
    _lib.check(_lib.hip.qsim_set_tile_rb7(rb))


def set_tile_ctrl_out(mode: int = -1) -> None:
    """Tile-constant controls (qsim_set_tile_ctrl_out): 1 (default) a control qubit need not be a
    tile qubit (the op runs per tile where it reads 1), 0 every control is a tile qubit."""
    _lib.check(_lib.hip.qsim_set_tile_ctrl_out(mode))


# The shipped policy (include/qsim_hip.h; environment variables unset).
DEFAULTS = {"jit": (1, 20), "relabel": (1, 26), "relayout": (1, 20), "calibrate": (1, 26)}


def restore_defaults() -> None:
    """Put every process-wide planning policy back to the shipped defaults: background JIT from
    20 qubits, relabeling from 26, relayout plans from 20, calibrated first runs from 26 (with
    inline compilation), the size rule for tile heights (tests call this after changing any)."""
    set_jit(*DEFAULTS["jit"])
    set_relabel(*DEFAULTS["relabel"])
    set_relayout(*DEFAULTS["relayout"])
    set_calibrate(*DEFAULTS["calibrate"])
    set_tile_height(-1)
    set_tile_ctrl_out(1)


def plan_relabel(circuit: Circuit):
    """(perm, predicted_us_before, predicted_us_after): the logical -> physical qubit map the
    engine would choose for this circuit's fused plan (identity when none pays), host only."""
    n = circuit.getNumQubits()
    arr, cnt = circuit.to_abi()
    perm = (ctypes.c_int32 * n)()
    b, a = ctypes.c_double(), ctypes.c_double()
    _lib.check(_lib.hip.qsim_plan_relabel(n, arr, cnt, perm, ctypes.byref(b), ctypes.byref(a)))
    return list(perm), b.value, a.value


def plan_exec_host(circuit: Circuit, mode: int = 1, state=None):
    """Plan the circuit (mode 0: fixed-layout planner under the identity labels, 1: relayout
    planner) and execute the plan on the host exactly as the staged pass kernels address the
    state (qsim_plan_exec_host; tests of the planners' index math, no GPU).  Returns
    (state in logical order, start/end layout, pass count)."""
    n = circuit.getNumQubits()
    arr, cnt = circuit.to_abi()
    if state is None:
        st = np.zeros(1 << n, np.complex128)
        st[0] = 1.0
    else:
        st = np.array(state, dtype=np.complex128)
    st = np.ascontiguousarray(st)
    perm = (ctypes.c_int32 * n)()
    passes = ctypes.c_int(0)
    _lib.check(_lib.hip.qsim_plan_exec_host(n, arr, cnt, mode, st.ctypes.data_as(ctypes.c_void_p),
                                            perm, ctypes.byref(passes)))
    return st, list(perm), passes.value


def plan_relayout(circuit: Circuit):
    """(perm, passes, predicted_us) of the circuit's relayout plan (qsim_plan_relayout, host
    only); passes = 0 when no relayout plan exists."""
    n = circuit.getNumQubits()
    arr, cnt = circuit.to_abi()
    perm = (ctypes.c_int32 * n)()
    passes = ctypes.c_int(0)
    pred = ctypes.c_double(0.0)
    _lib.check(_lib.hip.qsim_plan_relayout(n, arr, cnt, perm, ctypes.byref(passes), ctypes.byref(pred)))
    return list(perm), passes.value, pred.value


def jit_build_relayout(circuit: Circuit) -> int:
    """Compile the circuit's relayout plan (qsim_jit_build_relayout, hipRTC for gfx950, no GPU
    needed); returns the code-object size in bytes."""
    arr, cnt = circuit.to_abi()
    n = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_jit_build_relayout(circuit.getNumQubits(), arr, cnt, ctypes.byref(n)))
    return n.value
