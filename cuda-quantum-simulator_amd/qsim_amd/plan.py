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
