"""Low-level Lanczos entry points — mirror of the reference's ``src/algorithms``.

=====================================  ================================================
this module                            reference
=====================================  ================================================
``TridiagonalSystemView``              src/algorithms/mod.rs:57-67
``LanczosDecomposition``               src/algorithms/mod.rs:94-108
``LanczosOutput``                      src/algorithms/mod.rs:115-122
``LanczosPassTwoOutput``               src/algorithms/mod.rs:130-135
``lanczos_standard``                   src/algorithms/lanczos.rs:55-156
``lanczos_pass_one``                   src/algorithms/lanczos_two_pass.rs:65-110
``lanczos_pass_two``                   src/algorithms/lanczos_two_pass.rs:128-140
``lanczos_pass_two_with_basis``        src/algorithms/lanczos_two_pass.rs:149-166
=====================================  ================================================

Every call runs the recurrence on the GPU through libtpl_amd.so (C ABI,
include/tpl.h). ``b`` may be a numpy array (results come back as numpy) or a torch
CUDA tensor (results stay on the device as torch tensors).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_double, c_size_t
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import _lib
from ._vec import Vec
from .error import check
from .operator import HipCsrOp, as_operator

BREAKDOWN_TOLERANCE = 1000.0 * np.finfo(np.float64).eps  # src/algorithms/mod.rs:140-143


@dataclass
class TridiagonalSystemView:
    alphas: np.ndarray
    betas: np.ndarray
    steps_taken: int


@dataclass
class LanczosDecomposition:
    alphas: np.ndarray
    betas: np.ndarray
    steps_taken: int
    b_norm: float


@dataclass
class LanczosOutput:
    v_k: object  # (n, steps) column-major; numpy or torch
    decomposition: LanczosDecomposition


@dataclass
class LanczosPassTwoOutput:
    x_k: object
    v_k: object


class DeviceBasisView:
    """The ``MatRef`` V_k handed to a step callback: a device pointer plus shape.

    ``numpy()`` copies it to the host (n x k, column-major like the reference)."""

    def __init__(self, ptr: int, n: int, k: int):
        self.ptr, self.shape = ptr, (n, k)

    def numpy(self) -> np.ndarray:
        n, k = self.shape
        out = np.empty((k, n), dtype=np.float64)
        if n * k:
            check(_lib.tpl_copy_to_host(out.ctypes.data, self.ptr, n * k * 8))
        return out.T


def _op(operator) -> HipCsrOp:
    """A HipCsrOp, or the caller's scipy matrix uploaded once (operator.as_operator)."""
    return as_operator(operator)


def _reorth_mode(r) -> int:
    if r in (False, None, 0):
        return 0
    if r in (True, 1, "cgs2"):
        return 1
    if r in (2, "selective"):
        return 2
    raise ValueError("reorthogonalize must be False, True / 'cgs2' or 'selective'")


def lanczos_standard(operator, b, k: int, callback: Optional[Callable] = None,
                     reorthogonalize=False) -> LanczosOutput:
    """One-pass Lanczos storing V_k (in HBM); src/algorithms/lanczos.rs:55-156.

    ``callback(k, v_k_view, t_k_view) -> bool`` mirrors ``LanczosCallback``
    (src/algorithms/mod.rs:82-86): return False to stop early.
    ``reorthogonalize=True`` (or ``"cgs2"``) adds CGS2 full re-orthogonalisation against
    V_k, ``"selective"`` the Kahan–Parlett variant (second pass only when needed) —
    extensions with no reference counterpart (not used by any reference path).
    """
    op = _op(operator)
    bv = Vec(b)
    alphas = np.zeros(max(k, 1))
    betas = np.zeros(max(k, 1))
    steps = c_size_t(0)
    bnorm = c_double(0.0)
    v_full = bv.empty(max(k, 1), op.nrows())  # C-order (k, n) == column-major (n, k)
    cb_c = None
    raised = []
    if callback is not None:
        def _cb(kk, vptr, n, pa, na, pb, nb, user):
            va = np.ctypeslib.as_array(pa, (na,)).copy() if na else np.zeros(0)
            vb = np.ctypeslib.as_array(pb, (nb,)).copy() if nb else np.zeros(0)
            try:
                return 1 if callback(int(kk), DeviceBasisView(vptr, int(n), int(kk)),
                                     TridiagonalSystemView(va, vb, int(kk))) else 0
            except BaseException as e:  # stop the device loop, re-raised below
                raised.append(e)
                return 0
        cb_c = _lib.STEP_CB(_cb)
    check(_lib.tpl_lanczos_standard(
        op.handle, bv.ptr, bv.n, k, alphas.ctypes.data_as(POINTER(c_double)),
        betas.ctypes.data_as(POINTER(c_double)), byref(steps), byref(bnorm), Vec.ptr_of(v_full),
        bv.mem, _reorth_mode(reorthogonalize), cb_c, None))
    if raised:
        raise raised[0]
    s = steps.value
    v_k = v_full[:s].T
    dec = LanczosDecomposition(alphas[:s].copy(), betas[:max(s - 1, 0)].copy(), s, bnorm.value)
    return LanczosOutput(v_k, dec)


def lanczos_pass_one(operator, b, k: int) -> LanczosDecomposition:
    """First pass: scalars only, O(n) memory; src/algorithms/lanczos_two_pass.rs:65-110."""
    op = _op(operator)
    bv = Vec(b)
    alphas = np.zeros(max(k, 1))
    betas = np.zeros(max(k, 1))
    steps = c_size_t(0)
    bnorm = c_double(0.0)
    check(_lib.tpl_lanczos_pass_one(op.handle, bv.ptr, bv.n, k,
                                    alphas.ctypes.data_as(POINTER(c_double)),
                                    betas.ctypes.data_as(POINTER(c_double)), byref(steps),
                                    byref(bnorm), bv.mem))
    s = steps.value
    return LanczosDecomposition(alphas[:s].copy(), betas[:max(s - 1, 0)].copy(), s, bnorm.value)


def _pass_two(operator, b, decomposition: LanczosDecomposition, y_k, store_basis: bool):
    op = _op(operator)
    bv = Vec(b)
    y = np.ascontiguousarray(np.asarray(y_k, dtype=np.float64).reshape(-1)) \
        if not hasattr(y_k, "is_cuda") else y_k.detach().double().cpu().numpy().reshape(-1)
    a = np.ascontiguousarray(decomposition.alphas, dtype=np.float64).reshape(-1)
    bb = np.ascontiguousarray(decomposition.betas, dtype=np.float64).reshape(-1)
    s = int(decomposition.steps_taken)
    x = bv.empty(op.nrows())
    v = bv.empty(max(s, 1), op.nrows()) if store_basis else None
    check(_lib.tpl_lanczos_pass_two(
        op.handle, bv.ptr, bv.n, a.ctypes.data_as(POINTER(c_double)), a.shape[0],
        bb.ctypes.data_as(POINTER(c_double)), bb.shape[0], s, float(decomposition.b_norm),
        y.ctypes.data_as(POINTER(c_double)), y.shape[0], Vec.ptr_of(x),
        Vec.ptr_of(v) if v is not None else None, bv.mem))
    return x, (v[:s].T if v is not None else None)


def lanczos_pass_two(operator, b, decomposition: LanczosDecomposition, y_k):
    """Second pass: regenerate v_j on the fly, x = sum_j y_j v_j;
    src/algorithms/lanczos_two_pass.rs:128-140. ``y_k`` = f(T_k) e_1 * ||b||."""
    return _pass_two(operator, b, decomposition, y_k, False)[0]


def lanczos_pass_two_with_basis(operator, b, decomposition: LanczosDecomposition,
                                y_k) -> LanczosPassTwoOutput:
    """Test variant returning the regenerated basis V'_k;
    src/algorithms/lanczos_two_pass.rs:149-166."""
    x, v = _pass_two(operator, b, decomposition, y_k, True)
    return LanczosPassTwoOutput(x, v)
