"""f(T_k) e_1 solvers — the ``f_tk_solver`` closure of the reference
(``FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>``, src/solvers.rs:57,144).

A solver is either a Python callable ``f(alphas, betas) -> array (steps,) or (steps, 1)``
(raise to signal ``Err``) or one of the built-ins below, which run as native code
inside libtpl_amd.so (no Python on the solve path):

* ``INV`` — T_k^{-1} e_1 by tridiagonal LU with partial pivoting
  (src/bin/tradeoff.rs:245-258, tests/correctness.rs:171-179)
* ``EXP`` — Q exp(Lambda) Q^T e_1 by symmetric tridiagonal QL (src/bin/stability.rs:175-193)
* ``SQ``  — T_k^2 e_1 (tests/correctness.rs:287-299)
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_size_t

import numpy as np

from . import _lib
from .error import LanczosError


class BuiltinFtk:
    def __init__(self, name: str, ptr: int, fn):
        self.name = name
        self.ptr = ptr
        self._fn = fn

    def __call__(self, alphas, betas):
        """Evaluate on the host (same native code the solvers call)."""
        a = np.ascontiguousarray(alphas, dtype=np.float64)
        b = np.ascontiguousarray(betas, dtype=np.float64)
        n = a.shape[0]
        y = np.zeros(n, dtype=np.float64)
        ylen = c_size_t(0)
        err = ctypes.create_string_buffer(1024)
        rc = self._fn(a.ctypes.data_as(POINTER(c_double)), n, b.ctypes.data_as(POINTER(c_double)),
                      b.shape[0], y.ctypes.data_as(POINTER(c_double)), n, ctypes.byref(ylen),
                      err, 1024, None)
        if rc != 0:
            raise RuntimeError(err.value.decode())
        return y

    def __repr__(self):
        return f"tpl_amd.ftk.{self.name}"


INV = BuiltinFtk("INV", _lib.FTK_INV_PTR, _lib.tpl_ftk_inv)
EXP = BuiltinFtk("EXP", _lib.FTK_EXP_PTR, _lib.tpl_ftk_exp)
SQ = BuiltinFtk("SQ", _lib.FTK_SQ_PTR, _lib.tpl_ftk_sq)

BUILTINS = {"inv": INV, "exp": EXP, "sq": SQ}


class _PyFtk:
    """Wrap a Python callable as a tpl_ftk_fn C callback."""

    def __init__(self, f):
        self.f = f
        self.mismatch = None  # (expected, actual) when y' has ncols != 1
        self.c = _lib.FTK_FN(self._call)

    def _call(self, pa, na, pb, nb, py, ycap, pylen, perr, errcap, user):
        try:
            alphas = np.ctypeslib.as_array(pa, (na,)).copy() if na else np.zeros(0)
            betas = np.ctypeslib.as_array(pb, (nb,)).copy() if nb else np.zeros(0)
            y = self.f(alphas, betas)
            if type(y).__module__.startswith("torch"):
                y = y.detach().cpu().numpy()
            y = np.asarray(y, dtype=np.float64)
            if y.ndim == 2 and y.shape[1] != 1:
                # src/solvers.rs:78-85 — ncols != 1 is a ParameterMismatch on nrows
                self.mismatch = (na, y.shape[0])
                pylen[0] = y.shape[0] if y.shape[0] != na else na + 1
                return 0
            y = y.reshape(-1)
            pylen[0] = y.shape[0]
            m = min(y.shape[0], ycap)
            if m:
                ctypes.memmove(py, y.ctypes.data, m * 8)
            return 0
        except Exception as e:  # Err(e) -> SolverError(e.to_string())
            msg = str(e).encode("utf-8", "replace")[: max(errcap - 1, 0)]
            ctypes.memmove(perr, msg + b"\0", len(msg) + 1)
            return 1


def resolve(f):
    """Return (c function pointer, keepalive) for a solver spec."""
    if isinstance(f, str):
        f = BUILTINS[f.lower()]
    if isinstance(f, BuiltinFtk):
        return f.ptr, None
    if not callable(f):
        raise TypeError("f_tk_solver must be callable or a built-in solver")
    w = _PyFtk(f)
    return ctypes.cast(w.c, ctypes.c_void_p).value, w


def remap_error(err: LanczosError, keep) -> LanczosError:
    if keep is not None and keep.mismatch is not None:
        exp, act = keep.mismatch
        return LanczosError.parameter_mismatch("y_k_prime", exp, act)
    return err
