"""High-level solvers — mirror of the reference's ``src/solvers.rs``.

``lanczos(operator, b, k, f_tk_solver)``           src/solvers.rs:46-107
``lanczos_two_pass(operator, b, k, f_tk_solver)``  src/solvers.rs:133-175

Same argument meaning and error behaviour as the reference (the ``stack``
workspace argument has no counterpart: the device workspace belongs to the
operator). ``operator`` is a ``HipCsrOp`` (upload once) or the caller's own scipy CSR / CSC
matrix (uploaded on first use and re-used while unchanged: ``operator.as_operator``).
``f_tk_solver`` is a callable ``(alphas, betas) -> y'`` or a built-in
from :mod:`tpl_amd.ftk` (``"inv"``, ``"exp"``, ``"sq"``). Returns x_k with the
shape of ``b`` flattened to (n,) — numpy for host ``b``, torch CUDA for device ``b``.
"""
from __future__ import annotations

from . import _lib, ftk
from ._vec import Vec
from .error import LanczosError, check
from .operator import as_operator


def _run(fn, operator, b, k, f_tk_solver):
    operator = as_operator(operator)
    bv = Vec(b)
    x = bv.empty(operator.nrows())
    fptr, keep = ftk.resolve(f_tk_solver)
    try:
        check(fn(operator.handle, bv.ptr, bv.n, k, fptr, None, Vec.ptr_of(x), bv.mem))
    except LanczosError as e:
        raise ftk.remap_error(e, keep) from None
    return x


def lanczos(operator, b, k: int, f_tk_solver):
    """f(A) b by standard one-pass Lanczos: V_k kept in HBM, x = ||b|| V_k f(T_k) e_1."""
    return _run(_lib.tpl_lanczos, operator, b, k, f_tk_solver)


def lanczos_two_pass(operator, b, k: int, f_tk_solver):
    """f(A) b by two-pass Lanczos: O(n) memory, the basis is regenerated in pass two."""
    return _run(_lib.tpl_lanczos_two_pass, operator, b, k, f_tk_solver)
