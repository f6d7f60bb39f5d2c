"""Device-resident CSR operator — the MI355X replacement of faer's
``LinOp<f64>`` for ``SparseColMatRef<usize, f64>`` (used by the reference at
src/algorithms/mod.rs:177 and src/algorithms/lanczos_two_pass.rs:186).

``HipCsrOp`` uploads the matrix once; every solver call then keeps the whole
recurrence in HBM. Vectors may be numpy arrays (host) or torch CUDA tensors
(device, zero-copy through the C ABI's TPL_MEM_DEVICE mode).
"""
from __future__ import annotations

import ctypes
import threading
from ctypes import POINTER, byref, c_double, c_int32, c_int64, c_void_p

import numpy as np

from . import _lib
from .error import TplError, check

_ctx_lock = threading.Lock()
_contexts: dict[int, int] = {}


def device_count() -> int:
    return int(_lib.tpl_device_count())


def context(device: int = 0) -> int:
    """One HIP stream per device per process (created lazily)."""
    with _ctx_lock:
        if device not in _contexts:
            h = c_void_p()
            check(_lib.tpl_ctx_create(device, byref(h)))
            _contexts[device] = h.value
        return _contexts[device]


def _as_csr_arrays(a):
    """Accept a scipy sparse matrix (CSR/CSC; A symmetric), a KKTSystem, or a
    (n, row_ptr, col_idx, vals) tuple; return int64/int32/float64 CSR arrays."""
    if hasattr(a, "a") and hasattr(a, "num_arcs"):  # KKTSystem
        a = a.a
    if isinstance(a, tuple):
        n, rp, ci, v = a
        return (int(n), np.ascontiguousarray(rp, dtype=np.int64),
                np.ascontiguousarray(ci, dtype=np.int32), np.ascontiguousarray(v, dtype=np.float64))
    import scipy.sparse as sp
    if not sp.issparse(a):
        a = sp.csr_matrix(np.asarray(a, dtype=np.float64))
    # a private copy: the caller's matrix is never modified; duplicates are summed and
    # columns sorted (faer's try_new_from_triplets semantics), explicit zeros are kept
    m = a.tocsr(copy=True)
    m.sum_duplicates()
    if m.shape[0] != m.shape[1]:
        raise TplError(_lib.TPL_ERR_INVALID_ARGUMENT, "operator must be square")
    return (m.shape[0], m.indptr.astype(np.int64), m.indices.astype(np.int32),
            m.data.astype(np.float64))


def locality_order(a, short_row_max: int = -1, groups: int = 16):
    """The device's locality row order for matrix ``a`` (tpl_locality_order; host only):
    perm[i] = the row held at internal position i, or None when it is the identity."""
    n, rp, ci, _ = _as_csr_arrays(a)
    perm = np.zeros(max(n, 1), dtype=np.int32)
    applied = c_int32()
    check(_lib.tpl_locality_order(n, rp.ctypes.data_as(POINTER(c_int64)),
                                  ci.ctypes.data_as(POINTER(c_int32)), int(short_row_max),
                                  int(groups), perm.ctypes.data_as(POINTER(c_int32)),
                                  byref(applied)))
    return perm[:n].copy() if applied.value else None


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


class HostPlan:
    """The host half of an operator (tpl_plan_create): rows, order and SpMV layout of a
    single-GPU operator (``mode="single"``, ``order_groups`` as set_order_groups) or of
    rank ``rank`` of a partition (``"replicated"`` / ``"rows"`` / ``"halo"``), computed by the
    runtime's own code with no GPU. ``schedule()`` and ``local_rows`` are what the live
    operator would report; every device call on it fails."""

    _MODES = {"single": 0, "replicated": 1, "rows": 2, "halo": 3}

    def __init__(self, a, mode: str = "single", nranks: int = 1, rank: int = 0,
                 order_groups: int = 0):
        n, rp, ci, v = _as_csr_arrays(a)
        h = c_void_p()
        check(_lib.tpl_plan_create(n, rp.ctypes.data_as(POINTER(c_int64)),
                                   ci.ctypes.data_as(POINTER(c_int32)),
                                   v.ctypes.data_as(POINTER(c_double)), self._MODES[mode],
                                   int(nranks), int(rank), int(order_groups), byref(h)))
        self._op = h.value
        self.mode = mode
        self._n = int(_lib.tpl_op_nrows(self._op))
        rows = np.zeros(max(self._n, 1), dtype=np.int64)
        check(_lib.tpl_op_local_rows(self._op, rows.ctypes.data_as(POINTER(c_int64))))
        self.local_rows = rows[:self._n]

    schedule = None  # bound below (HipCsrOp.schedule: host reads only)

    @property
    def handle(self) -> int:
        return self._op

    def flags(self) -> int:
        return int(_lib.tpl_op_flags(self._op))

    def order_groups(self) -> int:
        return int(_lib.tpl_op_order_groups(self._op))

    def algo_bytes(self, kernel: int) -> float:
        """tpl_kernel_algo_bytes: e.g. the bytes a rank receives per exchange."""
        return float(_lib.tpl_kernel_algo_bytes(self._op, int(kernel)))

    def close(self):
        if getattr(self, "_op", None):
            _lib.tpl_op_destroy(self._op)
            self._op = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HipCsrOp:
    """Symmetric sparse operator resident in the HBM of one MI355X.

    Mirrors ``LinOp``: ``nrows()``, ``ncols()``, ``apply(x)``.
    """

    def __init__(self, a, device: int = 0):
        n, rp, ci, v = _as_csr_arrays(a)
        self.device = device
        self._ctx = context(device)
        h = c_void_p()
        check(_lib.tpl_op_create_csr(
            self._ctx, n, int(rp[-1]) if n > 0 else 0,
            rp.ctypes.data_as(POINTER(c_int64)), ci.ctypes.data_as(POINTER(c_int32)),
            v.ctypes.data_as(POINTER(c_double)), byref(h)))
        self._op = h.value
        self._n = n
        self._nnz = int(rp[-1]) if n > 0 else 0

    # -- LinOp surface -------------------------------------------------------
    def nrows(self) -> int:
        return self._n

    def ncols(self) -> int:
        return self._n

    @property
    def nnz(self) -> int:
        return self._nnz

    @property
    def handle(self) -> int:
        return self._op

    @property
    def int8_values(self) -> bool:
        """True when the values are stored as int8 (lossless; tpl_op_set_value_format)."""
        return bool(int(_lib.tpl_op_flags(self._op)) & 4)

    def set_value_format(self, compress: bool):
        check(_lib.tpl_op_set_value_format(self._op, 1 if compress else 0))

    @property
    def uses_graphs(self) -> bool:
        """False when the passes are launched eagerly (see tpl_op_flags)."""
        return not (int(_lib.tpl_op_flags(self._op)) & 2)

    def apply(self, x):
        """y = A x (LinOp::apply)."""
        if _is_torch_cuda(x):
            import torch
            xx = x.reshape(-1).contiguous()
            torch.cuda.synchronize(xx.device)
            y = torch.empty_like(xx)
            check(_lib.tpl_op_apply(self._op, xx.data_ptr(), y.data_ptr(), _lib.TPL_MEM_DEVICE))
            return y
        xx = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
        y = np.empty_like(xx)
        check(_lib.tpl_op_apply(self._op, xx.ctypes.data, y.ctypes.data, _lib.TPL_MEM_HOST))
        return y

    # -- schedule / measurement ------------------------------------------------
    def schedule(self):
        """Device layout: dict(short_rows, long_rows, G2, E, slices, perm) — what the
        oracle needs to reproduce the device reduction order. Row lists are internal
        indices; perm[i] = the caller's row at internal position i (None: identity)."""
        ns, nl, g2, e = c_int32(), c_int32(), c_int32(), c_int64()
        check(_lib.tpl_op_schedule(self._op, byref(ns), byref(nl), byref(g2), byref(e), None, None))
        sr = np.zeros(max(ns.value, 1), dtype=np.int32)
        lr = np.zeros(max(nl.value, 1), dtype=np.int32)
        check(_lib.tpl_op_schedule(self._op, byref(ns), byref(nl), byref(g2), byref(e),
                                   sr.ctypes.data_as(POINTER(c_int32)),
                                   lr.ctypes.data_as(POINTER(c_int32))))
        sl = c_int32()
        check(_lib.tpl_op_slices(self._op, byref(sl)))
        n = int(_lib.tpl_op_nrows(self._op))
        perm = np.zeros(max(n, 1), dtype=np.int32)
        check(_lib.tpl_op_permutation(self._op, perm.ctypes.data_as(POINTER(c_int32))))
        perm = perm[:n]
        ident = bool(np.array_equal(perm, np.arange(n, dtype=np.int32)))
        return {"short_rows": sr[:ns.value].copy(), "long_rows": lr[:nl.value].copy(),
                "G2": g2.value, "E": e.value, "slices": sl.value,
                "perm": None if ident else perm.copy()}

    def tune_order(self, groups=None, iters: int = 100):
        """Time the pass-one and pass-two SpMV under each locality-order group count
        (default 12..20, 22, 24) and keep the fastest: -> (groups, microseconds)."""
        g = np.ascontiguousarray(groups if groups is not None else [], dtype=np.int32)
        chosen, us = c_int32(), c_double()
        check(_lib.tpl_op_tune_order(self._op, g.ctypes.data_as(POINTER(c_int32)) if g.size else None,
                                     int(g.size), int(iters), byref(chosen), byref(us)))
        return int(chosen.value), float(us.value)

    def set_order_groups(self, groups: int = 0):
        """Pin the locality order's group count (0: the default 16); deterministic, unlike
        tune_order (tpl_op_set_order_groups)."""
        check(_lib.tpl_op_set_order_groups(self._op, int(groups)))

    def order_groups(self) -> int:
        """Group count of the order the device holds (0: the caller's order)."""
        return int(_lib.tpl_op_order_groups(self._op))

    def set_reorder(self, mode=2):
        """Locality row order on the device (rebuilds the layout): False / 0 off,
        True / 1 on, 2 auto (default: on up to 2^20 rows). The caller's row order is
        kept at the boundary either way."""
        check(_lib.tpl_op_set_reorder(self._op, int(mode)))

    def set_schedule(self, short_row_max=0, max_g2=0):
        check(_lib.tpl_op_set_schedule(self._op, short_row_max, max_g2))

    def set_slices(self, slices=0):
        """Column slices of the long rows: 1, 2, 4, 8, or 0 for the auto rule."""
        check(_lib.tpl_op_set_slices(self._op, slices))

    def profile_kernel(self, kernel: int, iters: int = 200):
        """(avg microseconds per launch, algorithmic bytes per launch) via HIP events."""
        us, by = c_double(), c_double()
        check(_lib.tpl_profile_kernel(self._op, kernel, iters, byref(us), byref(by)))
        return us.value, by.value

    def reorth_second_passes(self) -> int:
        """Second Gram-Schmidt passes of the last re-orthogonalised lanczos_standard."""
        v = c_int64()
        check(_lib.tpl_op_reorth_second_passes(self._op, byref(v)))
        return int(v.value)

    def flags(self) -> int:
        """tpl_op_flags bits (include/tpl.h)."""
        return int(_lib.tpl_op_flags(self._op))

    def device_bytes(self) -> int:
        """Device memory the operator holds (layout, vectors, state, V_k once allocated)."""
        v = ctypes.c_uint64()
        check(_lib.tpl_op_device_bytes(self._op, ctypes.byref(v)))
        return int(v.value)

    def set_device_ftk(self, mode=2):
        """Built-in inv of lanczos_two_pass: 0 / False host (two graphs), 1 / True on the
        device, the whole solve one graph, 2 auto (default: device for k <= 128)."""
        check(_lib.tpl_op_set_device_ftk(self._op, int(mode)))

    def ftk_device(self, which: str, alphas, betas):
        """The device f(T_k) kernel alone ("inv" / "exp") on this operator's GPU:
        -> (y' = f(T_k) e_1, evaluated on the device?)."""
        a = np.ascontiguousarray(alphas, dtype=np.float64)
        b = np.ascontiguousarray(betas, dtype=np.float64)
        y = np.zeros(a.shape[0])
        on = ctypes.c_int()
        check(_lib.tpl_op_ftk_device(self._op, {"inv": 0, "exp": 1}[which],
                                     a.ctypes.data_as(POINTER(c_double)), a.shape[0],
                                     b.ctypes.data_as(POINTER(c_double)),
                                     y.ctypes.data_as(POINTER(c_double)), byref(on)))
        return y, bool(on.value)

    def enable_timing(self, on: bool = True):
        """Record HIP events inside the captured passes of later solves."""
        check(_lib.tpl_op_enable_timing(self._op, 1 if on else 0))

    def pass_timing(self):
        """-> (pass-one span us, pass-two step-launch span us, pass-two launches) of the
        last timed two-pass solve."""
        p1, p2, n2 = c_double(), c_double(), c_int64()
        check(_lib.tpl_op_pass_timing(self._op, byref(p1), byref(p2), byref(n2)))
        return p1.value, p2.value, n2.value

    def step_samples(self):
        """-> (k_p1_spmv us, k_p1_axpy us, samples): live in-graph durations of pass one's
        two kernels, averaged over the sampled steps of the last timed one-graph solve."""
        s, a, n = c_double(), c_double(), c_int32()
        check(_lib.tpl_op_step_samples(self._op, byref(s), byref(a), byref(n)))
        return s.value, a.value, n.value

    def algo_bytes(self, kernel: int) -> float:
        return float(_lib.tpl_kernel_algo_bytes(self._op, kernel))

    def close(self):
        if getattr(self, "_op", None):
            _lib.tpl_op_destroy(self._op)
            self._op = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return f"HipCsrOp(n={self._n}, nnz={self._nnz}, device={self.device})"


HostPlan.schedule = HipCsrOp.schedule


# -- the caller's own matrix as `operator` (the reference's call sites pass `&a.as_ref()`,
# src/bin/tradeoff.rs:268-284): upload on first use, re-use while its operand key is unchanged
KEY_SAMPLES = 4096  # words of each array the key's checksum samples (tpl_operand_key)
_uploaded = threading.local()


def operand_key(a) -> tuple:
    """include/tpl.h tpl_operand_key of a scipy CSR / CSC matrix's OWN arrays (no copy):
    (identity: the arrays' addresses and sizes and n, checksum of the first and last 8 and
    KEY_SAMPLES evenly spaced words of each) — O(KEY_SAMPLES) host work, not O(nnz)."""
    ip, ix, v = a.indptr, a.indices, a.data
    for arr in (ip, ix):
        if arr.dtype.itemsize not in (4, 8) or not arr.flags.c_contiguous:
            raise TypeError("index arrays must be contiguous 32- or 64-bit integers")
    if v.dtype != np.float64 or not v.flags.c_contiguous:
        raise TypeError("values must be a contiguous float64 array")
    key = (ctypes.c_uint64 * 2)()
    check(_lib.tpl_operand_key(int(a.shape[0]), ip.ctypes.data, ip.size, ip.dtype.itemsize,
                               ix.ctypes.data, ix.size, ix.dtype.itemsize,
                               v.ctypes.data_as(POINTER(c_double)), v.size, KEY_SAMPLES, key))
    return (int(key[0]), int(key[1]))


def _upload(a, device: int) -> "HipCsrOp":
    return HipCsrOp(a, device=device)


def as_operator(operator, device: int = 0) -> "HipCsrOp":
    """A solver's `operator`: a HipCsrOp as is (the zero-overhead form), or a scipy sparse
    matrix uploaded on first use and re-used on this thread while its operand key is
    unchanged (the Rust shim's `HipOperand for SparseColMatRef` rule,
    integration/rust/hip.rs). After changing a matrix's values IN PLACE call
    ``refresh_uploaded()``: the key sees new arrays, sizes and sampled words, not every word."""
    if isinstance(operator, HipCsrOp):
        return operator
    import scipy.sparse as sp
    if not sp.issparse(operator) or operator.format not in ("csr", "csc"):
        raise TypeError("operator must be a tpl_amd.HipCsrOp or a scipy CSR / CSC matrix")
    key = operand_key(operator)
    slot = getattr(_uploaded, "slot", None)
    if slot is None or slot[0] != key:
        _uploaded.slot = None  # free the previous upload before the new one
        _uploaded.slot = (key, _upload(operator, device))
    return _uploaded.slot[1]


def refresh_uploaded() -> None:
    """Forget this thread's upload of a caller's matrix: the next call uploads it again."""
    _uploaded.slot = None
