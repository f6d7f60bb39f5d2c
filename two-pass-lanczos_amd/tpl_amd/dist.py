"""Row-partitioned operator over several GPUs (include/tpl.h).

One process per GPU. Rank r owns the rows [starts[r], starts[r+1]) of A (contiguous
blocks balanced by algorithmic bytes, ``partition``); each SpMV all-gathers the
vector in place over RCCL/xGMI — the whole blocks ("rows") or only the rows another
rank references ("halo") — and alpha/beta combine the ranks' totals in rank
order, so every rank holds the same alpha, beta and steps bit for bit. The solver
entry points (``tpl_amd.lanczos_two_pass``, ``algorithms.*``) take a ``DistHipCsrOp``
unchanged; ``b`` and the returned ``x`` are then this rank's block of rows.

Transports: ``"rccl"`` (the product path; the RCCL unique id is broadcast with
torch.distributed) and ``"host"`` (tests: all-gathers through torch.distributed on
host memory, eager launches) — e.g. several ranks sharing one GPU.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_double, c_int32, c_int64, c_void_p

import numpy as np

from . import _lib
from .error import check
from .operator import HipCsrOp, _as_csr_arrays


def halo_width(a, starts) -> int:
    """H = max over ranks q of |B_q|, B_q = the rows of q's block [starts[q], starts[q+1])
    that a row of another block references: the doubles per rank a halo all-gather moves
    (tpl_dist_op_create_halo computes the same on the host side of the ABI)."""
    n, rp, ci, _ = _as_csr_arrays(a)
    starts = np.asarray(starts, dtype=np.int64)
    row_owner = np.repeat(np.searchsorted(starts, np.arange(n), "right") - 1, np.diff(rp))
    col_owner = np.searchsorted(starts, ci, "right") - 1
    need = np.unique(ci[row_owner != col_owner])
    if need.size == 0:
        return 0
    return int(np.bincount(np.searchsorted(starts, need, "right") - 1,
                           minlength=len(starts) - 1).max())


_MODE_NAMES = {_lib.TPL_PLAN_REPLICATED: "replicated", _lib.TPL_PLAN_ROWS: "rows",
               _lib.TPL_PLAN_HALO: "halo"}


def choose_partition(a, nranks: int) -> str:
    """The partition mode="auto" takes for `nranks` ranks (tpl_dist_choose_partition, the
    rule every binding shares; host only): "replicated", "halo" or "rows"."""
    n, rp, ci, _ = _as_csr_arrays(a)
    m = ctypes.c_int()
    check(_lib.tpl_dist_choose_partition(n, rp.ctypes.data_as(POINTER(c_int64)),
                                         ci.ctypes.data_as(POINTER(c_int32)), int(nranks),
                                         byref(m)))
    return _MODE_NAMES[m.value]


def partition(a, nranks: int) -> np.ndarray:
    """starts[nranks + 1] of the byte-balanced contiguous row blocks (tpl_dist_partition)."""
    n, rp, _, _ = _as_csr_arrays(a)
    starts = np.zeros(nranks + 1, dtype=np.int64)
    check(_lib.tpl_dist_partition(n, rp.ctypes.data_as(POINTER(c_int64)), nranks,
                                  starts.ctypes.data_as(POINTER(c_int64))))
    return starts


class DistContext:
    """This process's rank of a partitioned solve (tpl_dist_create / _create_host)."""

    def __init__(self, rank: int, world: int, device: int = 0, transport: str = "rccl",
                 group=None):
        import torch.distributed as tdist
        self.rank, self.world, self.device, self.transport = rank, world, device, transport
        h = c_void_p()
        if transport == "rccl":
            idb = (ctypes.c_uint8 * _lib.TPL_DIST_ID_BYTES)()
            if rank == 0:
                check(_lib.tpl_dist_unique_id(idb))
            obj = [bytes(idb) if rank == 0 else None]
            tdist.broadcast_object_list(obj, src=0, group=group)
            ctypes.memmove(idb, obj[0], _lib.TPL_DIST_ID_BYTES)
            check(_lib.tpl_dist_create(device, rank, world, idb, byref(h)))
        elif transport == "host":
            import torch

            def allgather(send, recv, nbytes, _user):
                try:
                    src = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)),
                                           dtype=torch.uint8)
                    parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                    tdist.all_gather(parts, src.clone(), group=group)
                    out = torch.cat(parts).numpy()
                    ctypes.memmove(recv, out.ctypes.data, nbytes * world)
                    return 0
                except Exception:  # pragma: no cover - reported as a device error
                    return 1

            self._cb = _lib.ALLGATHER_FN(allgather)  # keep alive
            check(_lib.tpl_dist_create_host(device, rank, world, self._cb, None, byref(h)))
        else:
            raise ValueError(f"unknown transport {transport!r}")
        self._d = h.value

    @property
    def handle(self) -> int:
        return self._d

    def close(self):
        if getattr(self, "_d", None):
            _lib.tpl_dist_destroy(self._d)
            self._d = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class DistHipCsrOp(HipCsrOp):
    """This rank's part of a symmetric A, resident in its GPU's HBM.

    mode "replicated" (tpl_dist_op_create_replicated): short rows in byte-balanced
    blocks, long rows replicated on every rank, n_long partials exchanged per SpMV;
    mode "rows" (tpl_dist_op_create_csr): contiguous row blocks, the whole vector
    all-gathered per SpMV; mode "halo" (tpl_dist_op_create_halo): the same blocks and
    bits, only the rows another rank references all-gathered (``halo_width`` per rank);
    "auto" (tpl_dist_op_create_auto, the rule the C++ and Rust bindings share):
    replicated when the matrix allows it (no short row references another rank's short
    rows — the KKT case), else halo when its width is at most half the widest block (a
    banded or mesh-like matrix), else rows.
    ``local_rows``: global row of each entry of this rank's vectors (``local(v)``).
    """

    def __init__(self, a, ctx: DistContext, starts=None, mode: str = "auto"):
        n, rp, ci, v = _as_csr_arrays(a)
        self.device = ctx.device
        self.dist = ctx
        self.n_global = n
        h = c_void_p()
        self.mode = None
        if mode == "auto" and starts is None:
            m = ctypes.c_int()
            check(_lib.tpl_dist_op_create_auto(
                ctx.handle, n, rp.ctypes.data_as(POINTER(c_int64)),
                ci.ctypes.data_as(POINTER(c_int32)), v.ctypes.data_as(POINTER(c_double)),
                byref(h), byref(m)))
            self.mode = _MODE_NAMES[m.value]
            if self.mode != "replicated":
                self.starts = partition((n, rp, ci, v), ctx.world)
        if mode == "replicated" and starts is None:
            st = _lib.tpl_dist_op_create_replicated(
                ctx.handle, n, rp.ctypes.data_as(POINTER(c_int64)),
                ci.ctypes.data_as(POINTER(c_int32)), v.ctypes.data_as(POINTER(c_double)),
                byref(h))
            if st == _lib.TPL_OK:
                self.mode = "replicated"
            else:
                check(st)
        if self.mode is None:
            self.starts = (partition((n, rp, ci, v), ctx.world) if starts is None
                           else np.ascontiguousarray(starts, dtype=np.int64))
        if self.mode is None and mode in ("auto", "halo"):
            # explicit starts: halo when asked, or (auto) when it is at most half the widest
            # block — tpl_dist_choose_partition's rule over the caller's split
            if mode == "halo" or 2 * halo_width((n, rp, ci, v), self.starts) <= int(
                    np.diff(self.starts).max()):
                check(_lib.tpl_dist_op_create_halo(
                    ctx.handle, n, self.starts.ctypes.data_as(POINTER(c_int64)),
                    rp.ctypes.data_as(POINTER(c_int64)), ci.ctypes.data_as(POINTER(c_int32)),
                    v.ctypes.data_as(POINTER(c_double)), byref(h)))
                self.mode = "halo"
        if self.mode is None:
            if mode not in ("auto", "rows"):
                raise ValueError(f"unknown partition mode {mode!r}")
            r0, r1 = int(self.starts[ctx.rank]), int(self.starts[ctx.rank + 1])
            lrp = np.ascontiguousarray(rp[r0:r1 + 1] - rp[r0], dtype=np.int64)
            lci = np.ascontiguousarray(ci[rp[r0]:rp[r1]], dtype=np.int32)
            lv = np.ascontiguousarray(v[rp[r0]:rp[r1]], dtype=np.float64)
            check(_lib.tpl_dist_op_create_csr(
                ctx.handle, n, self.starts.ctypes.data_as(POINTER(c_int64)),
                lrp.ctypes.data_as(POINTER(c_int64)), lci.ctypes.data_as(POINTER(c_int32)),
                lv.ctypes.data_as(POINTER(c_double)), byref(h)))
            self.mode = "rows"
        self._op = h.value
        self._n = int(_lib.tpl_op_nrows(self._op))
        self._nnz = int(_lib.tpl_op_nnz(self._op))
        self.local_rows = np.zeros(max(self._n, 1), dtype=np.int64)
        check(_lib.tpl_op_local_rows(self._op, self.local_rows.ctypes.data_as(POINTER(c_int64))))
        self.local_rows = self.local_rows[:self._n]

    def ncols(self) -> int:
        return self.n_global

    def local(self, v):
        """This rank's entries of a global vector."""
        return v[self.local_rows]
