"""ctypes binding of libtpl_amd.so (the C ABI declared in include/tpl.h).

The shared library is built in-tree by ``make -C two-pass-lanczos_amd/csrc`` (or
``__graft_entry__.build()``). There is deliberately NO fallback: if the library is
missing, importing the package raises, so a GPU run can never silently use a
CPU path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, c_char, c_char_p, c_double, c_int, c_int32,
                    c_int64, c_size_t, c_void_p)

LIB_PATH = os.environ.get("TPL_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libtpl_amd.so")  # override: experiments only

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"tpl_amd: {LIB_PATH} is missing — build it with `make -C two-pass-lanczos_amd/csrc` "
        "(or __graft_entry__.build()); there is no CPU fallback")

# PyTorch-ROCm wheels bundle their own libamdhip64 / libhsa-runtime64 (same SONAMEs
# as /opt/rocm's). Whichever is loaded first wins the SONAME; loading ours first makes
# torch pull in a SECOND HIP runtime that cannot see the GPU. Importing torch first
# (when installed) keeps exactly one HIP runtime in the process, shared by torch
# (device buffers, torch.distributed) and libtpl_amd.so.
try:  # pragma: no cover - environment dependent
    import torch  # noqa: F401
except ImportError:
    pass

lib = ctypes.CDLL(LIB_PATH)

# status codes (tpl_status)
TPL_OK = 0
TPL_ERR_BREAKDOWN = 1
TPL_ERR_DIMENSION_MISMATCH = 2
TPL_ERR_INPUT = 3
TPL_ERR_PARAMETER_MISMATCH = 4
TPL_ERR_EVD = 5
TPL_ERR_SOLVER = 6
TPL_ERR_INVALID_ARGUMENT = 100
TPL_ERR_DEVICE = 101
TPL_ERR_OUT_OF_MEMORY = 102
TPL_ERR_DATA_LOADER = 103
TPL_ERR_UNSUPPORTED = 104

TPL_MEM_HOST = 0
TPL_MEM_DEVICE = 1

TPL_KERNEL_PASS1_SPMV = 0
TPL_KERNEL_PASS1_AXPY = 1
TPL_KERNEL_PASS2_SPMV = 2
TPL_KERNEL_SPMV = 3
TPL_KERNEL_EXCHANGE_P1 = 4
TPL_KERNEL_EXCHANGE_P2 = 5
TPL_KERNEL_PASS1_STEP = 6

PD = POINTER(c_double)

FTK_FN = CFUNCTYPE(c_int, PD, c_size_t, PD, c_size_t, PD, c_size_t, POINTER(c_size_t),
                   POINTER(c_char), c_size_t, c_void_p)
STEP_CB = CFUNCTYPE(c_int, c_size_t, c_void_p, c_int64, PD, c_size_t, PD, c_size_t, c_void_p)


class CsrHost(ctypes.Structure):
    _fields_ = [("n", c_int64), ("nnz", c_int64), ("num_nodes", c_int64), ("num_arcs", c_int64),
                ("row_ptr", POINTER(c_int64)), ("col_idx", POINTER(c_int32)),
                ("vals", PD)]


def _sig(name, restype, *argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = list(argtypes)
    return fn


tpl_last_error = _sig("tpl_last_error", c_char_p)
tpl_version = _sig("tpl_version", c_char_p)
tpl_device_count = _sig("tpl_device_count", c_int)
tpl_ctx_create = _sig("tpl_ctx_create", c_int, c_int, POINTER(c_void_p))
tpl_ctx_destroy = _sig("tpl_ctx_destroy", c_int, c_void_p)
tpl_ctx_synchronize = _sig("tpl_ctx_synchronize", c_int, c_void_p)
tpl_op_create_csr = _sig("tpl_op_create_csr", c_int, c_void_p, c_int64, c_int64,
                         POINTER(c_int64), POINTER(c_int32), PD, POINTER(c_void_p))
tpl_op_destroy = _sig("tpl_op_destroy", c_int, c_void_p)
tpl_op_nrows = _sig("tpl_op_nrows", c_int64, c_void_p)
tpl_op_nnz = _sig("tpl_op_nnz", c_int64, c_void_p)
tpl_op_flags = _sig("tpl_op_flags", c_int, c_void_p)
tpl_op_set_value_format = _sig("tpl_op_set_value_format", c_int, c_void_p, c_int)
tpl_op_apply = _sig("tpl_op_apply", c_int, c_void_p, c_void_p, c_void_p, c_int)
tpl_lanczos = _sig("tpl_lanczos", c_int, c_void_p, c_void_p, c_int64, c_size_t, c_void_p,
                   c_void_p, c_void_p, c_int)
tpl_lanczos_two_pass = _sig("tpl_lanczos_two_pass", c_int, c_void_p, c_void_p, c_int64,
                            c_size_t, c_void_p, c_void_p, c_void_p, c_int)
tpl_lanczos_standard = _sig("tpl_lanczos_standard", c_int, c_void_p, c_void_p, c_int64, c_size_t,
                            PD, PD, POINTER(c_size_t), PD, c_void_p, c_int, c_int, c_void_p,
                            c_void_p)
tpl_lanczos_pass_one = _sig("tpl_lanczos_pass_one", c_int, c_void_p, c_void_p, c_int64, c_size_t,
                            PD, PD, POINTER(c_size_t), PD, c_int)
tpl_lanczos_pass_two = _sig("tpl_lanczos_pass_two", c_int, c_void_p, c_void_p, c_int64, PD,
                            c_size_t, PD, c_size_t, c_size_t, c_double, PD, c_size_t, c_void_p,
                            c_void_p, c_int)
tpl_load_kkt_system = _sig("tpl_load_kkt_system", c_int, c_char_p, c_char_p, POINTER(CsrHost))
tpl_csr_host_free = _sig("tpl_csr_host_free", None, POINTER(CsrHost))
tpl_generate_kkt = _sig("tpl_generate_kkt", c_int, c_int64, c_int64, ctypes.c_uint64,
                        POINTER(CsrHost))
tpl_op_schedule = _sig("tpl_op_schedule", c_int, c_void_p, POINTER(c_int32), POINTER(c_int32),
                       POINTER(c_int32), POINTER(c_int64), POINTER(c_int32), POINTER(c_int32))
tpl_op_set_schedule = _sig("tpl_op_set_schedule", c_int, c_void_p, c_int32, c_int32)
tpl_op_slices = _sig("tpl_op_slices", c_int, c_void_p, POINTER(c_int32))
tpl_op_set_slices = _sig("tpl_op_set_slices", c_int, c_void_p, c_int32)
tpl_profile_kernel = _sig("tpl_profile_kernel", c_int, c_void_p, c_int, c_int, PD, PD)
tpl_kernel_algo_bytes = _sig("tpl_kernel_algo_bytes", c_double, c_void_p, c_int)
tpl_copy_to_host = _sig("tpl_copy_to_host", c_int, c_void_p, c_void_p, c_size_t)
tpl_op_enable_timing = _sig("tpl_op_enable_timing", c_int, c_void_p, c_int)
tpl_op_pass_timing = _sig("tpl_op_pass_timing", c_int, c_void_p, PD, PD, POINTER(c_int64))
tpl_op_step_samples = _sig("tpl_op_step_samples", c_int, c_void_p, PD, PD, POINTER(c_int32))
tpl_op_set_device_ftk = _sig("tpl_op_set_device_ftk", c_int, c_void_p, c_int)
tpl_op_device_bytes = _sig("tpl_op_device_bytes", c_int, c_void_p, POINTER(ctypes.c_uint64))
tpl_op_set_reorder = _sig("tpl_op_set_reorder", c_int, c_void_p, c_int)
tpl_op_permutation = _sig("tpl_op_permutation", c_int, c_void_p, POINTER(c_int32))
tpl_op_tune_order = _sig("tpl_op_tune_order", c_int, c_void_p, POINTER(c_int32), c_int32,
                         c_int32, POINTER(c_int32), POINTER(c_double))
tpl_locality_order = _sig("tpl_locality_order", c_int, c_int64, POINTER(c_int64),
                          POINTER(c_int32), c_int32, c_int32, POINTER(c_int32),
                          POINTER(c_int32))
tpl_op_reorth_second_passes = _sig("tpl_op_reorth_second_passes", c_int, c_void_p, POINTER(c_int64))
tpl_op_ftk_device = _sig("tpl_op_ftk_device", c_int, c_void_p, c_int, PD, c_size_t, PD, PD,
                         POINTER(c_int))
tpl_op_set_order_groups = _sig("tpl_op_set_order_groups", c_int, c_void_p, c_int32)
tpl_op_order_groups = _sig("tpl_op_order_groups", c_int32, c_void_p)


class ErrorDetail(ctypes.Structure):
    """tpl_error_detail: the fields of the last failing call's LanczosErrorKind."""
    _fields_ = [("status", c_int32), ("message", c_char_p), ("inner", c_char_p),
                ("param_name", c_char_p), ("expected", ctypes.c_uint64),
                ("actual", ctypes.c_uint64), ("operator_cols", ctypes.c_uint64),
                ("vector_rows", ctypes.c_uint64), ("breakdown_step", ctypes.c_uint64)]


tpl_last_error_detail = _sig("tpl_last_error_detail", c_int, POINTER(ErrorDetail))

# built-in f(T_k) solvers: raw C function pointers usable as tpl_ftk_fn
FTK_INV_PTR = ctypes.cast(lib.tpl_ftk_inv, c_void_p).value
FTK_EXP_PTR = ctypes.cast(lib.tpl_ftk_exp, c_void_p).value
FTK_SQ_PTR = ctypes.cast(lib.tpl_ftk_sq, c_void_p).value
tpl_ftk_inv = _sig("tpl_ftk_inv", c_int, PD, c_size_t, PD, c_size_t, PD, c_size_t,
                   POINTER(c_size_t), POINTER(c_char), c_size_t, c_void_p)
tpl_ftk_exp = _sig("tpl_ftk_exp", c_int, PD, c_size_t, PD, c_size_t, PD, c_size_t,
                   POINTER(c_size_t), POINTER(c_char), c_size_t, c_void_p)
tpl_ftk_sq = _sig("tpl_ftk_sq", c_int, PD, c_size_t, PD, c_size_t, PD, c_size_t,
                  POINTER(c_size_t), POINTER(c_char), c_size_t, c_void_p)

# Every symbol include/tpl.h declares (checked by tests/test_boundary.py).
EXPORTED = [
    "tpl_last_error", "tpl_version", "tpl_ctx_create", "tpl_ctx_destroy", "tpl_ctx_synchronize",
    "tpl_device_count", "tpl_op_create_csr", "tpl_op_destroy", "tpl_op_nrows", "tpl_op_nnz",
    "tpl_op_apply", "tpl_ftk_inv", "tpl_ftk_exp", "tpl_ftk_sq", "tpl_lanczos",
    "tpl_lanczos_two_pass", "tpl_lanczos_standard", "tpl_lanczos_pass_one",
    "tpl_lanczos_pass_two", "tpl_load_kkt_system", "tpl_csr_host_free", "tpl_op_schedule",
    "tpl_op_set_schedule", "tpl_op_slices", "tpl_op_set_slices", "tpl_profile_kernel", "tpl_kernel_algo_bytes", "tpl_copy_to_host",
    "tpl_op_enable_timing", "tpl_op_pass_timing", "tpl_op_step_samples", "tpl_generate_kkt", "tpl_op_flags",
    "tpl_op_set_value_format", "tpl_op_set_device_ftk",
    "tpl_op_device_bytes", "tpl_op_reorth_second_passes", "tpl_op_set_reorder",
    "tpl_op_permutation", "tpl_locality_order", "tpl_op_tune_order",
    "tpl_last_error_detail", "tpl_op_set_order_groups", "tpl_op_order_groups",
    "tpl_op_ftk_device",
]


def last_error() -> str:
    m = tpl_last_error()
    return m.decode("utf-8", "replace") if m else ""


def last_error_detail() -> dict:
    """tpl_last_error_detail as a dict (strings decoded)."""
    d = ErrorDetail()
    if tpl_last_error_detail(ctypes.byref(d)) != TPL_OK:
        raise RuntimeError("tpl_last_error_detail failed")
    dec = (lambda b: b.decode("utf-8", "replace") if b else "")
    return {"status": d.status, "message": dec(d.message), "inner": dec(d.inner),
            "param_name": dec(d.param_name), "expected": int(d.expected),
            "actual": int(d.actual), "operator_cols": int(d.operator_cols),
            "vector_rows": int(d.vector_rows), "breakdown_step": int(d.breakdown_step)}

# row-partitioned operator (include/tpl.h, "row-partitioned operator over several GPUs")
TPL_DIST_ID_BYTES = 128
ALLGATHER_FN = CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, c_void_p)
tpl_dist_partition = _sig("tpl_dist_partition", c_int, c_int64, POINTER(c_int64), c_int,
                          POINTER(c_int64))
tpl_dist_unique_id = _sig("tpl_dist_unique_id", c_int, POINTER(ctypes.c_uint8))
tpl_dist_create = _sig("tpl_dist_create", c_int, c_int, c_int, c_int, POINTER(ctypes.c_uint8),
                       POINTER(c_void_p))
tpl_dist_create_host = _sig("tpl_dist_create_host", c_int, c_int, c_int, c_int, ALLGATHER_FN,
                            c_void_p, POINTER(c_void_p))
tpl_dist_destroy = _sig("tpl_dist_destroy", c_int, c_void_p)
tpl_dist_op_create_csr = _sig("tpl_dist_op_create_csr", c_int, c_void_p, c_int64, POINTER(c_int64),
                              POINTER(c_int64), POINTER(c_int32), PD, POINTER(c_void_p))
tpl_dist_op_create_replicated = _sig("tpl_dist_op_create_replicated", c_int, c_void_p, c_int64,
                                     POINTER(c_int64), POINTER(c_int32), PD, POINTER(c_void_p))
tpl_dist_op_create_halo = _sig("tpl_dist_op_create_halo", c_int, c_void_p, c_int64, POINTER(c_int64),
                               POINTER(c_int64), POINTER(c_int32), PD, POINTER(c_void_p))
tpl_op_local_rows = _sig("tpl_op_local_rows", c_int, c_void_p, POINTER(c_int64))
tpl_dist_choose_partition = _sig("tpl_dist_choose_partition", c_int, c_int64, POINTER(c_int64),
                                 POINTER(c_int32), c_int, POINTER(c_int))
tpl_dist_op_create_auto = _sig("tpl_dist_op_create_auto", c_int, c_void_p, c_int64,
                               POINTER(c_int64), POINTER(c_int32), PD, POINTER(c_void_p),
                               POINTER(c_int))
tpl_operand_key = _sig("tpl_operand_key", c_int, c_int64, c_void_p, c_size_t, c_size_t, c_void_p,
                       c_size_t, c_size_t, PD, c_size_t, c_size_t, POINTER(ctypes.c_uint64))
# host-only plans (include/tpl.h "host-only plans")
TPL_PLAN_SINGLE, TPL_PLAN_REPLICATED, TPL_PLAN_ROWS, TPL_PLAN_HALO = 0, 1, 2, 3
tpl_plan_create = _sig("tpl_plan_create", c_int, c_int64, POINTER(c_int64), POINTER(c_int32), PD,
                       c_int, c_int, c_int, c_int32, POINTER(c_void_p))
EXPORTED += ["tpl_plan_create"]
EXPORTED += ["tpl_dist_op_create_replicated", "tpl_op_local_rows", "tpl_dist_partition", "tpl_dist_unique_id", "tpl_dist_create",
             "tpl_dist_create_host", "tpl_dist_destroy", "tpl_dist_op_create_csr",
             "tpl_dist_op_create_halo", "tpl_dist_choose_partition", "tpl_dist_op_create_auto",
             "tpl_operand_key"]
