"""Error types — mirror of the reference's ``src/error.rs`` (LanczosError /
LanczosErrorKind, :11-58) and ``src/utils/data_loader.rs`` (DataLoaderError, :16-43).

``str(err)`` is exactly the reference's ``Display`` text, and equality compares the
kind and payload like the reference's ``PartialEq`` (src/error.rs:62-66).
"""
from __future__ import annotations

import enum

from . import _lib


class LanczosErrorKind(enum.Enum):
    BREAKDOWN = "Breakdown"                    # declared, never constructed by the reference
    DIMENSION_MISMATCH = "DimensionMismatch"   # reference panics instead (faer); we report
    INPUT_ERROR = "InputError"
    PARAMETER_MISMATCH = "ParameterMismatch"
    EVD_ERROR = "EvdError"
    SOLVER_ERROR = "SolverError"


class LanczosError(Exception):
    """``LanczosError(LanczosErrorKind)``; ``str()`` follows src/error.rs:20-58."""

    def __init__(self, kind: LanczosErrorKind, message: str, payload=None):
        super().__init__(message)
        self.kind = kind
        self.message = message
        self.payload = payload

    def __str__(self) -> str:
        return self.message

    def __eq__(self, other) -> bool:
        return (isinstance(other, LanczosError) and self.kind == other.kind
                and self.message == other.message)

    def __hash__(self):
        return hash((self.kind, self.message))

    # -- constructors with the reference's #[error(...)] formats -----------------
    @classmethod
    def breakdown(cls, k: int) -> "LanczosError":
        return cls(LanczosErrorKind.BREAKDOWN,
                   f"Lanczos iteration breakdown at step {k}: Beta coefficient is zero. "
                   "The Krylov subspace is invariant.", {"k": k})

    @classmethod
    def dimension_mismatch(cls, operator_cols: int, vector_rows: int) -> "LanczosError":
        return cls(LanczosErrorKind.DIMENSION_MISMATCH,
                   f"Dimension mismatch: operator has {operator_cols} columns but vector has "
                   f"{vector_rows} rows.", {"operator_cols": operator_cols,
                                             "vector_rows": vector_rows})

    @classmethod
    def input_error(cls, what: str) -> "LanczosError":
        return cls(LanczosErrorKind.INPUT_ERROR, f"Invalid input parameter: {what}", what)

    @classmethod
    def parameter_mismatch(cls, param_name: str, expected: int, actual: int) -> "LanczosError":
        return cls(LanczosErrorKind.PARAMETER_MISMATCH,
                   f"Parameter mismatch: `{param_name}` expects size {expected}, but got {actual}.",
                   {"param_name": param_name, "expected": expected, "actual": actual})

    @classmethod
    def evd_error(cls, err: str) -> "LanczosError":
        return cls(LanczosErrorKind.EVD_ERROR,
                   f"A numerical error occurred during the eigendecomposition of T_k: {err}", err)

    @classmethod
    def solver_error(cls, err: str) -> "LanczosError":
        return cls(LanczosErrorKind.SOLVER_ERROR,
                   f"The user-provided f(T_k) solver failed: {err}", err)


class TplError(RuntimeError):
    """Engine failure with no LanczosErrorKind counterpart (bad argument, HIP error)."""

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class DataLoaderError(Exception):
    """``DataLoaderError`` (src/utils/data_loader.rs:16-43); ``str()`` is its Display."""


_KIND_OF_STATUS = {
    _lib.TPL_ERR_BREAKDOWN: LanczosErrorKind.BREAKDOWN,
    _lib.TPL_ERR_DIMENSION_MISMATCH: LanczosErrorKind.DIMENSION_MISMATCH,
    _lib.TPL_ERR_INPUT: LanczosErrorKind.INPUT_ERROR,
    _lib.TPL_ERR_PARAMETER_MISMATCH: LanczosErrorKind.PARAMETER_MISMATCH,
    _lib.TPL_ERR_EVD: LanczosErrorKind.EVD_ERROR,
    _lib.TPL_ERR_SOLVER: LanczosErrorKind.SOLVER_ERROR,
}


def from_detail(d: dict) -> "LanczosError":
    """Rebuild the LanczosErrorKind variant from tpl_last_error_detail's fields (not by
    parsing the message): the same constructors a Rust binding uses."""
    st = d["status"]
    if st == _lib.TPL_ERR_INPUT:
        return LanczosError.input_error(d["inner"])
    if st == _lib.TPL_ERR_PARAMETER_MISMATCH:
        return LanczosError.parameter_mismatch(d["param_name"], d["expected"], d["actual"])
    if st == _lib.TPL_ERR_DIMENSION_MISMATCH:
        return LanczosError.dimension_mismatch(d["operator_cols"], d["vector_rows"])
    if st == _lib.TPL_ERR_SOLVER:
        return LanczosError.solver_error(d["inner"])
    if st == _lib.TPL_ERR_EVD:
        return LanczosError.evd_error(d["inner"])
    if st == _lib.TPL_ERR_BREAKDOWN:
        return LanczosError.breakdown(d["breakdown_step"])
    raise ValueError(f"status {st} is not a LanczosErrorKind")


def check(status: int) -> None:
    """Raise the Python mirror of a non-zero tpl_status."""
    if status == _lib.TPL_OK:
        return
    msg = _lib.last_error()
    if status in _KIND_OF_STATUS:
        err = from_detail(_lib.last_error_detail())
        if err.message != msg:  # the fields must reproduce the engine's Display text
            raise TplError(_lib.TPL_ERR_INVALID_ARGUMENT,
                           f"error detail does not match the message: {err.message!r} != {msg!r}")
        raise err
    if status == _lib.TPL_ERR_DATA_LOADER:
        raise DataLoaderError(msg)
    raise TplError(status, msg)
