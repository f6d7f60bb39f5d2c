"""f(T_k) e_1 reference solvers via LAPACK (scipy) — TEST INFRASTRUCTURE (oracle).

Restate the reference harness closures on the projected tridiagonal T_k:
  inv: src/bin/tradeoff.rs:245-258 / src/bin/stability.rs:161-170 (sparse LU),
       tests/correctness.rs:171-179 (dense partial-pivot LU)  -> LAPACK dgtsv
  exp: src/bin/stability.rs:175-193, tests/correctness.rs:215-240
       (Q exp(Lambda) Q^T e_1 from a self-adjoint EVD)          -> LAPACK dstev
  sq : tests/correctness.rs:287-299 (T_k^2 e_1)
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import eigh_tridiagonal
from scipy.linalg.lapack import dgtsv


def tridiag(alphas, betas) -> np.ndarray:
    k = len(alphas)
    t = np.diag(np.asarray(alphas, dtype=np.float64))
    if k > 1:
        t += np.diag(betas[:k - 1], 1) + np.diag(betas[:k - 1], -1)
    return t


def inv(alphas, betas) -> np.ndarray:
    k = len(alphas)
    if k == 0:
        return np.zeros(0)
    if k == 1:
        return np.array([1.0 / float(alphas[0])])
    e1 = np.zeros(k)
    e1[0] = 1.0
    b = np.asarray(betas[:k - 1], dtype=np.float64)
    _, _, _, x, info = dgtsv(b.copy(), np.asarray(alphas, dtype=np.float64).copy(), b.copy(), e1)
    if info != 0:
        return np.full(k, np.nan)
    return x


def exp(alphas, betas) -> np.ndarray:
    k = len(alphas)
    if k == 0:
        return np.zeros(0)
    if k == 1:
        return np.array([np.exp(float(alphas[0]))])
    d = np.asarray(alphas, dtype=np.float64)
    e = np.asarray(betas[:k - 1], dtype=np.float64)
    try:
        lam, q = eigh_tridiagonal(d, e)
    except np.linalg.LinAlgError:
        # dstemr (MRRR) gives up on some large zero-diagonal KKT projections (k = 500
        # on the 500k instance); implicit QL/QR (dstev) is the classical fallback
        lam, q = eigh_tridiagonal(d, e, lapack_driver="stev")
    return q @ (np.exp(lam) * q[0, :])


def sq(alphas, betas) -> np.ndarray:
    t = tridiag(alphas, betas)
    if t.shape[0] == 0:
        return np.zeros(0)
    return (t @ t)[:, 0]


SOLVERS = {"inv": inv, "exp": exp, "sq": sq}
