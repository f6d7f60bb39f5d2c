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


def exp_chebyshev(alphas, betas, shifts: int = 256) -> np.ndarray:
    """Restatement of the device exp (two-pass-lanczos_amd/csrc/tpl_kernels.hip k_ftk_exp)
    in numpy — TEST INFRASTRUCTURE: it checks the algorithm (Sturm multisection bracket,
    Debye-sized Chebyshev expansion, Clenshaw + Miller's backward Bessel recurrence)
    against LAPACK on the CPU; the device's bits are not reproduced (libm exp/asinh differ).
    One round of 2 * shifts Sturm shifts over the Gershgorin interval serves both ends.
    Returns y' = exp(T) e_1, or None where the device hands the case back to the host."""
    al = np.asarray(alphas, dtype=np.float64)
    n = len(al)
    be = np.zeros(n)
    be[:n - 1] = np.asarray(betas[:n - 1], dtype=np.float64)
    if not (np.all(np.isfinite(al)) and np.all(np.isfinite(be))):
        return None
    if n == 1:
        return np.array([np.exp(al[0])])
    bl = np.concatenate([[0.0], be[:n - 1]])
    rad = np.abs(bl) + np.abs(be)
    glo, ghi = float(np.min(al - rad)), float(np.max(al + rad))
    pivmin = 2.2250738585072014e-308 * max(1.0, float(np.max(be * be)))

    def count(sig):
        q = al[0] - sig
        if abs(q) < pivmin:
            q = -pivmin
        c = int(q < 0)
        for i in range(1, n):
            q = (al[i] - sig) - (be[i - 1] * be[i - 1]) / q
            if abs(q) < pivmin:
                q = -pivmin
            c += int(q < 0)
        return c

    w = (ghi - glo) / (2 * shifts + 1)
    cnts = [count(glo + w * (s + 1)) for s in range(2 * shifts)]
    f0 = next((s for s in range(2 * shifts) if cnts[s] >= 1), 2 * shifts)
    f1 = next((s for s in range(2 * shifts) if cnts[s] >= n), 2 * shifts)
    lo_b = glo + w * f0 if f0 > 0 else glo
    hi_b = glo + w * (f1 + 1) if f1 < 2 * shifts else ghi
    scale = max(abs(glo), abs(ghi))
    a = lo_b - 1e-9 * (1.0 + scale)
    b = hi_b + 1e-9 * (1.0 + scale)
    c = 0.5 * (a + b)
    r = max(0.5 * (b - a), 1e-30 * (1.0 + abs(c)))

    def lsi(m):
        s = np.sqrt(m * m + r * r)
        return -r + s - m * np.arcsinh(m / r) - 0.9189385332046727 - 0.25 * np.log(s * s)

    lo_m, hi_m = 0, 16384
    if lsi(hi_m) >= -50.66:
        return None
    while lo_m < hi_m:
        mid = (lo_m + hi_m) >> 1
        if lsi(mid) < -50.66:
            hi_m = mid
        else:
            lo_m = mid + 1
    N = lo_m + 8

    def xprod(v):
        out = (al - c) * v
        out[1:] += be[:n - 1] * v[:n - 1]
        out[:n - 1] += be[:n - 1] * v[1:]
        return out / r

    b1, b2 = np.zeros(n), np.zeros(n)
    ip1, im, ssum = 0.0, 1.0, 0.0
    for m in range(N, 0, -1):
        v = 2.0 * xprod(b1) - b2
        v[0] += 2.0 * im
        b2, b1 = b1, v
        ssum += 2.0 * im
        ip1, im = im, ip1 + (2.0 * m / r) * im
        if abs(im) > 1e200:
            im, ip1, ssum = im * 1e-200, ip1 * 1e-200, ssum * 1e-200
            b1, b2 = b1 * 1e-200, b2 * 1e-200
    v = xprod(b1) - b2
    v[0] += im
    yv = v / (ssum + im)
    if not np.sum(yv * yv) >= 1e-6:  # ||exp(T - bI) e_1|| < 1e-3: handed to the host
        return None
    return np.exp(b) * yv
