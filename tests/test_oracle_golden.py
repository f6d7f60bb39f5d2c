"""CPU: pin the oracle (CPU restatement of the reference hot path) against the
reference's own golden data and unit-test values. No GPU needed.

Golden sources (copied verbatim as data into tests/golden/reference_results):
  results/accuracy_*.csv       relative errors per k (src/bin/stability.rs:257-310)
  results/orthogonality_*.csv  basis_drift_fro == 0.0 (src/bin/orthogonality.rs:180-215)
Unit values: src/algorithms/mod.rs:385-428; thresholds: tests/correctness.rs:42,51,
src/algorithms/mod.rs:360; doctest src/lib.rs:35-84.
"""
import csv
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import REF_RESULTS, canon_schedule, harness_b

import oracle
from oracle import ftk_ref
from oracle.rng import std_rng_vector

N_STAB = 10000


def stability_eigs(func, scen, n=N_STAB):
    """create_diagonal_problem, src/bin/stability.rs:98-157 (same as orthogonality.rs:90-146)."""
    i = np.arange(n, dtype=np.float64)
    if func == "exp" and scen == "well":
        return -10.0 + (9.9 / max(n - 1, 1)) * i
    if func == "exp" and scen == "ill":
        return -1000.0 + (999.9 / max(n - 1, 1)) * i
    if func == "inv" and scen == "well":
        return 0.1 + (99.9 / max(n - 1, 1)) * i
    mid = n // 2
    e = np.empty(n)
    e[:mid] = 0.1 + (0.9 / max(mid - 1, 1)) * i[:mid]
    e[mid:] = -1.0 + (0.9 / max(n - mid - 1, 1)) * (i[mid:] - mid)
    e[mid] = 1e-8
    return e


# Published-row tolerance policy: the Lanczos recurrence without re-orthogonalisation
# is chaotic in the summation order past ~130-150 steps, so rows
# past that depend on faer's unpinned SIMD order. rel = bound on |e - e_ref| / e_ref,
# abs = floor for rows at the 1e-15 noise level.
ACC_POLICY = {
    ("inv", "well"): (200, 1e-9, 1e-13),
    ("inv", "ill"): (130, 1e-9, 1e-13),
    ("exp", "well"): (200, 1e-5, 1e-13),
    ("exp", "ill"): (140, 1e-5, 1e-13),
}


def test_std_rng_restatement():
    b = std_rng_vector(8)
    np.testing.assert_allclose(b[:4], [0.52655741, 0.54272521, 0.6364651, 0.40590176], atol=5e-9)
    assert np.all((b >= 0) & (b < 1))


@pytest.mark.parametrize("func,scen", sorted(ACC_POLICY))
def test_accuracy_csv_reproduced(func, scen):
    kmax, rtol, atol = ACC_POLICY[(func, scen)]
    lam = stability_eigs(func, scen)
    b = std_rng_vector(N_STAB)
    op = oracle.Operator(sp.diags(lam).tocsr())
    f = ftk_ref.SOLVERS[func]
    fx = (1.0 / lam if func == "inv" else np.exp(lam)) * b
    rows = list(csv.DictReader(open(os.path.join(REF_RESULTS,
                                                 f"accuracy_{func}_{scen}-conditioned.csv"))))
    checked = 0
    for r in rows:
        k = int(r["k"])
        if k > kmax:
            continue
        x1 = op.lanczos(b, k, f)
        x2 = op.lanczos_two_pass(b, k, f)
        for x, col in ((x1, "relative_error_standard"), (x2, "relative_error_two_pass")):
            e = np.linalg.norm(x - fx) / np.linalg.norm(fx)
            ref = float(r[col])
            assert abs(e - ref) <= rtol * ref + atol, (func, scen, k, col, e, ref)
        dev = np.linalg.norm(x1 - x2) / np.linalg.norm(x1)
        assert dev < 1e-14 and float(r["relative_solution_deviation"]) < 1e-14
        checked += 1
    assert checked >= 13


@pytest.mark.parametrize("func,scen", [("inv", "well"), ("inv", "ill"), ("exp", "well"),
                                       ("exp", "ill")])
def test_orthogonality_csv(func, scen):
    """basis_drift_fro == 0.0 and solution_deviation == 0.0 (bit-identical regeneration)
    in both reduction orders; ortho_loss magnitude within x3 of the published value.

    The magnitude check uses the device (tree) order: faer's dot/norm are blocked,
    and a strictly sequential sum loses ~10x more orthogonality than the published
    curve (measured: sequential 10-15x, tree 0.5-1.25x of ortho_loss_standard)."""
    lam = stability_eigs(func, scen)
    b = std_rng_vector(N_STAB)
    a = sp.diags(lam).tocsr()
    seq = oracle.Operator(a)
    op = oracle.Operator(a, canon_schedule(a))
    rows = list(csv.DictReader(open(os.path.join(REF_RESULTS,
                                                 f"orthogonality_{func}_{scen}-conditioned.csv"))))
    for r in rows[:6]:
        k = int(r["k"])
        assert float(r["basis_drift_fro"]) == 0.0
        for o in (seq, op):
            al, be, s, bn, V = o.pass_one(b, k, store_basis=True)
            _, V2 = o.pass_two(b, al, be, s, bn, np.zeros(s), store_basis=True)
            assert np.array_equal(V, V2)
        loss = np.linalg.norm(np.eye(s) - V.T @ V)
        ref = float(r["ortho_loss_standard"])
        assert ref / 3 <= loss <= ref * 3, (k, loss, ref)


def test_unit_recurrence_alpha_beta():
    """src/algorithms/mod.rs:385-407: tridiag(-1,2,-1), v = e1 -> alpha = 2, beta = 1."""
    a = sp.diags([-np.ones(3), 2 * np.ones(4), -np.ones(3)], [-1, 0, 1]).tocsr()
    for sched in (None, {"short_rows": [0, 1, 2, 3], "long_rows": [], "G2": 1, "E": 512,
                            "slices": 1}):
        op = oracle.Operator(a, sched)
        al, be, s, bn, _ = op.pass_one(np.array([1.0, 0, 0, 0]), 2)
        assert abs(al[0] - 2.0) < 1e-15 and abs(be[0] - 1.0) < 1e-15


def test_unit_breakdown_and_zero_vector():
    """src/algorithms/mod.rs:410-428."""
    op = oracle.Operator(sp.diags([2.0, 3.0]).tocsr())
    _, _, s, _, _ = op.pass_one(np.array([1.0, 0.0]), 2)
    assert s == 1
    with pytest.raises(ValueError, match="must not be a zero vector"):
        oracle.Operator(sp.identity(2).tocsr()).pass_one(np.zeros(2), 2)


def test_doctest_one_pass_equals_two_pass():
    """src/lib.rs:35-84: 4x4 [-1,2,-1], b = (1,2,3,4), k = 3, ||x1 - x2|| < 1e-12."""
    a = sp.diags([-np.ones(3), 2 * np.ones(4), -np.ones(3)], [-1, 0, 1]).tocsr()
    op = oracle.Operator(a)
    b = np.array([1.0, 2.0, 3.0, 4.0])
    x1 = op.lanczos(b, 3, ftk_ref.inv)
    x2 = op.lanczos_two_pass(b, 3, ftk_ref.inv)
    assert np.linalg.norm(x1 - x2) < 1e-12


@pytest.mark.parametrize("fname,f,tol", [("inv", lambda z: 1.0 / z, 1e-3),
                                         ("exp", np.exp, 1e-3),
                                         ("sq", lambda z: z ** 2, 1e-12)])
def test_correctness_rs(fname, f, tol):
    """tests/correctness.rs: diag(1..100), k = 30, StdRng(42) b."""
    n = 100
    lam = np.arange(1, n + 1, dtype=np.float64)
    b = std_rng_vector(n)
    op = oracle.Operator(sp.diags(lam).tocsr())
    xt = f(lam) * b
    for x in (op.lanczos(b, 30, ftk_ref.SOLVERS[fname]),
              op.lanczos_two_pass(b, 30, ftk_ref.SOLVERS[fname])):
        assert np.linalg.norm(x - xt) / np.linalg.norm(xt) < tol


def test_kkt_property_checks(kkt5k):
    """The four property runners of src/algorithms/mod.rs:434-587 at TOLERANCE = 5e-9,
    k = 30, b ~ StdRng(42) on the 5k-arc netgen KKT instance."""
    a = kkt5k.a
    n = a.shape[0]
    k = 30
    b = std_rng_vector(n)
    op = oracle.Operator(a)
    al, be, s, bn, V = op.pass_one(b, k, store_basis=True)
    al1, be1, s1, _, _ = op.pass_one(b, k)
    assert s == s1 and np.max(np.abs(al - al1), initial=0) < 5e-9
    assert np.max(np.abs(be - be1), initial=0) < 5e-9
    # Lanczos relation with beta_k, v_{k+1} from a k+1 run
    al2, be2, s2, _, V2 = op.pass_one(b, k + 1, store_basis=True)
    T = ftk_ref.tridiag(al, be)
    R = a @ V - V @ T
    E = np.outer(V2[:, k], np.eye(k)[k - 1]) * be2[k - 1]
    assert np.linalg.norm(R - E) < 5e-9
    assert np.linalg.norm(np.eye(s) - V.T @ V) < 5e-9
    y = 0.1 * np.arange(1, s + 1)
    _, Vr = op.pass_two(b, al1, be1, s1, bn, y, store_basis=True)
    assert np.sum((V - Vr) ** 2) < 5e-9


def test_kkt_alpha_identically_zero(kkt5k):
    """with the harness b = A (1/sqrt(n)) 1, every alpha is exactly 0."""
    a = kkt5k.a
    b = harness_b(a)
    assert np.all(b[:5000] == 0.0)
    al, be, s, bn, _ = oracle.Operator(a).pass_one(b, 50)
    assert s == 50 and np.all(al == 0.0)


def test_canonical_and_faithful_agree_before_chaos(kkt5k):
    """Config 1 (5k arcs, two-pass k = 50, f = inv): the device-order oracle and the
    reference-order oracle agree to 1e-10 relative (onset of order chaos ~ step 63)."""
    a = kkt5k.a
    b = harness_b(a)
    xc = oracle.Operator(a, canon_schedule(a)).lanczos_two_pass(b, 50, ftk_ref.inv)
    xf = oracle.Operator(a).lanczos_two_pass(b, 50, ftk_ref.inv)
    assert np.linalg.norm(xc - xf) / np.linalg.norm(xf) < 1e-10


def test_oracle_reorth_restatement(kkt5k):
    """The CGS2 restatement (extension, BASELINE configs[3]) keeps V_k orthonormal where
    the plain recurrence has lost orthogonality, agrees with it before the loss, and
    satisfies the Lanczos relation A V = V T + beta_k v_{k+1} e_k^T."""
    a = kkt5k.a
    b = std_rng_vector(a.shape[0])
    o = oracle.Operator(a, canon_schedule(a))
    k = 120
    al, be, st, bn, V = o.pass_one(b, k, reorth=True)
    alp, bep, stp, bnp, Vp = o.pass_one(b, k, store_basis=True)
    assert st == stp == k and bn == bnp
    assert np.linalg.norm(np.eye(st) - V.T @ V) < 1e-13
    assert np.linalg.norm(np.eye(stp) - Vp.T @ Vp) > 1e-6
    assert np.allclose(al[:8], alp[:8], atol=1e-12) and np.allclose(be[:8], bep[:8], rtol=1e-12)
    R = a @ V - V @ ftk_ref.tridiag(al, be)
    R[:, -1] = 0.0
    assert np.linalg.norm(R) < 1e-10
    with pytest.raises(ValueError):
        oracle.Operator(a).pass_one(b, 5, reorth=True)  # canonical order only
