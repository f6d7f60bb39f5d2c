"""GPU parity: the HIP path (libtpl_amd.so through its C ABI) against the CPU oracle.

Parity contract:
  P0  run-to-run bitwise determinism on the GPU
  P1  pass two regenerates pass one's basis bit for bit (reference: basis_drift_fro = 0.0)
  P2  GPU == oracle in the device's canonical reduction order: BITWISE (alphas, betas,
      ||b||, V_k, x), up to the full 500k-arc k = 500 headline configuration
  P3  GPU vs the reference-order (faithful) oracle and the published CSVs: 1e-10 on x
      for configs 1-2 (before the order-chaos onset), the reference's own thresholds
      (5e-9 property checks, 1e-3 / 1e-12 analytic checks) everywhere
"""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import canon_schedule, harness_b, load_kkt

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from oracle import ftk_ref  # noqa: E402
from oracle.rng import std_rng_vector  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
from tpl_amd import HipCsrOp, LanczosError, LanczosErrorKind, ftk, solvers  # noqa: E402
from tpl_amd import algorithms as alg  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def canon(op: HipCsrOp, a):
    """Oracle in the live operator's device order."""
    return oracle.Operator(a, op.schedule())


def skewed_matrix(n=12000, seed=7):
    """Symmetric test matrix with short rows (STREAM items), long rows of 33..900 nnz and
    three 6000+ nnz hubs (sliced), general (non +-1) values and a diagonal."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(n):
        k = rng.integers(0, 4)
        rows += [i] * k
        cols += list(rng.integers(0, n, size=k))
    for h in range(50, 70):           # medium hubs -> WAVE rows
        c = rng.choice(n, size=int(rng.integers(40, 900)), replace=False)
        rows += [h] * len(c)
        cols += list(c)
    for h in (100, 5000, 11000):      # big hubs -> BLOCK rows
        c = rng.choice(n, size=6000, replace=False)
        rows += [h] * len(c)
        cols += list(c)
    vals = rng.standard_normal(len(rows))
    s = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    a = (s + s.T + sp.diags(rng.uniform(1, 2, n))).tocsr()
    a.sum_duplicates()
    a.sort_indices()
    return a


@pytest.fixture(scope="module")
def skewed():
    return skewed_matrix()


@pytest.fixture(scope="module")
def op5k(kkt5k):
    return HipCsrOp(kkt5k)


@pytest.mark.parametrize("which", ["skewed", "kkt5k", "kkt50k"])
def test_schedule_matches_rule(which, skewed, kkt5k, kkt50k):
    a = {"skewed": skewed, "kkt5k": kkt5k.a, "kkt50k": kkt50k.a}[which]
    op = HipCsrOp(a)
    sch = op.schedule()
    ref = canon_schedule(a, reorder=True)      # the default locality order
    assert ref["perm"] is not None and np.array_equal(sch["perm"], ref["perm"])
    assert len(sch["short_rows"]) > 0 and len(sch["long_rows"]) > 0
    assert np.array_equal(sch["short_rows"], ref["short_rows"])
    assert np.array_equal(sch["long_rows"], ref["long_rows"])
    assert sch["G2"] == ref["G2"] and sch["E"] == ref["E"]
    assert sch["slices"] == ref["slices"]


@pytest.mark.parametrize("which", ["kkt5k", "kkt50k"])
def test_kkt_layouts_bitwise(which, kkt5k, kkt50k):
    """The KKT operators against the oracle in the layout's order: SpMV, pass one, pass
    two with its basis (== pass one's, bit for bit), x."""
    a = {"kkt5k": kkt5k.a, "kkt50k": kkt50k.a}[which]
    b = harness_b(a)
    op = HipCsrOp(a)
    o = canon(op, a)
    x = std_rng_vector(a.shape[0]) - 0.5
    assert np.array_equal(op.apply(x), o.apply(x))
    k = 60
    out = alg.lanczos_standard(op, b, k)
    al, be, st, bn, V = o.pass_one(b, k, store_basis=True)
    d = out.decomposition
    assert d.steps_taken == st and d.b_norm == bn
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
    assert np.array_equal(np.asarray(out.v_k), V)
    y = ftk.EXP(d.alphas, d.betas) * d.b_norm
    p2 = alg.lanczos_pass_two_with_basis(op, b, d, y)
    assert np.array_equal(np.asarray(p2.v_k), V)      # P1: regenerated basis
    xo, _ = o.pass_two(b, al, be, st, bn, y)
    assert np.array_equal(np.asarray(p2.x_k), xo)
    op.close()


@pytest.mark.parametrize("which", ["kkt5k", "skewed", "diag"])
def test_spmv_bitwise(which, kkt5k, skewed):
    a = {"kkt5k": kkt5k.a, "skewed": skewed,
         "diag": sp.diags(np.arange(1.0, 101.0)).tocsr()}[which]
    op = HipCsrOp(a)
    x = std_rng_vector(a.shape[0]) - 0.5
    y = op.apply(x)
    assert np.array_equal(y, canon(op, a).apply(x))
    yf = oracle.Operator(a).apply(x)
    assert np.linalg.norm(y - yf) <= 1e-13 * np.linalg.norm(yf)


@pytest.mark.parametrize("which,k", [("kkt5k", 50), ("skewed", 60), ("kkt5k_rand", 80)])
def test_pass_one_bitwise(which, k, kkt5k, skewed):
    a = skewed if which == "skewed" else kkt5k.a
    b = harness_b(a) if which == "kkt5k" else std_rng_vector(a.shape[0])
    op = HipCsrOp(a)
    d = alg.lanczos_pass_one(op, b, k)
    al, be, s, bn, _ = canon(op, a).pass_one(b, k)
    assert d.steps_taken == s == k
    assert d.b_norm == bn
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)


@pytest.mark.parametrize("slices", [1, 2, 4, 8])
def test_slice_counts_bitwise(slices, kkt5k, skewed):
    """Every long-row slice count (1: rows finished in place, no hand-off; 2-8: the
    last-arriver hand-off) against the oracle in that order: SpMV, pass one, and the
    two-pass x (pass two's grouped x updates)."""
    for a, b in ((kkt5k.a, harness_b(kkt5k.a)), (skewed, std_rng_vector(skewed.shape[0]))):
        op = HipCsrOp(a)
        op.set_slices(slices)
        assert op.schedule()["slices"] == slices
        o = canon(op, a)
        x = std_rng_vector(a.shape[0]) - 0.5
        assert np.array_equal(op.apply(x), o.apply(x))
        d = alg.lanczos_pass_one(op, b, 31)
        al, be, st, bn, _ = o.pass_one(b, 31)
        assert d.steps_taken == st
        assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
        op.set_device_ftk(0)  # the host exp: x bitwise against the oracle's
        assert np.array_equal(solvers.lanczos_two_pass(op, b, 31, ftk.EXP),
                              o.lanczos_two_pass(b, 31, ftk.EXP))
        op.close()


def test_basis_regeneration_bitwise(skewed):
    """P1 + P2: standard V_k == pass-two V'_k == oracle V_k, bit for bit."""
    a = skewed
    b = std_rng_vector(a.shape[0])
    op = HipCsrOp(a)
    out = alg.lanczos_standard(op, b, 40)
    dec = out.decomposition
    y = 0.1 * np.arange(1, dec.steps_taken + 1)
    p2 = alg.lanczos_pass_two_with_basis(op, b, dec, y)
    assert np.array_equal(out.v_k, p2.v_k)
    o = canon(op, a)
    al, be, s, bn, V = o.pass_one(b, 40, store_basis=True)
    assert np.array_equal(out.v_k, V)
    x_or, V2 = o.pass_two(b, al, be, s, bn, y, store_basis=True)
    assert np.array_equal(p2.x_k, x_or) and np.array_equal(p2.v_k, V2)
    # the production pass two (no basis) gives the same x
    assert np.array_equal(alg.lanczos_pass_two(op, b, dec, y), x_or)


@pytest.mark.parametrize("solver", ["two_pass", "one_pass"])
def test_solver_x_bitwise(solver, op5k, kkt5k):
    a = kkt5k.a
    b = harness_b(a)
    o = canon(op5k, a)
    if solver == "two_pass":
        x = solvers.lanczos_two_pass(op5k, b, 50, ftk.INV)
        xo = o.lanczos_two_pass(b, 50, ftk.INV)
    else:
        x = solvers.lanczos(op5k, b, 50, ftk.INV)
        xo = o.lanczos(b, 50, ftk.INV)
    assert np.array_equal(x, xo)


def test_determinism(op5k, kkt5k):
    b = std_rng_vector(kkt5k.a.shape[0])
    x1 = solvers.lanczos_two_pass(op5k, b, 60, ftk.INV)
    x2 = solvers.lanczos_two_pass(op5k, b, 60, ftk.INV)
    x3 = solvers.lanczos_two_pass(op5k, b, 60, "inv")
    assert np.array_equal(x1, x2) and np.array_equal(x1, x3)


def test_profile_kernel_ids(op5k, kkt5k):
    """tpl_profile_kernel (bench.py's isolated timings): every single-GPU id times its
    launches and reports SURVEY §8(d)'s bytes; the pass-one step is both launches; the
    exchange ids need a partitioned operator; a later solve is unaffected."""
    from tpl_amd import _lib
    n, nnz = kkt5k.a.shape[0], kkt5k.a.nnz
    spmv = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n
    want = {_lib.TPL_KERNEL_SPMV: spmv, _lib.TPL_KERNEL_PASS1_SPMV: spmv + 8.0 * n,
            _lib.TPL_KERNEL_PASS1_AXPY: 24.0 * n, _lib.TPL_KERNEL_PASS1_STEP: spmv + 32.0 * n,
            _lib.TPL_KERNEL_PASS2_SPMV: spmv + 8.0 * n + 16.0 * n / 3.0}
    b = std_rng_vector(n)
    x0 = solvers.lanczos_two_pass(op5k, b, 40, ftk.INV)
    us = {}
    for kid, by in want.items():
        us[kid], got = op5k.profile_kernel(kid, 20)
        assert us[kid] > 0.0 and got == pytest.approx(by, rel=1e-12), kid
    assert us[_lib.TPL_KERNEL_PASS1_STEP] > us[_lib.TPL_KERNEL_PASS1_SPMV]
    for kid in (_lib.TPL_KERNEL_EXCHANGE_P1, _lib.TPL_KERNEL_EXCHANGE_P2):
        with pytest.raises(tpl_amd.TplError):
            op5k.profile_kernel(kid, 5)
    with pytest.raises(tpl_amd.TplError):
        op5k.profile_kernel(99, 5)
    assert np.array_equal(solvers.lanczos_two_pass(op5k, b, 40, ftk.INV), x0)


def test_config1_vs_reference_order(op5k, kkt5k):
    """Config 1: 5k arcs, two-pass k = 50, f = inv: within 1e-10 of the reference-order
    oracle (row-sequential SpMV, sequential dot/norm, LAPACK solve)."""
    a = kkt5k.a
    b = harness_b(a)
    x = solvers.lanczos_two_pass(op5k, b, 50, ftk.INV)
    xf = oracle.Operator(a).lanczos_two_pass(b, 50, ftk_ref.inv)
    assert np.linalg.norm(x - xf) <= 1e-10 * np.linalg.norm(xf)


def test_config2_vs_reference_order(kkt50k):
    """Config 2: 50k arcs, two-pass k = 200, f = exp — the product path runs the whole
    solve as one device graph (exp(T_k) e_1 on the GPU, k_ftk_exp); x within 1e-10 of the
    faithful (reference-order) oracle with LAPACK's EVD. With the host exp the same
    operator's x is bitwise the canonical oracle's, and the two f paths agree to 1e-12."""
    a = kkt50k.a
    b = harness_b(a)
    op = HipCsrOp(a)
    x = solvers.lanczos_two_pass(op, b, 200, ftk.EXP)
    assert op.flags() & 32  # one device graph
    xf = oracle.Operator(a).lanczos_two_pass(b, 200, ftk_ref.exp)
    assert np.linalg.norm(x - xf) <= 1e-10 * np.linalg.norm(xf)
    op.set_device_ftk(0)
    xh = solvers.lanczos_two_pass(op, b, 200, ftk.EXP)
    assert not op.flags() & 32
    assert np.array_equal(xh, canon(op, a).lanczos_two_pass(b, 200, ftk.EXP))
    assert np.linalg.norm(x - xh) <= 1e-12 * np.linalg.norm(xh)


def test_kkt_property_checks_gpu(op5k, kkt5k):
    """src/algorithms/mod.rs:434-587 on the GPU, TOLERANCE = 5e-9, k = 30, StdRng(42) b."""
    a = kkt5k.a
    k = 30
    b = std_rng_vector(a.shape[0])
    out = alg.lanczos_standard(op5k, b, k)
    po = alg.lanczos_pass_one(op5k, b, k)
    d = out.decomposition
    assert d.steps_taken == po.steps_taken
    assert np.max(np.abs(d.alphas - po.alphas)) < 5e-9
    assert np.max(np.abs(d.betas - po.betas)) < 5e-9
    out1 = alg.lanczos_standard(op5k, b, k + 1)
    V = out.v_k
    T = ftk_ref.tridiag(d.alphas, d.betas)
    E = np.outer(out1.v_k[:, k], np.eye(k)[k - 1]) * out1.decomposition.betas[k - 1]
    assert np.linalg.norm(a @ V - V @ T - E) < 5e-9
    assert np.linalg.norm(np.eye(k) - V.T @ V) < 5e-9
    y = 0.1 * np.arange(1, k + 1)
    Vr = alg.lanczos_pass_two_with_basis(op5k, b, po, y).v_k
    assert np.sum((V - Vr) ** 2) < 5e-9


@pytest.mark.parametrize("fname,f,tol", [("inv", lambda z: 1.0 / z, 1e-3),
                                         ("exp", np.exp, 1e-3),
                                         ("sq", lambda z: z ** 2, 1e-12)])
def test_correctness_rs_gpu(fname, f, tol):
    """tests/correctness.rs (6 tests): diag(1..100), k = 30, StdRng(42) b."""
    lam = np.arange(1.0, 101.0)
    b = std_rng_vector(100)
    op = HipCsrOp(sp.diags(lam).tocsr())
    xt = f(lam) * b
    for solve in (solvers.lanczos, solvers.lanczos_two_pass):
        for fk in (ftk.BUILTINS[fname], ftk_ref.SOLVERS[fname]):  # native and Python closures
            x = solve(op, b, 30, fk)
            assert np.linalg.norm(x - xt) / np.linalg.norm(xt) < tol


def test_doctest_gpu():
    """src/lib.rs:35-84."""
    a = sp.diags([-np.ones(3), 2 * np.ones(4), -np.ones(3)], [-1, 0, 1]).tocsr()
    op = HipCsrOp(a)
    b = np.array([1.0, 2.0, 3.0, 4.0])
    x1 = solvers.lanczos(op, b, 3, ftk.INV)
    x2 = solvers.lanczos_two_pass(op, b, 3, ftk.INV)
    assert np.linalg.norm(x1 - x2) < 1e-12


def test_unit_values_and_breakdown():
    """src/algorithms/mod.rs:385-428."""
    a = sp.diags([-np.ones(3), 2 * np.ones(4), -np.ones(3)], [-1, 0, 1]).tocsr()
    d = alg.lanczos_pass_one(HipCsrOp(a), np.array([1.0, 0, 0, 0]), 2)
    assert abs(d.alphas[0] - 2.0) < 1e-15 and abs(d.betas[0] - 1.0) < 1e-15
    out = alg.lanczos_standard(HipCsrOp(sp.diags([2.0, 3.0]).tocsr()), np.array([1.0, 0.0]), 2)
    assert out.decomposition.steps_taken == 1 and out.v_k.shape == (2, 1)
    with pytest.raises(LanczosError) as e:
        alg.lanczos_standard(HipCsrOp(sp.identity(2).tocsr()), np.zeros(2), 2)
    assert e.value.kind == LanczosErrorKind.INPUT_ERROR


def test_error_semantics(op5k, kkt5k):
    n = kkt5k.a.shape[0]
    b = std_rng_vector(n)
    z = np.zeros(n)
    msg1 = "Invalid input parameter: Input vector `b` must not be a zero vector."
    for call in (lambda: solvers.lanczos_two_pass(op5k, z, 5, ftk.INV),
                 lambda: solvers.lanczos(op5k, z, 5, ftk.INV),
                 lambda: alg.lanczos_pass_one(op5k, z, 5)):
        with pytest.raises(LanczosError) as e:
            call()
        assert str(e.value) == msg1
    d = alg.lanczos_pass_one(op5k, b, 6)
    with pytest.raises(LanczosError) as e:
        alg.lanczos_pass_two(op5k, b, d, np.ones(5))
    assert str(e.value) == "Parameter mismatch: `y_k` expects size 6, but got 5."
    # the variant's fields crossed the C ABI (tpl_last_error_detail), not just its text
    assert e.value.payload == {"param_name": "y_k", "expected": 6, "actual": 5}
    d0 = alg.LanczosDecomposition(d.alphas, d.betas, d.steps_taken, 0.0)
    with pytest.raises(LanczosError) as e:
        alg.lanczos_pass_two(op5k, b, d0, np.ones(6))
    assert str(e.value) == ("Invalid input parameter: The initial vector `b` must not be a "
                            "zero vector.")

    def bad(al, be):
        raise RuntimeError("boom")
    with pytest.raises(LanczosError) as e:
        solvers.lanczos_two_pass(op5k, b, 5, bad)
    assert str(e.value) == "The user-provided f(T_k) solver failed: boom"
    assert e.value.kind == LanczosErrorKind.SOLVER_ERROR and e.value.payload == "boom"
    with pytest.raises(LanczosError) as e:
        solvers.lanczos(op5k, b, 5, lambda al, be: np.ones(3))
    assert str(e.value) == "Parameter mismatch: `y_k_prime` expects size 5, but got 3."
    assert e.value.payload == {"param_name": "y_k_prime", "expected": 5, "actual": 3}
    with pytest.raises(LanczosError) as e:
        solvers.lanczos_two_pass(op5k, b, 5, lambda al, be: np.ones((5, 2)))
    assert e.value.kind == LanczosErrorKind.PARAMETER_MISMATCH
    with pytest.raises(LanczosError) as e:
        solvers.lanczos_two_pass(op5k, b[:-1], 5, ftk.INV)
    assert str(e.value) == f"Dimension mismatch: operator has {n} columns but vector has {n - 1} rows."
    assert e.value.kind == LanczosErrorKind.DIMENSION_MISMATCH
    assert e.value.payload == {"operator_cols": n, "vector_rows": n - 1}
    with pytest.raises(LanczosError) as e:
        solvers.lanczos_two_pass(op5k, b, 0, ftk.INV)
    assert e.value.kind == LanczosErrorKind.INPUT_ERROR


@pytest.mark.parametrize("stop", [1, 2, 3, 7, 8, 31, 40])
def test_step_callback(stop, op5k, kkt5k):
    """LanczosCallback (src/algorithms/mod.rs:82-86, lanczos.rs:93-106): the callback sees
    every step in order with the reference's TridiagonalSystemView and V view, and an
    early stop at `stop` returns exactly the `stop`-step decomposition and basis — checked
    against the canonical oracle (the host polls in batches of 1, 2, 4, ... 32 steps, so
    stops fall inside and at the edges of batches)."""
    a = kkt5k.a
    n = a.shape[0]
    b = std_rng_vector(n)
    seen = []

    def cb(k, v_view, t):
        seen.append((k, len(t.alphas), len(t.betas), v_view.shape))
        return k < stop
    out = alg.lanczos_standard(op5k, b, 50, callback=cb)
    assert out.decomposition.steps_taken == stop
    assert [s[0] for s in seen] == list(range(1, stop + 1))
    assert seen[-1] == (stop, stop, stop - 1, (n, stop))
    al, be, steps, bn, V = canon(op5k, a).pass_one(b, stop, store_basis=True)
    assert steps == stop
    assert np.array_equal(out.decomposition.alphas, al[:stop])
    assert np.array_equal(out.decomposition.betas, be[:stop - 1])
    assert np.array_equal(np.asarray(out.v_k), V[:, :stop])


def test_step_callback_views_and_exception(op5k, kkt5k):
    """The T view at step k holds the first k alphas / k-1 betas of the final run; an
    exception raised by the callback stops the loop and propagates to the caller."""
    b = std_rng_vector(kkt5k.a.shape[0])
    views = []
    alg.lanczos_standard(op5k, b, 20, callback=lambda k, v, t: views.append(
        (t.alphas.copy(), t.betas.copy())) or True)
    full = alg.lanczos_standard(op5k, b, 20)
    for k, (va, vb) in enumerate(views, start=1):
        assert np.array_equal(va, full.decomposition.alphas[:k])
        assert np.array_equal(vb, full.decomposition.betas[:k - 1])

    class Boom(Exception):
        pass

    def bad(k, v, t):
        if k == 5:
            raise Boom("stop here")
        return True
    with pytest.raises(Boom):
        alg.lanczos_standard(op5k, b, 20, callback=bad)


ACC_ROWS = {("inv", "well"): [10, 50, 100, 200], ("inv", "ill"): [10, 60, 120],
            ("exp", "well"): [10, 20, 30], ("exp", "ill"): [10, 70, 140]}


@pytest.mark.parametrize("func,scen", sorted(ACC_ROWS))
def test_accuracy_csv_gpu(func, scen):
    """Published results/accuracy_*.csv rows reproduced through the GPU path."""
    import csv
    import os

    from conftest import REF_RESULTS
    from test_oracle_golden import ACC_POLICY, stability_eigs
    kmax, rtol, atol = ACC_POLICY[(func, scen)]
    lam = stability_eigs(func, scen)
    b = std_rng_vector(lam.shape[0])
    op = HipCsrOp(sp.diags(lam).tocsr())
    fx = (1.0 / lam if func == "inv" else np.exp(lam)) * b
    rows = {int(r["k"]): r for r in csv.DictReader(open(os.path.join(
        REF_RESULTS, f"accuracy_{func}_{scen}-conditioned.csv")))}
    for k in ACC_ROWS[(func, scen)]:
        for solve, col in ((solvers.lanczos, "relative_error_standard"),
                           (solvers.lanczos_two_pass, "relative_error_two_pass")):
            x = solve(op, b, k, ftk.BUILTINS[func])
            e = np.linalg.norm(x - fx) / np.linalg.norm(fx)
            ref = float(rows[k][col])
            assert abs(e - ref) <= rtol * ref + atol, (k, col, e, ref)


def test_orthogonality_drift_zero_gpu():
    """results/orthogonality_*.csv: basis_drift_fro = 0.0 — standard V_k vs regenerated V'_k."""
    from test_oracle_golden import stability_eigs
    lam = stability_eigs("inv", "ill")
    b = std_rng_vector(lam.shape[0])
    op = HipCsrOp(sp.diags(lam).tocsr())
    for k in (20, 100, 300):
        out = alg.lanczos_standard(op, b, k)
        s = out.decomposition.steps_taken
        p2 = alg.lanczos_pass_two_with_basis(op, b, out.decomposition, np.zeros(s))
        assert np.linalg.norm(out.v_k - p2.v_k) == 0.0
        assert np.linalg.norm(p2.x_k) == 0.0


def test_reorthogonalization_extension(op5k, kkt5k):
    """Config 4 extension (no reference counterpart): CGS2 keeps V_k orthonormal."""
    a = kkt5k.a
    b = std_rng_vector(a.shape[0])
    k = 150
    plain = alg.lanczos_standard(op5k, b, k)
    re = alg.lanczos_standard(op5k, b, k, reorthogonalize=True)
    s = re.decomposition.steps_taken
    V = re.v_k
    loss_re = np.linalg.norm(np.eye(s) - V.T @ V)
    loss_plain = np.linalg.norm(np.eye(plain.decomposition.steps_taken) - plain.v_k.T @ plain.v_k)
    assert loss_re < 1e-12 < loss_plain
    # early steps agree with the plain recurrence
    assert np.allclose(re.decomposition.alphas[:10], plain.decomposition.alphas[:10], atol=1e-12)
    T = ftk_ref.tridiag(re.decomposition.alphas, re.decomposition.betas)
    R = a @ V - V @ T
    R[:, -1] = 0.0  # last column carries beta_k v_{k+1}
    assert np.linalg.norm(R) < 1e-10
    # bitwise against the oracle's CGS2 restatement in the device order
    al, be, st, bn, Vo = canon(op5k, a).pass_one(b, k, reorth=True)
    assert st == s and bn == re.decomposition.b_norm
    assert np.array_equal(re.decomposition.alphas, al)
    assert np.array_equal(re.decomposition.betas, be)
    assert np.array_equal(np.asarray(V), Vo)


@pytest.mark.parametrize("which", ["kkt5k", "skewed"])
def test_selective_reorthogonalization_bitwise(which, op5k, kkt5k, skewed):
    """Selective (Kahan–Parlett) re-orthogonalisation: the second Gram-Schmidt pass only
    where the first removed more than half of ||r||^2 — the device's decisions and every
    value bit for bit against the oracle's restatement; orthonormal like CGS2."""
    a = kkt5k.a if which == "kkt5k" else skewed
    op = op5k if which == "kkt5k" else HipCsrOp(a)
    b = std_rng_vector(a.shape[0])
    k = 150
    re = alg.lanczos_standard(op, b, k, reorthogonalize="selective")
    second = op.reorth_second_passes()
    s = re.decomposition.steps_taken
    V = np.asarray(re.v_k)
    assert np.linalg.norm(np.eye(s) - V.T @ V) < 1e-12
    assert 0 <= second < s
    al, be, st, bn, Vo = canon(op, a).pass_one(b, k, reorth="selective")
    assert st == s and bn == re.decomposition.b_norm
    assert np.array_equal(re.decomposition.alphas, al)
    assert np.array_equal(re.decomposition.betas, be)
    assert np.array_equal(V, Vo)
    cg = alg.lanczos_standard(op, b, k, reorthogonalize=True)
    assert op.reorth_second_passes() == cg.decomposition.steps_taken - 1
    with pytest.raises(ValueError):
        alg.lanczos_standard(op, b, k, reorthogonalize="mgs")


def test_device_pointer_path(op5k, kkt5k):
    torch = pytest.importorskip("torch")
    b = harness_b(kkt5k.a)
    xh = solvers.lanczos_two_pass(op5k, b, 40, ftk.INV)
    bd = torch.from_numpy(b).cuda()
    xd = solvers.lanczos_two_pass(op5k, bd, 40, ftk.INV)
    assert xd.is_cuda and np.array_equal(xd.cpu().numpy(), xh)


@pytest.mark.timeout(900)
def test_headline_500k_bitwise(kkt_tmp):
    """Config 3 at full size: 500k arcs, two-pass k = 500, f = inv — alphas/betas/x
    bit-identical to the canonical-order oracle; alpha == 0 exactly;
    and the result solves A x = b (A singular: x is one of many solutions)."""
    kkt = load_kkt(500000, kkt_tmp)
    a = kkt.a
    b = harness_b(a)
    op = HipCsrOp(a)
    o = canon(op, a)
    d = alg.lanczos_pass_one(op, b, 500)
    al, be, s, bn, _ = o.pass_one(b, 500)
    assert d.steps_taken == s == 500 and d.b_norm == bn
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
    assert np.all(d.alphas == 0.0)
    x = solvers.lanczos_two_pass(op, b, 500, ftk.INV)
    xo, _ = o.pass_two(b, al, be, s, bn, ftk.INV(al, be) * bn)
    assert np.array_equal(x, xo)
    assert np.linalg.norm(a @ x - b) / np.linalg.norm(b) < 1e-8


def test_headline_pinned_order_bitwise(kkt_tmp):
    """The operator the bench times, exactly: 500k arcs in the locality order with the
    pinned group count (bench.py PINNED_ORDER_GROUPS), two-pass k = 500, f = inv (the
    one-graph host-f path the bench takes at k = 500). alpha / beta / x are bitwise the
    canonical oracle's on that permutation, and a second operator built the same way
    (what the next bench run builds) reproduces x bit for bit."""
    sys.path.insert(0, ROOT)
    from bench import PINNED_ORDER_GROUPS
    g = PINNED_ORDER_GROUPS[500000]
    kkt = load_kkt(500000, kkt_tmp)
    a = kkt.a
    b = harness_b(a)
    op = HipCsrOp(a)
    op.set_order_groups(g)
    assert op.flags() & 64 and op.order_groups() == g
    sch = op.schedule()
    import tpl_amd
    assert np.array_equal(sch["perm"], tpl_amd.locality_order(a, groups=g))
    o = oracle.Operator(a, sch)
    d = alg.lanczos_pass_one(op, b, 500)
    al, be, s, bn, _ = o.pass_one(b, 500)
    assert d.steps_taken == s == 500 and d.b_norm == bn
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
    x = solvers.lanczos_two_pass(op, b, 500, ftk.INV)
    xo, _ = o.pass_two(b, al, be, s, bn, ftk.INV(al, be) * bn)
    assert np.array_equal(x, xo)
    op2 = HipCsrOp(a)
    op2.set_order_groups(g)
    assert np.array_equal(solvers.lanczos_two_pass(op2, b, 500, ftk.INV), x)
    # the host-only plan the parity fixture is made from holds this exact layout, and the
    # fixture's digest is this x (tests/golden/make_parity.py, bench.py `parity`)
    plan = tpl_amd.HostPlan(a, order_groups=g)
    ps = plan.schedule()
    for key in ("short_rows", "long_rows", "perm"):
        assert np.array_equal(ps[key], sch[key]), key
    assert (ps["G2"], ps["E"], ps["slices"]) == (sch["G2"], sch["E"], sch["slices"])
    import json
    import hashlib
    with open(os.path.join(ROOT, "tests", "golden", "parity.json")) as f:
        exp = json.load(f)["workloads"]["headline"]
    assert hashlib.sha256(x.tobytes()).hexdigest()[:16] == exp["x"]
    op.close()
    op2.close()


def test_int8_value_format_bitwise(kkt_tmp):
    """Lossless value compression: the KKT's +-1 values are kept as int8 and every result
    keeps its bits (tpl_op_set_value_format); non-integer values stay fp64."""
    import tpl_amd
    a = load_kkt(50000, kkt_tmp).a
    b = harness_b(a)
    op = tpl_amd.HipCsrOp(a)
    assert op.int8_values
    from tpl_amd import _lib
    assert int(_lib.tpl_op_flags(op.handle)) & 24 == 24  # uint16 columns in chunks and bins
    x8 = tpl_amd.lanczos_two_pass(op, b, 100, "exp")
    d8 = tpl_amd.algorithms.lanczos_pass_one(op, b, 100)
    op.set_value_format(False)
    assert not op.int8_values and int(_lib.tpl_op_flags(op.handle)) & 24 == 0
    x64 = tpl_amd.lanczos_two_pass(op, b, 100, "exp")
    d64 = tpl_amd.algorithms.lanczos_pass_one(op, b, 100)
    assert np.array_equal(x8, x64)
    assert np.array_equal(d8.alphas, d64.alphas) and np.array_equal(d8.betas, d64.betas)
    op2 = tpl_amd.HipCsrOp(a * 0.5)
    assert not op2.int8_values
    # +-2 values: int8 as well; bitwise the oracle on the same layout
    a2 = (a * 2.0).tocsr()
    op3 = tpl_amd.HipCsrOp(a2)
    assert op3.int8_values and int(_lib.tpl_op_flags(op3.handle)) & 24 == 24
    o3 = canon(op3, a2)
    d3 = tpl_amd.algorithms.lanczos_pass_one(op3, b, 60)
    al, be, st, bn, _ = o3.pass_one(b, 60)
    assert np.array_equal(d3.alphas, al) and np.array_equal(d3.betas, be)
    x3 = tpl_amd.lanczos_two_pass(op3, b, 60, "inv")  # device inv: bitwise the host's
    assert np.array_equal(x3, o3.lanczos_two_pass(b, 60, ftk.INV))
    op3.close()


def test_synthetic_generator_instance_bitwise():
    """BASELINE configs[4]'s instance family (tpl_generate_kkt, the 5M-arc multi-GPU
    workload) at 200k arcs on one GPU: the layout rules that apply at that size
    (4 column slices, chunk window) against the oracle, bit for bit; run to run equal."""
    from tpl_amd.utils.data_loader import generate_kkt
    a = generate_kkt(200000, seed=42).a
    n = a.shape[0]
    b = harness_b(a)
    op = HipCsrOp(a)
    sch = op.schedule()
    assert sch["slices"] == canon_schedule(a)["slices"]
    o = canon(op, a)
    k = 80
    d = alg.lanczos_pass_one(op, b, k)
    al, be, st, bn, _ = o.pass_one(b, k)
    assert d.steps_taken == st and d.b_norm == bn
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
    x = solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert np.array_equal(x, o.lanczos_two_pass(b, k, ftk.INV))
    assert np.array_equal(x, solvers.lanczos_two_pass(op, b, k, ftk.INV))
    assert n == a.shape[1]
    op.close()
