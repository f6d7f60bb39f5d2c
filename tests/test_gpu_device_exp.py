"""GPU: the device exp(T_k) e_1 (k_ftk_exp) and the one-graph
exp solve it enables.

The reference forms exp(T_k) e_1 = Q exp(Lambda) Q^T e_1 from a dense EVD
(src/bin/stability.rs:175-193). The device evaluates the same function with a Chebyshev
expansion over the Sturm-bracketed spectrum (tpl_kernels.hip k_ftk_exp). Its contract is
a tolerance, not bits: an EVD-based result carries an error of a few eps * ||T|| *
exp(lambda_max) (backward stability), the expansion a few eps * (terms) * exp(lambda_max).
Stated tolerance: ||y_dev - y_lapack|| <= TOL_SCALE * exp(lambda_max) (TOL_SCALE =
1e-12) and, because the kernel hands back to the host every case with ||y|| < 1e-3
exp(lambda_max) (where an absolute bound would not be small against ||y||), normwise
||y_dev - y_lapack|| <= TOL_NORM * ||y|| (TOL_NORM = 1e-11) for every case it keeps.
On configs[1]'s own T_k (50k arcs, k = 200) the expansion is within 6e-16 of a 35-digit
evaluation (LAPACK 4e-15, the host QL 3.4e-14; tests/test_exp_chebyshev.py).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import harness_b, load_kkt

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from oracle import ftk_ref  # noqa: E402
from oracle.rng import std_rng_vector  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
from tpl_amd import HipCsrOp, ftk, solvers  # noqa: E402
from tpl_amd import algorithms as alg  # noqa: E402

TOL_SCALE = 1e-12   # error bound in units of exp(lambda_max)
TOL_NORM = 1e-11    # normwise, relative to ||y|| (cases without cancellation)
ONE_GRAPH = 32


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


@pytest.fixture(scope="module")
def op_small():
    n = 64
    return HipCsrOp(sp.diags(np.arange(1.0, n + 1.0)).tocsr())


def lam_max(al, be):
    from scipy.linalg import eigvalsh_tridiagonal
    if len(al) == 1:
        return float(al[0])
    return float(eigvalsh_tridiagonal(np.asarray(al), np.asarray(be[:len(al) - 1]))[-1])


def check_close(y, al, be):
    yr = ftk_ref.exp(al, be)
    err = np.linalg.norm(y - yr)
    assert err <= TOL_SCALE * np.exp(lam_max(al, be)), err
    assert err <= TOL_NORM * np.linalg.norm(yr), (err, np.linalg.norm(yr))


def kkt_like(k, rng):
    """Zero diagonal, positive off-diagonal: the shape of T_k on the KKT runs (alpha = 0)."""
    return np.zeros(k), rng.uniform(0.5, 20.0, k - 1)


@pytest.mark.parametrize("k", [1, 2, 3, 7, 50, 200, 511, 1000, 1800])
def test_device_exp_random_tridiagonals(op_small, k):
    rng = np.random.default_rng(1000 + k)
    cases = [kkt_like(k, rng),
             (rng.standard_normal(k) * 5.0, rng.uniform(0.01, 3.0, k - 1)),
             (rng.uniform(-1000.0, -0.1, k), rng.uniform(0.0, 50.0, k - 1)),   # exp "ill"
             (rng.uniform(-10.0, -0.1, k), rng.uniform(0.0, 1.0, k - 1))]      # exp "well"
    if k > 200:  # large random T keep e_1 far from the top of the spectrum: add a
        # Lanczos T_k (diagonal spectrum in [-10, -0.1], random b), the shape the solver sees
        lam = np.linspace(-10.0, -0.1, 4 * k)
        v = rng.random(4 * k)
        v /= np.linalg.norm(v)
        vp = np.zeros_like(v)
        al_l, be_l, bprev = [], [], 0.0
        for _ in range(k):
            w = lam * v - bprev * vp
            a_ = v @ w
            w = w - a_ * v
            al_l.append(a_)
            bprev = np.linalg.norm(w)
            be_l.append(bprev)
            vp, v = v, w / bprev
        cases.append((np.array(al_l), np.array(be_l[:k - 1])))
    kept = 0
    for al, be in cases:
        y, on = op_small.ftk_device("exp", al, be)
        # the device keeps exactly the cases its numpy restatement keeps (same rules)
        ref = ftk_ref.exp_chebyshev(al, be) if k <= 200 else None
        if k <= 200:
            assert on == (ref is not None)
        if on:
            kept += 1
            check_close(y, al, be)
        else:
            assert np.all(y == 0.0)
    assert kept >= 1  # random T: e_1 is often far from the top of the spectrum


def test_device_exp_clusters_and_ghosts(op_small):
    """Repeated / nearly repeated eigenvalues (Lanczos ghosts): no eigenvectors are formed,
    so clusters need no special handling — still within the EVD's tolerance."""
    k = 300
    rng = np.random.default_rng(3)
    lam = np.repeat(rng.uniform(-5, 5, 30), 10) + rng.standard_normal(k) * 1e-13
    q, _ = np.linalg.qr(rng.standard_normal((k, k)))
    # tridiagonalise Q diag(lam) Q^T (Lanczos from e_1, full reorthogonalisation)
    A = (q * lam) @ q.T
    V = np.zeros((k, k))
    al, be = np.zeros(k), np.zeros(k - 1)
    v = np.zeros(k)
    v[0] = 1.0
    V[:, 0] = v
    m = k
    for j in range(k):
        w = A @ V[:, j]
        al[j] = V[:, j] @ w
        w -= V[:, :j + 1] @ (V[:, :j + 1].T @ w)
        w -= V[:, :j + 1] @ (V[:, :j + 1].T @ w)
        if j + 1 < k:
            be[j] = np.linalg.norm(w)
            if be[j] < 1e-10:
                m = j + 1
                break
            V[:, j + 1] = w / be[j]
    al, be = al[:m], be[:m - 1]
    y, on = op_small.ftk_device("exp", al, be)
    assert on
    check_close(y, al, be)


def test_device_exp_hands_back_when_it_must(op_small):
    """Non-finite T_k, or a spectrum too wide for the expansion: the kernel hands the case
    to the host (y = 0, on_device False); the solver then runs the host QL."""
    al = np.array([0.0, np.nan, 0.0])
    be = np.array([1.0, 1.0])
    y, on = op_small.ftk_device("exp", al, be)
    assert not on and np.all(y == 0.0)
    al = np.array([-1e6, 1e6, 0.0])
    y, on = op_small.ftk_device("exp", al, np.array([1.0, 1.0]))
    assert not on


def test_device_inv_kernel_alone_is_bitwise(op_small):
    """The device inv kernel alone (k_ftk_inv) on random tridiagonals: bitwise the host's."""
    rng = np.random.default_rng(9)
    for k in (1, 2, 5, 64, 500):
        al, be = rng.standard_normal(k), rng.uniform(0.1, 2.0, k - 1)
        y, on = op_small.ftk_device("inv", al, be)
        assert on and np.array_equal(y, ftk.INV(al, be))


def test_one_graph_exp_solve_matches_host_path(kkt5k):
    """The two-pass solve with the built-in exp as one device graph vs the same solve with
    the host QL between two graphs: same alpha / beta (pass one is shared), x within the
    exp tolerance; breakdown and zero b behave as on the host."""
    a = kkt5k.a
    b = harness_b(a)
    op = HipCsrOp(a)
    for k in (1, 2, 3, 30, 50, 120):
        xd = solvers.lanczos_two_pass(op, b, k, ftk.EXP)
        assert op.flags() & ONE_GRAPH
        op.set_device_ftk(0)
        xh = solvers.lanczos_two_pass(op, b, k, ftk.EXP)
        op.set_device_ftk(2)
        assert np.linalg.norm(xd - xh) <= 1e-12 * np.linalg.norm(xh), k
    with pytest.raises(tpl_amd.LanczosError):
        solvers.lanczos_two_pass(op, np.zeros_like(b), 10, ftk.EXP)
    # early breakdown: a b in a 3-dimensional invariant subspace
    d = sp.diags(np.repeat([1.0, 2.0, 3.0], 100)).tocsr()
    opd = HipCsrOp(d)
    bd = np.ones(300)
    xd = solvers.lanczos_two_pass(opd, bd, 40, ftk.EXP)
    assert opd.flags() & ONE_GRAPH
    assert alg.lanczos_pass_one(opd, bd, 40).steps_taken == 3
    xt = np.exp(np.repeat([1.0, 2.0, 3.0], 100))
    assert np.linalg.norm(xd - xt) <= 1e-12 * np.linalg.norm(xt)


def test_harness_ill_conditioned_exp(op_small):
    """The reference's hardest exp case (src/bin/stability.rs:113-119: diagonal spectrum
    in [-1000, -0.1], n = 10000, b = StdRng(42)): one device graph, x within the EVD's
    tolerance of the host path and of exp(A) b itself at the published accuracy level."""
    n = 10000
    lam = -1000.0 + (999.9 / (n - 1)) * np.arange(n)
    a = sp.diags(lam).tocsr()
    b = std_rng_vector(n)
    op = HipCsrOp(a)
    for k in (10, 70, 140, 200):
        xd = solvers.lanczos_two_pass(op, b, k, ftk.EXP)
        assert op.flags() & ONE_GRAPH
        op.set_device_ftk(0)
        xh = solvers.lanczos_two_pass(op, b, k, ftk.EXP)
        op.set_device_ftk(2)
        assert np.linalg.norm(xd - xh) <= 1e-11 * np.linalg.norm(xh), k
    xt = np.exp(lam) * b
    assert np.linalg.norm(xd - xt) / np.linalg.norm(xt) < 1e-6


def test_solvers_hand_exp_back_to_the_host():
    """Solver-level hand-back: a spectrum far too wide for the expansion
    (diag(-1e7 .. 0)) — the device kernel hands f(T_k) back, both solvers then run the host
    QL inside the same call, and x is bit for bit the host-path solve's (set_device_ftk(0));
    the one-graph flag (bit 5) is clear."""
    n = 2000
    lam = np.linspace(-1e7, 0.0, n)
    a = sp.diags(lam).tocsr()
    b = std_rng_vector(n)
    op = HipCsrOp(a)
    for solve in (solvers.lanczos_two_pass, solvers.lanczos):
        for k in (5, 40):
            x2 = solve(op, b, k, ftk.EXP)
            assert not op.flags() & ONE_GRAPH, (solve.__name__, k)
            op.set_device_ftk(0)
            xh = solve(op, b, k, ftk.EXP)
            op.set_device_ftk(2)
            assert np.array_equal(x2, xh), (solve.__name__, k)
            assert np.all(np.isfinite(x2))
    op.close()
