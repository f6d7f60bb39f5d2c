"""GPU: the one-graph two-pass solve — the built-in f = inv evaluated
on the device (k_ftk_inv) between the passes, no host round trip.

The device solver performs the host solver's operations in the same order
(tpl_ftk.cpp tpl_ftk_inv, the dgtsv scheme), so the contract is BITWISE: the same x as
the host-f path (two graphs around tpl_ftk_inv on the host) and as the canonical
oracle, for every steps_taken residue mod 3 (the last step's pending x terms are added
by k_p2_tail), under breakdown (the graph's step launches past steps_taken do
nothing), with live timing on (three graphs) and for the error cases.
Reference: src/solvers.rs:133-175, src/bin/tradeoff.rs:245-258.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import harness_b

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from oracle.rng import std_rng_vector  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
from tpl_amd import HipCsrOp, LanczosError, LanczosErrorKind, ftk, solvers  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


def same_bits(x, y):
    """Bitwise equality (NaN payloads included: T_1 = [0] is singular on the KKT runs)."""
    return x.shape == y.shape and np.array_equal(x.view(np.int64), y.view(np.int64))


def same_bits_nan(x, y):
    """Bitwise where finite or infinite; NaN at the same places (host and device may
    encode a NaN differently)."""
    nx, ny = np.isnan(x), np.isnan(y)
    return np.array_equal(nx, ny) and same_bits(x[~nx], y[~ny])


ONE_GRAPH = 32  # tpl_op_flags bit 5: the last two-pass solve ran as one device graph


def both_paths(op, b, k):
    op.set_device_ftk(True)
    xd = solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert op.flags() & ONE_GRAPH, "the one-graph path was not taken"
    op.set_device_ftk(False)
    xh = solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert not op.flags() & ONE_GRAPH
    op.set_device_ftk(2)
    return xd, xh


@pytest.mark.parametrize("k", [1, 2, 3, 4, 49, 50, 51, 52])
@pytest.mark.parametrize("rhs", ["harness", "rng"])
def test_device_inv_bitwise_every_tail(k, rhs, kkt5k):
    """steps_taken - 1 = 0..51 covers every pending-term count of the last step. With the
    harness b (alpha == 0) an odd k gives a singular T_k: y' and x are non-finite on both
    paths, and a NaN's encoding may differ between the host's and the device's
    division, so NaN positions are compared, every other value bit for bit."""
    a = kkt5k.a
    op = HipCsrOp(a)
    b = harness_b(a) if rhs == "harness" else std_rng_vector(a.shape[0])
    xd, xh = both_paths(op, b, k)
    assert same_bits_nan(xd, xh)
    if rhs == "rng" or k % 2 == 0:
        assert np.all(np.isfinite(xd)) and same_bits(xd, xh)
    xo = oracle.Operator(a, op.schedule()).lanczos_two_pass(b, k, ftk.INV)
    assert same_bits_nan(xd, xo)


def test_device_inv_50k_k200_and_repeat(kkt50k):
    a = kkt50k.a
    op = HipCsrOp(a)
    b = std_rng_vector(a.shape[0])
    xd, xh = both_paths(op, b, 200)
    assert same_bits(xd, xh)
    assert same_bits(solvers.lanczos_two_pass(op, b, 200, ftk.INV), xd)  # graph replay


def test_device_inv_breakdown_no_op_launches():
    """Pass one stops at steps_taken < k (invariant subspace): the remaining step
    launches of the one graph must leave x untouched."""
    rng = np.random.default_rng(5)
    n = 40
    a = sp.diags(np.repeat(np.arange(1.0, 11.0), 4)).tocsr()  # 10 distinct eigenvalues
    b = rng.standard_normal(n)
    op = HipCsrOp(a)
    for k in (12, 30):
        xd, xh = both_paths(op, b, k)
        assert same_bits(xd, xh)
        dec = tpl_amd.algorithms.lanczos_pass_one(op, b, k)
        assert dec.steps_taken <= 10
    assert np.linalg.norm(a @ xd - b) / np.linalg.norm(b) < 1e-10


def test_auto_mode(kkt5k):
    """Default (auto): one graph for the built-in inv up to k = 500 (round 5: the largest
    k measured no slower than the host path, profiles/r05_ftk_timing.txt), the host solver
    between two graphs above; mode 1 takes the device inv up to its LDS bound, 1365."""
    a = kkt5k.a
    op = HipCsrOp(a)
    b = std_rng_vector(a.shape[0])
    for k in (128, 129, 500):
        solvers.lanczos_two_pass(op, b, k, ftk.INV)
        assert op.flags() & ONE_GRAPH, k
    for k in (501, 1365):
        solvers.lanczos_two_pass(op, b, k, ftk.INV)
        assert not op.flags() & ONE_GRAPH, k
    op.set_device_ftk(1)
    solvers.lanczos_two_pass(op, b, 1365, ftk.INV)
    assert op.flags() & ONE_GRAPH
    solvers.lanczos_two_pass(op, b, 1366, ftk.INV)
    assert not op.flags() & ONE_GRAPH
    op.set_device_ftk(2)
    solvers.lanczos_two_pass(op, b, 50, ftk.EXP)  # the built-in exp: on the device too
    assert op.flags() & ONE_GRAPH
    solvers.lanczos_two_pass(op, b, 50, lambda al, be: ftk.EXP(al, be))  # a host f stays
    assert not op.flags() & ONE_GRAPH
    with pytest.raises(tpl_amd.TplError):
        op.set_device_ftk(3)


def test_device_inv_timed_three_graphs(kkt5k):
    a = kkt5k.a
    op = HipCsrOp(a)
    b = harness_b(a)
    op.set_device_ftk(1)
    x0 = solvers.lanczos_two_pass(op, b, 50, ftk.INV)
    op.enable_timing(True)
    x1 = solvers.lanczos_two_pass(op, b, 50, ftk.INV)
    p1_us, p2_us, n2 = op.pass_timing()
    op.enable_timing(False)
    assert same_bits(x0, x1)
    assert n2 == 49 and p1_us > 0 and p2_us > 0


@pytest.mark.parametrize("k", [11, 50])
def test_step_samples_live_pass_one(kkt50k, k):
    """tpl_op_step_samples (round 5): the launch stamps of 8 middle steps of a timed
    solve's pass-one graph give each kernel's start-to-start time; the two add up to the
    pass-one step the events around the whole pass measure, and the stamped graph gives
    the same bits as the untimed one-graph solve. A pass without stamps clears them."""
    a = kkt50k.a
    op = HipCsrOp(a)
    b = harness_b(a)
    x0 = solvers.lanczos_two_pass(op, b, k, ftk.INV)
    op.enable_timing(True)
    with pytest.raises(tpl_amd.TplError):
        op.step_samples()  # nothing timed yet
    for _ in range(3):
        x1 = solvers.lanczos_two_pass(op, b, k, ftk.INV)
        assert same_bits(x0, x1)
    s1, a1, ns = op.step_samples()
    p1_us, _, _ = op.pass_timing()
    assert ns == 8 and 0.5 < s1 < 100 and 0.5 < a1 < 100
    # the stamped steps are middle steps; the pass mean includes the prologue and step 1
    assert abs((s1 + a1) - p1_us / k) < 0.25 * (p1_us / k), (s1, a1, p1_us / k)
    op.set_device_ftk(0)  # host f: pass one without stamps
    solvers.lanczos_two_pass(op, b, k, ftk.INV)
    with pytest.raises(tpl_amd.TplError):
        op.step_samples()
    # a re-orthogonalised standard pass and an untimed one-graph solve clear
    # the stamps of an earlier timed solve too
    op.set_device_ftk(2)
    solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert op.step_samples()[2] == 8
    tpl_amd.algorithms.lanczos_standard(op, b, k, reorthogonalize=True)
    with pytest.raises(tpl_amd.TplError):
        op.step_samples()
    solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert op.step_samples()[2] == 8
    op.enable_timing(False)
    solvers.lanczos_two_pass(op, b, k, ftk.INV)
    with pytest.raises(tpl_amd.TplError):
        op.step_samples()


def test_device_inv_zero_b_error(kkt5k):
    op = HipCsrOp(kkt5k.a)
    with pytest.raises(LanczosError) as e:
        solvers.lanczos_two_pass(op, np.zeros(kkt5k.a.shape[0]), 10, ftk.INV)
    assert e.value.kind == LanczosErrorKind.INPUT_ERROR
    assert str(e.value) == "Invalid input parameter: Input vector `b` must not be a zero vector."
    # the operator stays usable
    b = harness_b(kkt5k.a)
    xd, xh = both_paths(op, b, 10)
    assert same_bits(xd, xh)


def test_device_inv_device_pointers(kkt5k):
    torch = pytest.importorskip("torch")
    a = kkt5k.a
    op = HipCsrOp(a)
    b = harness_b(a)
    op.set_device_ftk(1)
    x_host = solvers.lanczos_two_pass(op, b, 50, ftk.INV)
    bd = torch.from_numpy(b).cuda()
    xd = torch.empty_like(bd)
    from tpl_amd import _lib
    from tpl_amd.error import check
    check(_lib.tpl_lanczos_two_pass(op.handle, bd.data_ptr(), a.shape[0], 50, _lib.FTK_INV_PTR,
                                    None, xd.data_ptr(), _lib.TPL_MEM_DEVICE))
    torch.cuda.synchronize()
    assert same_bits(xd.cpu().numpy(), x_host)


def test_one_pass_device_f(kkt5k):
    """solvers::lanczos with a built-in f: f(T_k) on the device between the standard pass
    and the reconstruction GEMV (no host round trip; tpl_op_flags bit 5). inv is bitwise
    the host path (the same operations; y' unscaled, the GEMV multiplies by ||b||); exp is
    within the device exp's tolerance; zero b and early breakdown behave as on the host."""
    a = kkt5k.a
    op = HipCsrOp(a)
    b = std_rng_vector(a.shape[0])
    for k in (1, 2, 40, 128):
        xd = solvers.lanczos(op, b, k, ftk.INV)
        assert op.flags() & ONE_GRAPH
        op.set_device_ftk(False)
        xh = solvers.lanczos(op, b, k, ftk.INV)
        assert not op.flags() & ONE_GRAPH
        op.set_device_ftk(2)
        assert same_bits_nan(xd, xh), k
        xe = solvers.lanczos(op, b, k, ftk.EXP)
        assert op.flags() & ONE_GRAPH
        op.set_device_ftk(False)
        xeh = solvers.lanczos(op, b, k, ftk.EXP)
        op.set_device_ftk(2)
        assert np.linalg.norm(xe - xeh) <= 1e-12 * np.linalg.norm(xeh), k
        # one-pass and two-pass through the same device f (reference results/accuracy_*.csv
        # relative_solution_deviation ~ 1e-16)
        xt = solvers.lanczos_two_pass(op, b, k, ftk.EXP)
        assert np.linalg.norm(xe - xt) <= 1e-13 * np.linalg.norm(xt), k
    xd = solvers.lanczos(op, b, 500, ftk.INV)  # auto: the device inv up to k = 500
    assert op.flags() & ONE_GRAPH
    op.set_device_ftk(False)
    assert same_bits_nan(xd, solvers.lanczos(op, b, 500, ftk.INV))
    op.set_device_ftk(2)
    solvers.lanczos(op, b, 1366, ftk.INV)  # above: the host solver
    assert not op.flags() & ONE_GRAPH
    with pytest.raises(tpl_amd.LanczosError):
        solvers.lanczos(op, np.zeros_like(b), 10, ftk.INV)
    d = sp.diags(np.repeat([1.0, 2.0, 3.0], 50)).tocsr()
    opd = HipCsrOp(d)
    xd = solvers.lanczos(opd, np.ones(150), 20, ftk.INV)
    assert opd.flags() & ONE_GRAPH
    assert np.linalg.norm(xd - 1.0 / np.repeat([1.0, 2.0, 3.0], 50)) < 1e-12


def test_device_inv_headline_k500(kkt_tmp):
    """The headline workload (500k arcs, pinned order, k = 500) with the device inv forced:
    T_k's LU eliminated during pass one (k_p1_axpy's extra workgroup) and the back
    substitution with Markstein divisions — x bit for bit the host-f solve's, which the
    parity fixture pins (tests/golden/parity.json `headline`)."""
    import hashlib
    import json
    import os
    from conftest import load_kkt, ROOT
    a = load_kkt(500000, kkt_tmp).a
    b = harness_b(a)
    op = HipCsrOp(a)
    op.set_order_groups(13)
    xd, xh = both_paths(op, b, 500)
    assert same_bits(xd, xh)
    with open(os.path.join(ROOT, "tests", "golden", "parity.json")) as f:
        assert hashlib.sha256(xd.tobytes()).hexdigest()[:16] == json.load(f)["workloads"]["headline"]["x"]
    op.close()


@pytest.mark.parametrize("seed", range(6))
def test_device_inv_kernel_any_tridiagonal(kkt5k, seed):
    """k_ftk_inv alone (tpl_op_ftk_device: every elimination row on the device, then the
    back substitution) against the host solver on random T_k of 1..1365 rows: ordinary
    scales, 1e-300 / 1e300 scales (div_rn's range check hands those rows to IEEE
    division), exact zeros on the diagonal (pivoting, singular T_k: non-finite y' at the
    same positions) — y' bit for bit."""
    rng = np.random.default_rng(seed)
    op = HipCsrOp(kkt5k.a)
    for n in (1, 2, 3, 7, 64, 500, 1365):
        for scale in (1.0, 1e-300, 1e300, 1e-160):
            al = rng.standard_normal(n) * scale
            be = rng.standard_normal(max(n - 1, 0)) * scale
            if seed % 2:
                al[rng.random(n) < 0.5] = 0.0  # zero diagonal entries: row swaps, zeros in x
            yd, on = op.ftk_device("inv", al, be)
            assert on
            yh = ftk.INV(al, be)
            assert same_bits_nan(yd, yh), (n, scale)
    op.close()
