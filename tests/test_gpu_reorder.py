"""GPU: the locality row order (tpl_op_set_reorder, include/tpl.h).

The device holds P A P^T and permutes every vector at the boundary. Checked here:
  * the permutation is the rule restated in conftest.locality_perm;
  * with the order on (default) and off, every result is bitwise the oracle's in that
    operator's own layout (P2), and the two agree with each other to rounding (the
    permutation changes the summation order, nothing else);
  * everything the caller sees is in the caller's row order: apply's y, pass one's V_k,
    pass two's basis, the step callback's V_k view, host and device memory alike.
"""
import numpy as np
import pytest

from conftest import canon_schedule, harness_b, locality_perm

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
import torch  # noqa: E402
from tpl_amd import HipCsrOp, ftk, solvers  # noqa: E402
from tpl_amd import algorithms as alg  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


def same_bits(x, y):
    x, y = np.asarray(x), np.asarray(y)
    return x.shape == y.shape and np.array_equal(x.view(np.int64), y.view(np.int64))


@pytest.fixture(scope="module")
def ops(kkt50k):
    a = kkt50k.a
    on = HipCsrOp(a)
    off = HipCsrOp(a)
    off.set_reorder(False)
    yield a, on, off
    on.close()
    off.close()


def test_flag_and_permutation(ops):
    a, on, off = ops
    assert on.flags() & 64 and not off.flags() & 64
    perm = on.schedule()["perm"]
    assert perm is not None and np.array_equal(perm, locality_perm(a))
    assert np.array_equal(np.sort(perm), np.arange(a.shape[0]))
    assert off.schedule()["perm"] is None
    # the rule's schedule on P A P^T is the live one
    ref = canon_schedule(a, reorder=True)
    sch = on.schedule()
    for key in ("short_rows", "long_rows"):
        assert np.array_equal(sch[key], ref[key])
    assert (sch["G2"], sch["E"], sch["slices"]) == (ref["G2"], ref["E"], ref["slices"])


def test_no_long_rows_is_identity():
    import scipy.sparse as sp
    n = 3000
    a = sp.diags([np.ones(n - 1), 2 * np.ones(n), np.ones(n - 1)], [-1, 0, 1]).tocsr()
    op = HipCsrOp(a)
    assert op.schedule()["perm"] is None and not op.flags() & 64
    op.close()


def test_both_orders_bitwise_and_close(ops):
    a, on, off = ops
    n = a.shape[0]
    b = harness_b(a)
    x = np.random.default_rng(3).standard_normal(n)
    k = 80
    res = {}
    for name, op in (("on", on), ("off", off)):
        o = oracle.Operator(a, op.schedule())
        y = op.apply(x)
        assert same_bits(y, o.apply(x)), name
        d = alg.lanczos_pass_one(op, b, k)
        al, be, st, bn, _ = o.pass_one(b, k)
        assert d.steps_taken == st and same_bits(d.alphas, al) and same_bits(d.betas, be)
        assert d.b_norm == bn
        xt = solvers.lanczos_two_pass(op, b, k, ftk.INV)
        assert same_bits(xt, o.lanczos_two_pass(b, k, ftk.INV)), name
        xs = solvers.lanczos(op, b, k, ftk.INV)
        assert same_bits(xs, o.lanczos(b, k, ftk.INV)), name
        res[name] = (y, d.alphas, xt)
    ref = a @ x
    for name in res:
        assert np.linalg.norm(res[name][0] - ref) <= 1e-13 * np.linalg.norm(ref)
    assert np.allclose(res["on"][1][:20], res["off"][1][:20], rtol=1e-10, atol=0)
    xt_on, xt_off = res["on"][2], res["off"][2]
    assert np.linalg.norm(xt_on - xt_off) <= 1e-8 * np.linalg.norm(xt_off)


def test_basis_in_caller_order(ops):
    """V_k of pass one and pass two's regenerated basis come back in the caller's order:
    v_1 = b / ||b|| row for row, and A V - V T holds row for row."""
    a, on, _ = ops
    b = harness_b(a)
    k = 40
    out = alg.lanczos_standard(on, b, k)
    V = np.asarray(out.v_k)
    d = out.decomposition
    assert same_bits(V[:, 0], b / d.b_norm) or np.allclose(V[:, 0], b / d.b_norm, rtol=1e-15)
    s = d.steps_taken
    T = np.diag(d.alphas) + np.diag(d.betas[:s - 1], 1) + np.diag(d.betas[:s - 1], -1)
    R = a @ V[:, :s - 1] - V @ T[:, :s - 1]
    assert np.linalg.norm(R) < 1e-10 * np.linalg.norm(V)
    o = oracle.Operator(a, on.schedule())
    _, _, _, _, Vo = o.pass_one(b, k, store_basis=True)
    assert same_bits(V, Vo)
    y = np.random.default_rng(5).standard_normal(s)
    x2 = alg.lanczos_pass_two_with_basis(on, b, d, y)
    xo, Vo2 = o.pass_two(b, d.alphas, d.betas, s, d.b_norm, y, store_basis=True)
    assert same_bits(x2.x_k, xo) and same_bits(x2.v_k, Vo2) and same_bits(x2.v_k, V)


def test_callback_view_in_caller_order(ops):
    a, on, _ = ops
    b = harness_b(a)
    seen = []

    def cb(kk, view, t):
        seen.append(view.numpy()[:, kk - 1].copy())
        return kk < 23

    out = alg.lanczos_standard(on, b, 60, callback=cb)
    V = np.asarray(out.v_k)
    assert out.decomposition.steps_taken == 23 and len(seen) == 23
    for j, col in enumerate(seen):
        assert same_bits(col, V[:, j]), j


def test_device_memory_vectors(ops):
    """torch (device) inputs and outputs take the device-side permutation path."""
    a, on, _ = ops
    b = harness_b(a)
    x = np.random.default_rng(9).standard_normal(a.shape[0])
    yd = on.apply(torch.from_numpy(x).cuda())
    assert same_bits(yd.cpu().numpy(), on.apply(x))
    bd = torch.from_numpy(b).cuda()
    xd = solvers.lanczos_two_pass(on, bd, 50, ftk.INV)
    assert same_bits(xd.cpu().numpy(), solvers.lanczos_two_pass(on, b, 50, ftk.INV))
    out_d = alg.lanczos_standard(on, bd, 30)
    out_h = alg.lanczos_standard(on, b, 30)
    assert same_bits(out_d.v_k.cpu().numpy(), np.asarray(out_h.v_k))


def test_modes(kkt5k):
    op = HipCsrOp(kkt5k.a)
    assert op.flags() & 64                       # auto: on below 2^20 rows
    with pytest.raises(Exception):
        op.set_reorder(3)
    op.set_reorder(0)
    assert not op.flags() & 64
    op.set_reorder(2)
    assert op.flags() & 64
    op.close()


def test_toggle_rebuilds(kkt5k):
    a = kkt5k.a
    op = HipCsrOp(a)
    b = harness_b(a)
    x_on = solvers.lanczos_two_pass(op, b, 30, ftk.INV)
    op.set_reorder(False)
    assert op.schedule()["perm"] is None
    x_off = solvers.lanczos_two_pass(op, b, 30, ftk.INV)
    op.set_reorder(True)
    assert same_bits(solvers.lanczos_two_pass(op, b, 30, ftk.INV), x_on)
    assert np.linalg.norm(x_on - x_off) <= 1e-9 * np.linalg.norm(x_off)
    op.close()


def test_tune_order(kkt50k):
    """tpl_op_tune_order keeps one of the candidates, switches the order on, and the
    tuned operator is bitwise the oracle's on its own permutation."""
    a = kkt50k.a
    op = HipCsrOp(a)
    op.set_reorder(0)
    g, us = op.tune_order([12, 16, 20], iters=20)
    assert g in (12, 16, 20) and us > 0 and op.flags() & 64
    sch = op.schedule()
    assert np.array_equal(sch["perm"], tpl_amd.locality_order(a, groups=g))
    b = harness_b(a)
    o = oracle.Operator(a, sch)
    assert same_bits(solvers.lanczos_two_pass(op, b, 40, ftk.INV), o.lanczos_two_pass(b, 40, ftk.INV))
    with pytest.raises(Exception):
        op.tune_order([0])
    op.close()
