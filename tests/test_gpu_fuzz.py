"""GPU: randomized parity sweep — many random symmetric matrices and layouts through
the HIP path, each checked BITWISE against the canonical oracle (P2): the SpMV, pass one
(alphas, betas, steps, ||b||), the two-pass x, and the one-pass x.

The shapes cover what the fixed tests do not: tiny and empty-row matrices, a single
long row, rows straddling the short/long threshold, many hubs that need several bins
per slice, non-integer values (fp64 storage) and small integers (int8 storage), explicit
short-row thresholds (wider sliced-ELL chunks, the generic chunk width), and every slice
count. Seeds are fixed, so a failure names a reproducible case.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
from tpl_amd import HipCsrOp, ftk, solvers  # noqa: E402
from tpl_amd import algorithms as alg  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


def random_symmetric(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 2, 3, 17, 300, 2048, 5000, 20000]))
    density = rng.uniform(0, 4)
    rows, cols = [], []
    for i in range(n):
        k = rng.poisson(density)
        rows += [i] * k
        cols += list(rng.integers(0, n, size=k))
    for _ in range(int(rng.integers(0, 12)) if n > 4 else 0):  # hubs
        h = int(rng.integers(0, n))
        c = rng.choice(n, size=int(min(n, rng.integers(5, 3000))), replace=False)
        rows += [h] * len(c)
        cols += list(c)
    ints = bool(rng.integers(0, 2))
    vals = (rng.integers(-3, 4, len(rows)).astype(np.float64) if ints
            else rng.standard_normal(len(rows)))
    s = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    diag = rng.integers(1, 3, n).astype(np.float64) if ints else rng.uniform(1, 2, n)
    a = (s + s.T + sp.diags(diag)).tocsr()
    a.sum_duplicates()
    a.sort_indices()
    return a, rng


def same_bits(x, y):
    x, y = np.asarray(x), np.asarray(y)
    return x.shape == y.shape and np.array_equal(x.view(np.int64), y.view(np.int64))


@pytest.mark.parametrize("seed", range(64))
def test_random_matrix_bitwise(seed):
    a, rng = random_symmetric(seed)
    n = a.shape[0]
    op = HipCsrOp(a)
    srm = int(rng.choice([-1, -1, 2, 8, 32]))      # -1: auto threshold
    if srm > 0:
        op.set_schedule(short_row_max=srm)
    slices = int(rng.choice([0, 1, 2, 4, 8]))
    if slices:
        op.set_slices(slices)
    o = oracle.Operator(a, op.schedule())
    x = rng.standard_normal(n)
    assert same_bits(op.apply(x), o.apply(x)), "spmv"
    b = rng.standard_normal(n)
    k = int(min(rng.integers(1, 60), 4 * n + 1))
    d = alg.lanczos_pass_one(op, b, k)
    al, be, st, bn, _ = o.pass_one(b, k)
    assert d.steps_taken == st and d.b_norm == bn
    assert same_bits(d.alphas, al) and same_bits(d.betas, be)
    xt = solvers.lanczos_two_pass(op, b, k, ftk.INV)
    assert same_bits(xt, o.lanczos_two_pass(b, k, ftk.INV)), "two-pass"
    xs = solvers.lanczos(op, b, k, ftk.INV)
    assert same_bits(xs, o.lanczos(b, k, ftk.INV)), "one-pass"
    op.close()
