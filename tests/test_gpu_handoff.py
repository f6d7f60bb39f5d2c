"""GPU: targeted stress of the long-row hand-off (tpl_kcommon.h long_bin: sc1 piece
stores, vmcnt(0), one agent-scope add per row, the last arriver reads the slots with sc1
loads) and of the rank-total fold (fold_partials, the same pattern over a partial array).

MI355X_MICROARCH.md's valid-form table measured this hand-off with one workgroup per CU;
the engine's SpMV grid runs several (6 per CU at the 500k headline), which the table does not cover.
This test runs the guide's own acceptance recipe for that configuration: 8 column slices,
UNEVEN load across the slices (hub columns concentrated in two slices, so their bins finish
late and the finalising publisher varies), a grid of ~3,400 workgroups (~13 per CU: 1,152
short-row chunks, the bins of 2,400 hubs and 170k short-but-sliced rows), back-to-back
launches with the consumer L1-warm, and EVERY word of every result checked bit for bit
against the canonical oracle."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import harness_b

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402

tpl_amd = pytest.importorskip("tpl_amd")
from tpl_amd import HipCsrOp, ftk, solvers  # noqa: E402
from tpl_amd import algorithms as alg  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")


def uneven_matrix(n=760_000, hubs=2_400, seed=11):
    """Symmetric: short rows with 1-3 random entries, plus `hubs` long rows of 60..3,000
    entries whose columns fall 70 % into slice 1 and 20 % into slice 6 (of 8)."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    k = rng.integers(1, 4, size=n)
    rows.append(np.repeat(np.arange(n), k))
    cols.append(rng.integers(0, n, size=int(k.sum())))
    hub_ids = rng.choice(n, size=hubs, replace=False)
    s8 = n // 8
    for h in hub_ids:
        m = int(rng.integers(60, 3000))
        u = rng.random(m)
        c = np.where(u < 0.7, rng.integers(s8, 2 * s8, size=m),
                     np.where(u < 0.9, rng.integers(6 * s8, 7 * s8, size=m),
                              rng.integers(0, n, size=m)))
        rows.append(np.full(m, h))
        cols.append(c)
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    v = rng.integers(-3, 4, size=r.shape[0]).astype(np.float64)
    s = sp.coo_matrix((v, (r, c)), shape=(n, n)).tocsr()
    a = (s + s.T).tocsr()
    a.sum_duplicates()
    a.sort_indices()
    return a


@pytest.mark.timeout(600)
def test_handoff_uneven_8_slices_every_word():
    a = uneven_matrix()
    op = HipCsrOp(a)
    op.set_reorder(0)   # the caller's order: the hub columns stay clustered in their slices
    op.set_slices(8)
    sch = op.schedule()
    assert sch["slices"] == 8 and len(sch["long_rows"]) > 1000
    n_chunks = -(-len(sch["short_rows"]) // 512)
    long_nnz = int(np.diff(a.indptr)[sch["long_rows"]].sum())
    assert n_chunks + long_nnz // 2048 >= 1536  # chunks + bins: ~6 or more per CU
    o = oracle.Operator(a, sch)
    rng = np.random.default_rng(5)
    for trial in range(3):
        x = rng.standard_normal(a.shape[0])
        y_ref = o.apply(x)
        for rep in range(20):
            assert np.array_equal(op.apply(x), y_ref), (trial, rep)
    # back-to-back graph launches: every word of every step feeds the next step's gathers
    b = harness_b(a)
    d = alg.lanczos_pass_one(op, b, 120)
    al, be, s, bn, _ = o.pass_one(b, 120)
    assert d.steps_taken == s
    assert np.array_equal(d.alphas, al) and np.array_equal(d.betas, be)
    op.set_device_ftk(0)
    x = solvers.lanczos_two_pass(op, b, 120, ftk.INV)
    xo, _ = o.pass_two(b, al, be, s, bn, ftk.INV(al, be) * bn)
    assert np.array_equal(x, xo)
    op.close()
