"""CPU: the locality row order's rule (tpl_layout.cpp locality_order, through the
host-only C ABI tpl_locality_order) against its restatement in conftest.locality_perm,
on the KKT fixtures, a skewed hub matrix, random hub matrices, and the edge cases
(no long rows, rows that reference other short rows, explicit thresholds, empty)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_kkt, locality_perm

tpl_amd = pytest.importorskip("tpl_amd")


def same(a, short_row_max=-1):
    got = tpl_amd.locality_order(a, short_row_max)
    ref = locality_perm(a.tocsr(), short_row_max)
    if ref is None:
        return got is None
    return got is not None and np.array_equal(got, ref)


@pytest.mark.parametrize("arcs", [5000, 50000])
def test_kkt_fixtures(kkt_tmp, arcs):
    a = load_kkt(arcs, kkt_tmp).a
    assert same(a)
    perm = tpl_amd.locality_order(a)
    assert np.array_equal(np.sort(perm), np.arange(a.shape[0]))
    lens = np.diff(a.tocsr().indptr)
    n_long = int(np.sum(lens > 4))
    assert np.all(lens[perm[-n_long:]] > 4)           # long rows last


def hub_matrix(seed, n=4000, hubs=12, diag=False):
    rng = np.random.default_rng(seed)
    rows = list(rng.integers(0, n, 3 * n))
    cols = list(rng.integers(0, n, 3 * n))
    for h in rng.choice(n, hubs, replace=False):
        c = rng.choice(n, int(rng.integers(50, 900)), replace=False)
        rows += [h] * len(c)
        cols += list(c)
    s = sp.coo_matrix((np.ones(len(rows)), (rows, cols)), shape=(n, n)).tocsr()
    a = (s + s.T).tocsr()
    if diag:
        a = (a + sp.identity(n)).tocsr()
    a.sum_duplicates()
    a.sort_indices()
    return a


@pytest.mark.parametrize("seed", range(8))
def test_random_hub_matrices(seed):
    assert same(hub_matrix(seed, diag=bool(seed % 2)))


@pytest.mark.parametrize("srm", [2, 8, 32])
def test_explicit_threshold(srm):
    assert same(hub_matrix(11), srm)


def test_no_long_rows_and_empty():
    n = 500
    a = sp.diags([np.ones(n - 1), 2 * np.ones(n), np.ones(n - 1)], [-1, 0, 1]).tocsr()
    assert tpl_amd.locality_order(a) is None
    assert tpl_amd.locality_order(sp.csr_matrix((0, 0))) is None


def test_tail_rows_keep_chunk_spans(kkt_tmp):
    """The 500k-like case in small: a short node row (one arc) goes last among the short
    rows, together with the arc that references it."""
    a = load_kkt(5000, kkt_tmp).a.tolil()
    n = a.shape[0]
    # make the last node row short: keep one of its arcs
    row = a.rows[n - 1]
    for c in row[1:]:
        a[n - 1, c] = 0
        a[c, n - 1] = 0
    a = a.tocsr()
    a.eliminate_zeros()
    assert same(a)
    perm = tpl_amd.locality_order(a)
    lens = np.diff(a.indptr)
    n_short = int(np.sum(lens <= 4))
    tail = set(perm[n_short - 2:n_short].tolist())
    assert n - 1 in tail


@pytest.mark.parametrize("groups", [1, 7, 16, 24, 5000])
def test_group_counts(kkt_tmp, groups):
    a = load_kkt(50000, kkt_tmp).a
    got = tpl_amd.locality_order(a, groups=groups)
    ref = locality_perm(a.tocsr(), groups=groups)
    assert np.array_equal(got, ref)
