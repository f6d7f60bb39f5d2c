"""CPU checks of the partitioned-order restatement (tests/partition_oracle.py) that the
multi-GPU GPU tests compare against bit for bit:

* one rank, row blocks: the partitioned order IS the single-GPU canonical order (the
  rank total of a single rank passes through partials() unchanged), so the restatement
  must reproduce the canonical oracle bit for bit;
* two and three ranks, both partitions: the same Krylov process as the reference order
  (faithful oracle) within 1e-10 on the 5k instance, before its chaotic onset.
Layouts come from the device rule restated in conftest (canon_schedule)."""
import numpy as np
import pytest
import scipy.sparse as sp

import oracle
from oracle import ftk_ref
from conftest import canon_schedule, elem_layout, harness_b, short_row_threshold
from partition_oracle import PartitionOracle

K = 40


def _block_record(a, r0, r1):
    """rows-mode record of the rank owning rows [r0, r1): the device layout rule on the
    block (short/long by the block's own threshold; slices over the global columns)."""
    blk = sp.csr_matrix(a[r0:r1])
    lens = np.diff(blk.indptr)
    T = short_row_threshold(lens)
    sq = canon_schedule(a)          # slice count: a function of the global column count
    n = r1 - r0
    g2, E = elem_layout(n)
    return {"rows": np.arange(r0, r1), "s_short": np.nonzero(lens <= T)[0].astype(np.int32),
            "s_long": np.nonzero(lens > T)[0].astype(np.int32), "s_G2": g2, "s_E": E,
            "s_slices": sq["slices"]}


def _replicated_records(a, cuts):
    """replicated-mode records: rank r owns the short rows S[cuts[r]:cuts[r+1]] plus all
    long rows (local vector [short | long]); layout: long rows from ns on."""
    lens = np.diff(a.indptr)
    T = short_row_threshold(lens)
    S = np.nonzero(lens <= T)[0]
    L = np.nonzero(lens > T)[0]
    recs = []
    for r in range(len(cuts) - 1):
        rows = np.concatenate([S[cuts[r]:cuts[r + 1]], L])
        ns = cuts[r + 1] - cuts[r]
        n = rows.shape[0]
        g2, E = elem_layout(n)
        s = 1
        while s < 8 and n * 8.0 / s > 512 * 1024:
            s *= 2
        recs.append({"rows": rows, "s_short": np.arange(ns, dtype=np.int32),
                     "s_long": np.arange(ns, n, dtype=np.int32), "s_G2": g2, "s_E": E,
                     "s_slices": s})
    return recs


def test_one_rank_rows_is_canonical(kkt5k):
    a = kkt5k.a
    b = harness_b(a)
    po = PartitionOracle(a, [_block_record(a, 0, a.shape[0])], "rows")
    al, be, s, bn = po.pass_one(b, K)
    o = oracle.Operator(a, canon_schedule(a))
    al2, be2, s2, bn2, _ = o.pass_one(b, K)
    assert s == s2 and bn == bn2
    assert np.array_equal(al, al2) and np.array_equal(be, be2)
    y = ftk_ref.inv(al, be) * bn
    x = po.pass_two(b, al, be, s, bn, y)
    x2, _ = o.pass_two(b, al2, be2, s2, bn2, y)
    assert np.array_equal(x, x2)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["rows", "replicated"])
def test_partitioned_orders_vs_reference_order(kkt5k, world, mode):
    a = kkt5k.a
    n = a.shape[0]
    b = harness_b(a)
    if mode == "rows":
        cuts = [n * r // world for r in range(world + 1)]
        recs = [_block_record(a, cuts[r], cuts[r + 1]) for r in range(world)]
    else:
        ns = int(np.sum(np.diff(a.indptr) <= short_row_threshold(np.diff(a.indptr))))
        recs = _replicated_records(a, [ns * r // world for r in range(world + 1)])
    po = PartitionOracle(a, recs, mode)
    al, be, s, bn = po.pass_one(b, K)
    of = oracle.Operator(a)
    alf, bef, sf, bnf, _ = of.pass_one(b, K)
    assert s == sf
    np.testing.assert_allclose(be, bef, rtol=1e-10)
    np.testing.assert_allclose(al, alf, rtol=0, atol=1e-10)
    y = ftk_ref.inv(al, be) * bn
    x = po.pass_two(b, al, be, s, bn, y)
    xf, _ = of.pass_two(b, alf, bef, sf, bnf, ftk_ref.inv(alf, bef) * bnf)
    assert np.linalg.norm(x - xf) <= 1e-10 * np.linalg.norm(xf)
    # SpMV of the partitioned order: +-1 values, exact products
    v = np.cos(np.arange(n))
    np.testing.assert_allclose(po.spmv(v), a @ v, rtol=1e-13, atol=1e-12)
