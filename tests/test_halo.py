"""Host-side coverage of the halo-exchange row blocks (tpl_dist_op_create_halo; SURVEY.md
§8(e) "a halo-exchange general form covers non-KKT matrices"), no GPU: the runtime's own
per-rank plans (tpl_plan_create, TPL_PLAN_HALO) hold the plain row blocks' rows and
layout — so the same reduction order, and the partition oracle's "rows" order pins the
halo runs too (tests/test_gpu_dist.py) — while the exchange moves only the halo."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "two-pass-lanczos_amd"))

from conftest import banded_hub, harness_b  # noqa: E402

EX_P1, EX_P2 = 4, 5  # TPL_KERNEL_EXCHANGE_P1 / _P2


def _brute_halo_width(a, starts):
    """max_q |B_q| by a plain loop over the rows (B_q: rows of q's block that a row of
    another block references)."""
    a = sp.csr_matrix(a)
    R = len(starts) - 1
    need = [set() for _ in range(R)]
    owner = np.searchsorted(starts, np.arange(a.shape[0]), "right") - 1
    for i in range(a.shape[0]):
        for c in a.indices[a.indptr[i]:a.indptr[i + 1]]:
            if owner[c] != owner[i]:
                need[owner[c]].add(int(c))
    return max(len(s) for s in need)


@pytest.fixture(scope="module")
def banded():
    return banded_hub(n=6000, hub_every=499)


@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 8])
def test_halo_plans_are_the_row_block_plans(banded, nranks):
    import tpl_amd
    from tpl_amd.dist import halo_width, partition
    st = partition(banded, nranks)
    H = halo_width(banded, st)
    assert H == _brute_halo_width(banded, st)
    for r in range(nranks):
        ph = tpl_amd.HostPlan(banded, mode="halo", nranks=nranks, rank=r)
        pr = tpl_amd.HostPlan(banded, mode="rows", nranks=nranks, rank=r)
        assert np.array_equal(ph.local_rows, pr.local_rows)
        assert np.array_equal(ph.local_rows, np.arange(st[r], st[r + 1]))
        sh, sr = ph.schedule(), pr.schedule()
        for key in ("short_rows", "long_rows", "G2", "E", "slices"):
            assert np.array_equal(np.asarray(sh[key]), np.asarray(sr[key])), key
        # one rank receives 8 H bytes per rank and SpMV (+ the two totals in pass one);
        # plain row blocks the whole padded block
        assert ph.algo_bytes(EX_P2) == 8 * nranks * H
        assert ph.algo_bytes(EX_P1) == 8 * nranks * (H + 2)
        ld = -(-int(np.diff(st).max()) // 64) * 64
        assert pr.algo_bytes(EX_P2) == 8 * nranks * ld
        ph.close()
        pr.close()
    if nranks > 1:
        assert 0 < H <= 2 * 150 * 7  # the hubs' reach bounds the halo
    else:
        assert H == 0


def test_halo_of_a_kkt_matrix_is_wide(kkt5k):
    """The KKT's node rows reference every arc: the halo is about a whole block, which is
    why "auto" takes the replicated partition (or, failing it, plain row blocks) there."""
    from tpl_amd.dist import halo_width, partition
    st = partition(kkt5k.a, 4)
    assert 2 * halo_width(kkt5k.a, st) > int(np.diff(st).max())


def test_block_diagonal_has_no_halo():
    import tpl_amd
    from tpl_amd.dist import halo_width, partition
    blk = sp.random(500, 500, density=0.02, random_state=3)
    blk = blk + blk.T + sp.eye(500) * 10
    a = sp.block_diag([blk, blk, blk, blk]).tocsr()
    a.sort_indices()
    st = np.array([0, 500, 1000, 1500, 2000])
    assert halo_width(a, st) == 0
    # the tpl_dist_partition split cuts inside the blocks; the halo is then small
    st2 = partition(a, 4)
    assert halo_width(a, st2) <= 500
    p = tpl_amd.HostPlan(a, mode="halo", nranks=4, rank=2)
    assert p.algo_bytes(EX_P2) == 8 * 4 * halo_width(a, st2)
    p.close()


def test_halo_plan_errors():
    import tpl_amd
    from tpl_amd.error import TplError
    a = sp.identity(3, format="csr")
    with pytest.raises(TplError):
        tpl_amd.HostPlan(a, mode="halo", nranks=4, rank=0)  # fewer rows than ranks
    with pytest.raises(TplError):
        tpl_amd.HostPlan(a, mode="halo", nranks=2, rank=2)  # bad rank


def test_halo_order_is_the_row_block_order(banded):
    """The partition oracle driven by the halo plans (the order a halo run reduces in)
    and by the row-block plans: the same alpha, beta and x bits."""
    import tpl_amd
    from partition_oracle import PartitionOracle
    from oracle import ftk_ref

    def recs(mode, R):
        out = []
        for r in range(R):
            p = tpl_amd.HostPlan(banded, mode=mode, nranks=R, rank=r)
            s = p.schedule()
            out.append({"rows": p.local_rows.copy(), "s_short": s["short_rows"],
                        "s_long": s["long_rows"], "s_G2": s["G2"], "s_E": s["E"],
                        "s_slices": s["slices"]})
            p.close()
        return out

    b = harness_b(banded)
    res = []
    for mode in ("halo", "rows"):
        po = PartitionOracle(banded, recs(mode, 3), "rows")
        al, be, s, bn = po.pass_one(b, 20)
        x = po.pass_two(b, al, be, s, bn, ftk_ref.inv(al, be) * bn)
        res.append((al, be, x))
    for u, v in zip(*res):
        assert np.array_equal(u, v)
    # and the partitioned order agrees with the single-process order to rounding
    import oracle
    xo = oracle.Operator(banded).lanczos_two_pass(b, 20, ftk_ref.inv)
    assert np.linalg.norm(res[0][2] - xo) <= 1e-12 * np.linalg.norm(xo)
