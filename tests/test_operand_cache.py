"""The caller's own matrix as `operator` and the shared "auto" partition rule
(ADVICE r05), on the CPU.

* include/tpl.h tpl_operand_key: the same matrix object gives the same key, a copy (new
  arrays), a resized matrix or a change in a sampled word a new one — at O(samples) host
  cost, not O(nnz); a change in an unsampled word is the documented limit
  (``refresh_uploaded``).
* tpl_amd.operator.as_operator (the Rust shim's `HipOperand for SparseColMatRef` rule,
  integration/rust/hip.rs): the same matrix re-uses its upload, a changed one is uploaded
  again, ``refresh_uploaded`` forces it (uploads counted through a stub: no GPU here).
* tpl_dist_choose_partition: the one rule Python's mode="auto", C++'s and Rust's
  Partition::Auto all take — replicated for the KKT, halo for a banded matrix, rows when
  the halo is wider than half a block.
"""
import time

import numpy as np
import pytest
import scipy.sparse as sp

import tpl_amd
from tpl_amd import operator as opmod
from tpl_amd.dist import choose_partition, halo_width, partition


def _mat(n=20000, seed=0, per_row=5):
    """A random symmetric n x n CSR matrix with about 2 per_row entries per row."""
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n, n * per_row)
    c = rng.integers(0, n, n * per_row)
    a = sp.coo_matrix((rng.standard_normal(n * per_row), (r, c)), shape=(n, n)).tocsr()
    a = (a + a.T).tocsr()
    a.sort_indices()
    return a


def test_operand_key_identity_and_samples():
    a = _mat()
    k1 = opmod.operand_key(a)
    assert opmod.operand_key(a) == k1                      # the same object
    b = a.copy()
    kb = opmod.operand_key(b)
    assert kb[0] != k1[0] and kb[1] == k1[1]                # same contents, new arrays
    keep = a.data[0]
    a.data[0] += 1.0                                        # a sampled word (the first)
    assert opmod.operand_key(a)[1] != k1[1]
    a.data[0] = keep
    assert opmod.operand_key(a) == k1
    i = 7 * a.nnz // opmod.KEY_SAMPLES                      # an evenly spaced sample
    keep = a.data[i]
    a.data[i] = keep * 2.0 + 1.0
    assert opmod.operand_key(a)[1] != k1[1]
    a.data[i] = keep
    a.indices[a.nnz // 2 + 1] += 0                          # untouched: same key
    assert opmod.operand_key(a) == k1
    c = a[:-1, :-1].tocsr()                                 # another size
    assert opmod.operand_key(c)[0] != k1[0]


def test_operand_key_cost_is_not_o_nnz():
    """The key reads O(samples) words: a matrix 20x larger costs about the same."""
    small, big = _mat(20000), _mat(400000)
    def t(a):
        best = 1e9
        for _ in range(20):
            t0 = time.perf_counter()
            opmod.operand_key(a)
            best = min(best, time.perf_counter() - t0)
        return best
    ts, tb = t(small), t(big)
    assert big.nnz > 15 * small.nnz
    assert tb < 5 * ts + 2e-4, (ts, tb)


def test_as_operator_reuses_and_reuploads(monkeypatch):
    uploads = []

    class FakeOp(tpl_amd.HipCsrOp):
        def __init__(self, a, device=0):  # no GPU: count the uploads
            uploads.append(a)

        def __del__(self):
            pass
    monkeypatch.setattr(opmod, "_upload", lambda a, device: FakeOp(a, device))
    tpl_amd.refresh_uploaded()
    a = _mat()
    op1 = opmod.as_operator(a)
    assert opmod.as_operator(a) is op1 and len(uploads) == 1  # re-used
    a.data[0] = 3.5                                          # changed in a sampled word
    op2 = opmod.as_operator(a)
    assert op2 is not op1 and len(uploads) == 2
    b = a.copy()                                             # another matrix object
    assert opmod.as_operator(b) is not op2 and len(uploads) == 3
    assert opmod.as_operator(b) is opmod.as_operator(b) and len(uploads) == 3
    tpl_amd.refresh_uploaded()                               # explicit re-upload
    opmod.as_operator(b)
    assert len(uploads) == 4
    real = FakeOp(a)
    assert opmod.as_operator(real) is real                   # a HipCsrOp passes through
    with pytest.raises(TypeError):
        opmod.as_operator(np.eye(3))
    tpl_amd.refresh_uploaded()


def test_auto_partition_rule(kkt5k):
    from conftest import banded_hub
    banded_hub = banded_hub()
    assert choose_partition(kkt5k.a, 2) == "replicated"
    assert choose_partition(kkt5k.a, 8) == "replicated"
    # banded with hub rows: the halo is narrow against the blocks (tests/test_halo.py)
    for r in (2, 4, 8):
        st = partition(banded_hub, r)
        assert 2 * halo_width(banded_hub, st) <= int(np.diff(st).max())
        assert choose_partition(banded_hub, r) == "halo"
    # a random symmetric matrix references everything: the halo is about a whole block
    a = _mat(4000, 1)
    st = partition(a, 4)
    assert 2 * halo_width(a, st) > int(np.diff(st).max())
    assert choose_partition(a, 4) == "rows"
