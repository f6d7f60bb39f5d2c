"""Shared test setup.

Marker ``gpu``: needs an MI355X (run with ``-m gpu``); everything else runs on CPU.
"""
import hashlib
import lzma
import os
import sys

import numpy as np
import pytest

# Under pytest-xdist every worker would start one OpenMP thread per core in the oracle
# library, and the spin-waiting teams oversubscribe the CPUs (measured: the accuracy-CSV
# test 0.9 s alone, 676 s with -n 4). One thread per worker; set before libgomp loads.
if os.environ.get("PYTEST_XDIST_WORKER"):
    os.environ.setdefault("OMP_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "two-pass-lanczos_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
KKT_DIR = os.path.join(GOLDEN, "kkt")
REF_RESULTS = os.path.join(GOLDEN, "reference_results")
ELEM_ROWS = 2048   # kElemRows (two-pass-lanczos_amd/csrc/tpl_device.h): rows per element-wise block
ELEM_MIN_BLOCKS = 192  # kElemMinBlocks
CHUNK_ROWS = 512   # kChunkRows


def elem_layout(n, max_g2=1024):
    """(G2, E) of the element-wise kernels (tpl_layout.cpp build_layout): kElemRows rows
    per block, halved down to 512 while that leaves fewer than kElemMinBlocks blocks."""
    er = ELEM_ROWS
    while er > 512 and -(-n // er) < ELEM_MIN_BLOCKS:
        er //= 2
    g2 = max(1, min(max_g2, -(-n // er)))
    per = -(-n // g2)
    return g2, max(512, (per + 511) // 512 * 512)

# md5 of the decompressed netgen .dmx files (regenerated from the reference's own
# netgen sources + recorded .par seeds; tests/golden/make_fixtures.py)
KKT_MD5 = {
    5000: "b227b77b86336c8feba472d62304a499",
    50000: "d3724d6d6ea2d393f640ff07801d5deb",
    500000: "0266d4c66c21f949db1ac54883378c25",
}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD MI355X (gfx950) GPU")


def kkt_paths(arcs: int, tmpdir: str):
    """(dmx.xz path, 3-line qfc path) for a committed netgen instance."""
    from tpl_amd.utils.data_loader import write_qfc_3line
    dmx = os.path.join(KKT_DIR, f"netgen-{arcs}-3.dmx.xz")
    qfc = os.path.join(tmpdir, f"netgen-{arcs}-3.qfc")
    if not os.path.exists(qfc):
        write_qfc_3line(qfc, arcs)
    return dmx, qfc


_KKT_CACHE = {}


SYNTH_SEED = 42  # BASELINE configs[4]: tpl_generate_kkt(5_000_000, seed 42), as bench.py


def load_kkt(arcs: int, tmpdir: str):
    """The netgen instance of `arcs` arcs (5k / 50k / 500k fixtures), or — for any
    other size, e.g. configs[4]'s 5M arcs — the build's synthetic generator."""
    if arcs not in _KKT_CACHE:
        from tpl_amd.utils.data_loader import generate_kkt, load_kkt_system
        if arcs in KKT_MD5:
            dmx, qfc = kkt_paths(arcs, tmpdir)
            _KKT_CACHE[arcs] = load_kkt_system(dmx, qfc)
        else:
            _KKT_CACHE[arcs] = generate_kkt(arcs, seed=SYNTH_SEED)
    return _KKT_CACHE[arcs]


def banded_hub(n=20000, w=3, hub_every=997, hub_half=150, hub_step=7, seed=5):
    """A symmetric, diagonally dominant banded matrix (half-bandwidth w, uniform random
    values) with a long "hub" row every hub_every rows whose entries reach
    hub_half * hub_step columns to either side: a matrix without the KKT structure, whose
    row blocks need only a narrow halo (tpl_dist_op_create_halo) — and long rows (bins)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for k in range(1, w + 1):
        i = np.arange(n - k)
        rows.append(i)
        cols.append(i + k)
    off = np.arange(1, hub_half + 1) * hub_step
    for h in range(hub_every // 2, n, hub_every):
        j = h + off[h + off < n]
        rows.append(np.full(len(j), h))
        cols.append(j)
        j = h - off[h - off >= 0]
        rows.append(j)
        cols.append(np.full(len(j), h))
    r, c = np.concatenate(rows), np.concatenate(cols)
    up = sp.coo_matrix((rng.uniform(-1.0, 1.0, len(r)), (r, c)), shape=(n, n)).tocsr()
    up.sum_duplicates()
    a = up + up.T
    a = (a + sp.diags(np.asarray(abs(a).sum(axis=1)).ravel() + 1.0)).tocsr()
    a.sort_indices()
    return a


def block_diag_spd(blocks=3, m=1500, seed=7):
    """blocks independent SPD blocks of m rows (band + a long row each): a partition at
    the block boundaries needs no halo at all."""
    import scipy.sparse as sp
    parts = [banded_hub(n=m, hub_every=m // 3, seed=seed + i) for i in range(blocks)]
    a = sp.block_diag(parts).tocsr()
    a.sort_indices()
    return a


def harness_b(a):
    """b = A (1/sqrt(n)) 1, as src/bin/tradeoff.rs:235-236 (row-sequential sums)."""
    n = a.shape[0]
    x_true = np.full(n, 1.0 / np.sqrt(n))
    return a @ x_true


@pytest.fixture(scope="session")
def kkt_tmp(tmp_path_factory):
    return str(tmp_path_factory.mktemp("kkt"))


@pytest.fixture(scope="session")
def kkt5k(kkt_tmp):
    return load_kkt(5000, kkt_tmp)


@pytest.fixture(scope="session")
def kkt50k(kkt_tmp):
    return load_kkt(50000, kkt_tmp)


def md5_of_xz(path):
    h = hashlib.md5()
    with lzma.open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def short_row_threshold(lens, requested=-1):
    """tpl_runtime.cpp short_row_threshold: clamp(2 * lower-median row nnz, 4, 32)."""
    if requested > 0:
        return requested
    if lens.size == 0:
        return 32
    m = int(np.sort(np.minimum(lens, 33))[(lens.size + 1) // 2 - 1])
    return max(4, min(32, 2 * m))


def locality_perm(a, short_row_max=-1, groups=16):
    """tpl_layout.cpp locality_order restated: short rows sorted by (tail, group(lo),
    group(hi), lo, hi, row) — lo / hi the smallest / largest rank, among the long rows, of
    a long column the row references (none: after all others), group = rank //
    ceil(n_long / groups), tail = the row references another short row — then the long
    rows ascending.
    None when that is the identity (or no long rows)."""
    a = a.tocsr()
    n = a.shape[0]
    lens = np.diff(a.indptr)
    T = short_row_threshold(lens, short_row_max)
    long_ = np.nonzero(lens > T)[0]
    if long_.size == 0:
        return None
    rank = np.full(n, -1, dtype=np.int64)
    rank[long_] = np.arange(long_.size)
    big = np.iinfo(np.int32).max
    rows = np.repeat(np.arange(n), lens)
    r = rank[a.indices]
    m = r >= 0
    lo = np.full(n, big, dtype=np.int64)
    hi = np.full(n, -1, dtype=np.int64)
    np.minimum.at(lo, rows[m], r[m])
    np.maximum.at(hi, rows[m], r[m])
    hi[hi < 0] = big
    tail = np.zeros(n, dtype=np.int64)
    np.maximum.at(tail, rows, ((r < 0) & (a.indices != rows)).astype(np.int64))
    gsize = -(-long_.size // groups)
    grp = lambda x: np.where(x == big, big, x // gsize)
    short = np.nonzero(lens <= T)[0]
    o = np.lexsort((short, hi[short], lo[short], grp(hi[short]), grp(lo[short]), tail[short]))
    perm = np.concatenate([short[o], long_]).astype(np.int32)
    return None if np.array_equal(perm, np.arange(n)) else perm


def canon_schedule(a, short_row_max=-1, max_g2=1024, reorder=False):
    """The device's layout rule (two-pass-lanczos_amd/csrc/tpl_layout.cpp, build_layout)
    restated, for oracle runs without a GPU. The GPU tests take the layout from the
    live operator instead (HipCsrOp.schedule()). reorder: the single-GPU operator's
    default locality order (tpl_op_set_reorder) — the rule is then applied to P A P^T and
    the schedule carries "perm"."""
    if reorder:
        perm = locality_perm(a, short_row_max)
        if perm is not None:
            s = canon_schedule(a.tocsr()[perm][:, perm].tocsr(), short_row_max, max_g2)
            s["perm"] = perm
            return s
    rp = a.indptr
    n = a.shape[0]
    lens = np.diff(rp)
    T = short_row_threshold(lens, short_row_max)
    short = np.nonzero(lens <= T)[0].astype(np.int32)
    long_ = np.nonzero(lens > T)[0].astype(np.int32)
    g2, E = elem_layout(n, max_g2)
    return {"short_rows": short, "long_rows": long_, "G2": g2, "E": E,
            "slices": auto_slices(a, long_), "perm": None}


def auto_slices(a, long_rows, bin_max=7936):
    """tpl_runtime.cpp auto_slices + build_layout: the fewest of 1, 2, 4, 8 column slices
    whose share of the vector (8 n bytes) fits 512 KiB, doubled while a (long row, slice)
    piece holds more than bin_max entries."""
    n = a.shape[0]
    s = 1
    while s < 8 and n * 8.0 / s > 0.5 * 1024 * 1024:
        s *= 2

    def widest(S):
        w = 0
        for r in long_rows:
            c = a.indices[a.indptr[r]:a.indptr[r + 1]].astype(np.int64)
            sl = np.searchsorted(np.array([n * k // S for k in range(1, S)], dtype=np.int64),
                                 c, side="right")
            w = max(w, int(np.bincount(sl, minlength=S).max()) if c.size else 0)
        return w

    while s < 8 and widest(s) > bin_max:
        s *= 2
    return s
