"""KKT test-problem loader — mirror of ``src/utils/data_loader.rs``.

``load_kkt_system(dmx_path, qfc_path) -> KKTSystem`` (:211-259) parses a DIMACS
``.dmx`` network and a ``.qfc`` cost file with the reference's exact semantics
(native code in libtpl_amd.so, tpl_load_kkt_system) and returns the symmetric
operator A = [[D, E^T], [E, 0]] as a scipy CSR matrix. Note the reference's
``.qfc`` quirk (parse_qfc, :185-195): costs are read one per line after skipping
m lines, so qfcgen's 3-line files leave D empty.

Paths ending in ``.xz`` are decompressed to a temporary file first (the
committed fixtures under tests/golden/kkt are xz-compressed).
"""
from __future__ import annotations

import lzma
import os
import shutil
import tempfile
from ctypes import byref
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

from .. import _lib
from ..error import check


@dataclass
class KKTSystem:
    a: sp.csr_matrix      # A = [[D, E^T], [E, 0]], n = num_arcs + num_nodes
    num_nodes: int
    num_arcs: int


def _plain(path: str, tmpdir: str) -> str:
    if str(path).endswith(".xz"):
        out = os.path.join(tmpdir, os.path.basename(str(path))[:-3])
        with lzma.open(path, "rb") as src, open(out, "wb") as dst:
            shutil.copyfileobj(src, dst, 1 << 22)
        return out
    return str(path)


def _take(h) -> KKTSystem:
    try:
        n, nnz = h.n, h.nnz
        rp = np.ctypeslib.as_array(h.row_ptr, (n + 1,)).copy()
        ci = np.ctypeslib.as_array(h.col_idx, (max(nnz, 1),))[:nnz].copy()
        v = np.ctypeslib.as_array(h.vals, (max(nnz, 1),))[:nnz].copy()
        a = sp.csr_matrix((v, ci, rp), shape=(n, n))
        return KKTSystem(a=a, num_nodes=int(h.num_nodes), num_arcs=int(h.num_arcs))
    finally:
        _lib.tpl_csr_host_free(byref(h))


def load_kkt_system(dmx_path, qfc_path) -> KKTSystem:
    with tempfile.TemporaryDirectory(prefix="tpl_kkt_") as td:
        dmx = _plain(dmx_path, td)
        qfc = _plain(qfc_path, td)
        h = _lib.CsrHost()
        check(_lib.tpl_load_kkt_system(dmx.encode(), qfc.encode(), byref(h)))
        return _take(h)


def pargen_nodes(num_arcs: int) -> int:
    """Node count of a rho = 3 instance with m arcs (data/qcnd/pargen.c:41-50)."""
    return int(np.floor((1.0 + np.sqrt(1.0 + 8.0 * num_arcs / 0.75)) / 2.0))


def generate_kkt(num_arcs: int, num_nodes: int | None = None, seed: int = 42) -> KKTSystem:
    """Synthetic KKT instance (BASELINE.json configs[4], 5M arcs): uniform arcs u != v
    ordered by (tail, head), D empty, assembled like load_kkt_system (tpl_generate_kkt)."""
    p = pargen_nodes(num_arcs) if num_nodes is None else int(num_nodes)
    h = _lib.CsrHost()
    check(_lib.tpl_generate_kkt(int(num_arcs), p, int(seed), byref(h)))
    return _take(h)


def write_qfc_3line(path: str, m: int, seed: int = 0) -> None:
    """Write a qfcgen-format (3-line) .qfc for m arcs: line 1 = m, then one line of
    m fixed costs and one line of m quadratic costs (data/qcnd/qfcgen.c:209-218).
    With the reference's parse semantics this yields D = empty whatever the costs."""
    rng = np.random.default_rng(seed)
    fixed = rng.integers(1, 1000, size=m).astype(np.float64)
    quad = rng.uniform(1.0, 100.0, size=m)
    with open(path, "w") as f:
        f.write(f"{m}\n")
        f.write(" ".join(f"{c:f}" for c in fixed) + " \n")
        f.write(" ".join(f"{c:f}" for c in quad) + " \n")
