"""CPU: the drop-in boundary — C-ABI library loads and exports every symbol the
header declares, the native loader matches the reference's parse semantics, the
built-in f(T_k) solvers match LAPACK, and the error texts match src/error.rs.
No compute on the GPU here."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import KKT_DIR, KKT_MD5, ROOT, kkt_paths, md5_of_xz

import tpl_amd
from tpl_amd import _lib
from tpl_amd.error import DataLoaderError, LanczosError
from tpl_amd.utils.data_loader import load_kkt_system

from oracle import ftk_ref, kkt_ref


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "tpl.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tpl_[a-z0-9_]+)\s*\(", txt)) - {"tpl_ftk_fn", "tpl_step_cb"})


def test_library_exports_every_header_symbol():
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert set(syms) == set(_lib.EXPORTED)
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", nm), s


def test_header_constants_match_python_mirror():
    """Every TPL_KERNEL_* / TPL_MEM_* enumerator of the header has the same value in
    the ctypes mirror (tpl_amd._lib), so the Python side passes what the ABI means."""
    txt = open(os.path.join(ROOT, "include", "tpl.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    consts = dict(re.findall(r"\b(TPL_(?:KERNEL|MEM)_[A-Z0-9_]+)\s*=\s*(\d+)", txt))
    assert {"TPL_KERNEL_EXCHANGE_P1", "TPL_KERNEL_EXCHANGE_P2"} <= set(consts)
    for name, v in consts.items():
        assert getattr(_lib, name) == int(v), name


def test_library_is_gfx950_code_object():
    """The fat binary embeds an amdgcn code object for gfx950 (and nothing else)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"--gfx942" not in blob and b"--gfx90a" not in blob


def test_version_and_no_device_is_reported_cleanly():
    assert b"gfx950" in _lib.tpl_version()
    if tpl_amd.device_count() == 0:
        with pytest.raises(tpl_amd.TplError):
            tpl_amd.HipCsrOp(sp.identity(3).tocsr())


def test_error_detail_rebuilds_every_variant():
    """tpl_last_error_detail (the fields of a LanczosErrorKind across the C ABI): the
    Python mirror rebuilds each variant from the fields alone and gets the reference's
    Display text; a host-only call records its status, and success resets it."""
    from tpl_amd.error import from_detail
    base = {"status": 0, "message": "", "inner": "", "param_name": "", "expected": 0,
            "actual": 0, "operator_cols": 0, "vector_rows": 0, "breakdown_step": 0}
    cases = [
        (dict(status=_lib.TPL_ERR_PARAMETER_MISMATCH, param_name="y_k", expected=10, actual=9),
         "Parameter mismatch: `y_k` expects size 10, but got 9."),
        (dict(status=_lib.TPL_ERR_DIMENSION_MISMATCH, operator_cols=100, vector_rows=99),
         "Dimension mismatch: operator has 100 columns but vector has 99 rows."),
        (dict(status=_lib.TPL_ERR_INPUT, inner="The initial vector `b` must not be a zero vector."),
         "Invalid input parameter: The initial vector `b` must not be a zero vector."),
        (dict(status=_lib.TPL_ERR_SOLVER, inner="Custom solver failed"),
         "The user-provided f(T_k) solver failed: Custom solver failed"),
        (dict(status=_lib.TPL_ERR_EVD, inner="NoConvergence"),
         "A numerical error occurred during the eigendecomposition of T_k: NoConvergence"),
        (dict(status=_lib.TPL_ERR_BREAKDOWN, breakdown_step=42),
         "Lanczos iteration breakdown at step 42: Beta coefficient is zero. The Krylov "
         "subspace is invariant."),
    ]
    for fields, text in cases:
        assert str(from_detail({**base, **fields})) == text
    # a real failure through the C ABI (host-only entry point: no GPU needed)
    from ctypes import POINTER, byref, c_int32, c_int64
    rp = np.array([0, 2, 1], dtype=np.int64)  # decreasing row_ptr
    ci = np.array([1, 0], dtype=np.int32)
    perm = np.zeros(2, dtype=np.int32)
    applied = c_int32()
    st = _lib.tpl_locality_order(2, rp.ctypes.data_as(POINTER(c_int64)),
                                 ci.ctypes.data_as(POINTER(c_int32)), 0, 0,
                                 perm.ctypes.data_as(POINTER(c_int32)), byref(applied))
    assert st == _lib.TPL_ERR_INVALID_ARGUMENT
    d = _lib.last_error_detail()
    assert d["status"] == st and d["message"] == _lib.last_error() == "row_ptr not monotone"
    rp[:] = [0, 1, 2]
    assert _lib.tpl_locality_order(2, rp.ctypes.data_as(POINTER(c_int64)),
                                   ci.ctypes.data_as(POINTER(c_int32)), 0, 0,
                                   perm.ctypes.data_as(POINTER(c_int32)), byref(applied)) == 0
    assert _lib.last_error_detail()["status"] == 0


@pytest.mark.parametrize("arcs", [5000, 50000, 500000])
def test_fixture_md5(arcs):
    assert md5_of_xz(os.path.join(KKT_DIR, f"netgen-{arcs}-3.dmx.xz")) == KKT_MD5[arcs]


def test_native_loader_matches_restatement(kkt_tmp):
    dmx, qfc = kkt_paths(5000, kkt_tmp)
    k = load_kkt_system(dmx, qfc)
    import lzma
    plain = os.path.join(kkt_tmp, "5k.dmx")
    with lzma.open(dmx) as f, open(plain, "wb") as g:
        g.write(f.read())
    a, p, m = kkt_ref.load_kkt_system(plain, qfc)
    assert (k.num_nodes, k.num_arcs) == (p, m) == (115, 5000)
    assert k.a.shape == (5115, 5115) and k.a.nnz == 20000  # D empty (qfc quirk)
    assert (k.a != a).nnz == 0
    assert np.array_equal(k.a.indptr, a.indptr) and np.array_equal(k.a.indices, a.indices)
    assert abs(k.a - k.a.T).max() == 0


def test_loader_qfc_one_per_line_gives_diagonal(tmp_path):
    dmx = tmp_path / "t.dmx"
    dmx.write_text("c tiny\np min 3 3\na 1 2 0 1 1\na 2 3 0 1 1\na 3 1 0 1 1\n")
    qfc = tmp_path / "t.qfc"
    qfc.write_text("3\n1\n1\n1\n2.5\n3.5\n4.5\n")
    k = load_kkt_system(str(dmx), str(qfc))
    a, _, _ = kkt_ref.load_kkt_system(str(dmx), str(qfc))
    assert k.a.nnz == 15 and (k.a != a).nnz == 0
    assert np.allclose(k.a.diagonal()[:3], [2.5, 3.5, 4.5])
    # qfcgen 3-line format: D empty
    qfc.write_text("3\n1.0 2.0 3.0 \n4.0 5.0 6.0 \n")
    assert load_kkt_system(str(dmx), str(qfc)).a.nnz == 12


@pytest.mark.parametrize("dmx_text,qfc_text,msg", [
    ("p min 2 1\na 0 1\n", "1\n", "Format error: Invalid node index '0'. DIMACS format requires "
                                 "1-based positive integers."),
    ("c no problem line\na 1 2\n", "1\n",
     "Format error: The 'p min' problem line was not found or was malformed."),
    ("p max 2 1\n", "1\n", "Format error: The 'p min' problem line was not found or was malformed."),
    ("p min 2 1\na 1 x\n", "1\n", "Parse error: Failed to parse integer from 'x'"),
    ("p min 2 1\na 1 2\n", "2\n", "Dimension mismatch: qfc file specifies 2 arcs, but dmx file has 1."),
    ("p min 2 1\na 1 2\n", "", "Format error: Unexpected end of file while reading data."),
    ("p min 2 1\na 1 2\n", "m\n", "Parse error: Failed to parse integer from 'm'"),
    ("p min 2 1\na 1 2\n", "1\n1\nabc\n", "Parse error: Failed to parse float from 'abc'"),
])
def test_loader_errors(tmp_path, dmx_text, qfc_text, msg):
    (tmp_path / "e.dmx").write_text(dmx_text)
    (tmp_path / "e.qfc").write_text(qfc_text)
    with pytest.raises(DataLoaderError) as e:
        load_kkt_system(str(tmp_path / "e.dmx"), str(tmp_path / "e.qfc"))
    assert str(e.value) == msg


def test_loader_missing_file():
    with pytest.raises(DataLoaderError, match=r"^I/O error: No such file or directory \(os error 2\)$"):
        load_kkt_system("/nonexistent.dmx", "/nonexistent.qfc")


def _tridiags(rng):
    yield np.array([2.0]), np.array([])
    yield np.zeros(6), rng.uniform(0.5, 2.0, 5)                # KKT-like: zero diagonal, even k
    yield rng.standard_normal(40), rng.uniform(0.1, 3.0, 39)
    yield -np.abs(rng.standard_normal(200)) * 10, rng.uniform(0.1, 3.0, 199)
    yield np.zeros(500), rng.uniform(0.1, 1.0, 499)           # KKT-like at the headline k
    yield rng.standard_normal(7), rng.uniform(0.1, 3.0, 6)     # smaller after larger (exp reuses its buffers)


@pytest.mark.parametrize("name", ["inv", "exp", "sq"])
def test_builtin_ftk_matches_lapack(name):
    rng = np.random.default_rng(3)
    for al, be in _tridiags(rng):
        y = tpl_amd.ftk.BUILTINS[name](al, be)
        yr = ftk_ref.SOLVERS[name](al, be)
        scale = np.linalg.norm(yr)
        assert np.linalg.norm(y - yr) <= 1e-11 * max(scale, 1e-300), (name, len(al))


def test_error_display_strings():
    """The six message tests of src/error.rs:69-129."""
    assert str(LanczosError.breakdown(42)) == ("Lanczos iteration breakdown at step 42: Beta "
                                               "coefficient is zero. The Krylov subspace is invariant.")
    assert str(LanczosError.dimension_mismatch(100, 99)) == (
        "Dimension mismatch: operator has 100 columns but vector has 99 rows.")
    assert str(LanczosError.parameter_mismatch("y_k", 10, 9)) == (
        "Parameter mismatch: `y_k` expects size 10, but got 9.")
    assert str(LanczosError.input_error("The initial vector `b` must not be a zero vector.")) == (
        "Invalid input parameter: The initial vector `b` must not be a zero vector.")
    assert str(LanczosError.evd_error("NoConvergence")) == (
        "A numerical error occurred during the eigendecomposition of T_k: NoConvergence")
    assert str(LanczosError.solver_error("Custom solver failed")) == (
        "The user-provided f(T_k) solver failed: Custom solver failed")
    assert LanczosError.parameter_mismatch("y_k", 1, 2) == LanczosError.parameter_mismatch("y_k", 1, 2)


@pytest.mark.parametrize("arcs", [5000, 50000, 500000])
def test_netgen_fixture_regenerates_from_reference(arcs):
    """tests/golden/make_fixtures.py: every committed netgen fixture (5k, 50k and the
    500k headline instance) is byte-identical to the reference's own netgen (compiled
    from /root/reference sources into oracle/_ref) run on the recorded parameters."""
    if not os.path.exists("/root/reference/data/netgen/src"):
        pytest.skip("reference checkout not present (GPU box)")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_fixtures
    import hashlib
    assert hashlib.md5(make_fixtures.generate(arcs)).hexdigest() == KKT_MD5[arcs]


def test_harness_rng_matches_oracle_restatement():
    """The harness's StdRng (product utility) and the oracle's restatement agree."""
    from tpl_amd.utils.rng import std_rng_f64
    from oracle.rng import std_rng_vector
    assert np.array_equal(std_rng_f64(10000, 42), std_rng_vector(10000, 42))
    assert np.array_equal(std_rng_f64(7, 3), std_rng_vector(7, 3))


def test_operator_input_is_copied_and_canonicalised():
    """HipCsrOp's host conversion (no GPU needed) never touches the caller's matrix and
    sums duplicates like faer's try_new_from_triplets; explicit zeros stay."""
    from tpl_amd.operator import _as_csr_arrays
    indptr = np.array([0, 3, 4, 5])
    indices = np.array([2, 0, 2, 1, 0], dtype=np.int32)   # unsorted, (0, 2) twice
    data = np.array([1.0, 5.0, 2.0, 0.0, 3.0])
    m = sp.csr_matrix((data, indices, indptr), shape=(3, 3))
    before = (m.indices.copy(), m.data.copy())
    n, rp, ci, v = _as_csr_arrays(m)
    assert np.array_equal(m.indices, before[0]) and np.array_equal(m.data, before[1])
    assert n == 3 and list(rp) == [0, 2, 3, 4]
    assert list(ci) == [0, 2, 1, 0] and list(v) == [5.0, 3.0, 0.0, 3.0]


def test_rust_shim_binds_the_header():
    """integration/rust/hip.rs (the reference crate's src/hip.rs; no Rust toolchain here)
    declares only symbols include/tpl.h exports, each with the header's parameter count."""
    src = open(os.path.join(ROOT, "integration", "rust", "hip.rs")).read()
    block = src[src.index('extern "C" {\n    fn tpl_last_error_detail'):]
    block = block[:block.index("\n}\n")]
    rust = {m.group(1): m.group(2) for m in
            re.finditer(r"fn (tpl_[a-z0-9_]+)\((.*?)\)\s*->", block, flags=re.S)}
    hdr = open(os.path.join(ROOT, "include", "tpl.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    assert len(rust) >= 10
    for name, params in rust.items():
        m = re.search(rf"\b{name}\s*\((.*?)\);", hdr, flags=re.S)
        assert m, name
        n_h = 0 if m.group(1).strip() in ("", "void") else m.group(1).count(",") + 1
        n_r = 0 if not params.strip() else params.count(",") + 1
        assert n_h == n_r, (name, n_h, n_r)
