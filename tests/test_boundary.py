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


# ---- the Rust shim (integration/rust/hip.rs; no Rust toolchain in this image) ----------
HIP_RS = os.path.join(ROOT, "integration", "rust", "hip.rs")
REF_SRC = "/root/reference/src"

# C type (base name) -> the Rust type an `extern "C"` binding must use for it
_C_TO_RUST = {"double": "f64", "int": "c_int", "int32_t": "i32", "int64_t": "i64",
              "uint64_t": "u64", "uint8_t": "u8", "size_t": "usize", "char": "c_char",
              "void": "c_void", "tpl_status": "c_int", "tpl_ctx_t": "*mut TplCtx",
              "tpl_op_t": "*mut TplOp", "tpl_dist_t": "*mut TplDist", "tpl_ftk_fn": "FtkFn",
              # the step callback is optional (NULL = none): a nullable fn pointer
              "tpl_step_cb": "Option<StepCb>", "tpl_error_detail": "TplErrorDetail"}


def _c_header():
    return re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "tpl.h")).read(),
                  flags=re.S)


def _split_top(s, sep=","):
    """Split at `sep` outside (), <>, [] (Rust generics and C parameter lists)."""
    out, depth, cur = [], 0, ""
    for i, ch in enumerate(s):
        if ch in "(<[":
            depth += 1
        elif ch in ")]" or (ch == ">" and not (i > 0 and s[i - 1] == "-")):
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [p.strip() for p in out]


def _c_type_to_rust(ctype):
    """'const double*' -> '*const f64', 'tpl_ctx_t*' -> '*mut *mut TplCtx', ..."""
    t = ctype.replace("*", " * ").split()
    stars = t.count("*")
    const = "const" in t
    base = [w for w in t if w not in ("*", "const")]
    assert len(base) == 1, ctype
    rust = _C_TO_RUST[base[0]]
    for lvl in range(stars):
        rust = ("*const " if const and lvl == 0 else "*mut ") + rust
    return rust


def _c_params(plist, named=True):
    if plist.strip() in ("", "void"):
        return []
    out = []
    for p in _split_top(plist):
        p = p.replace("*", "* ")
        if named:
            p = re.sub(r"\b[A-Za-z_][A-Za-z0-9_]*\s*$", "", p)  # drop the parameter name
        out.append(_c_type_to_rust(p))
    return out


def _rust_norm(t):
    return re.sub(r"\s+", "", t).replace("*const", "*const ").replace("*mut", "*mut ")


def _extern_block():
    src = open(HIP_RS).read()
    block = src[src.index('extern "C" {'):]
    return src, block[:block.index("\n}\n")]


def test_rust_shim_extern_types_match_header():
    """Every `extern "C"` item of hip.rs is a symbol of include/tpl.h whose parameter and
    return TYPES are the header's, parameter by parameter (C -> Rust: const T* ->
    *const T, T* -> *mut T, handles -> *mut opaque, size_t -> usize, tpl_status -> c_int,
    the nullable step callback -> Option<fn>)."""
    _, block = _extern_block()
    hdr = _c_header()
    items = list(re.finditer(r"fn (tpl_[a-z0-9_]+)\((.*?)\)\s*->\s*([^;]+);", block, flags=re.S))
    assert len(items) >= 12
    for m in items:
        name, params, ret = m.group(1), m.group(2), m.group(3)
        h = re.search(rf"\n\s*([A-Za-z_][A-Za-z0-9_ ]*?\**)\s*\b{name}\s*\((.*?)\);", hdr, flags=re.S)
        assert h, name
        want = _c_params(h.group(2))
        got = [_rust_norm(p.split(":", 1)[1]) for p in _split_top(params)]
        assert got == [_rust_norm(w) for w in want], (name, got, want)
        assert _rust_norm(ret) == _rust_norm(_c_type_to_rust(h.group(1).strip())), name
    # the ones VERDICT r04 found missing
    names = {m.group(1) for m in items}
    assert {"tpl_lanczos_standard", "tpl_copy_to_host", "tpl_lanczos_pass_two"} <= names
    # the multi-GPU operators (HipDist, HipCsrOp::partitioned)
    assert {"tpl_dist_unique_id", "tpl_dist_create", "tpl_dist_destroy",
            "tpl_dist_op_create_replicated", "tpl_dist_op_create_halo",
            "tpl_op_local_rows", "tpl_op_nrows"} <= names
    src, _ = _extern_block()
    for item in ("pub struct HipDist", "pub fn partitioned", "pub fn local_rows",
                 "pub enum Partition", "pub fn unique_id"):
        assert item in src, item


def test_rust_shim_callback_and_struct_types_match_header():
    """FtkFn / StepCb carry tpl_ftk_fn / tpl_step_cb's parameter types in order, and the
    #[repr(C)] TplErrorDetail has tpl_error_detail's fields, names and types in order."""
    src, _ = _extern_block()
    hdr = _c_header()
    for rust_name, c_name in (("FtkFn", "tpl_ftk_fn"), ("StepCb", "tpl_step_cb")):
        r = re.search(rf'type {rust_name} = unsafe extern "C" fn\((.*?)\)\s*->\s*([^;]+);',
                      src, flags=re.S)
        c = re.search(rf"typedef\s+(\w+)\s*\(\*{c_name}\)\((.*?)\);", hdr, flags=re.S)
        assert r and c, rust_name
        assert [_rust_norm(p) for p in _split_top(r.group(1))] == \
            [_rust_norm(p) for p in _c_params(c.group(2))], rust_name
        assert _rust_norm(r.group(2)) == _c_type_to_rust(c.group(1))
    r = re.search(r"#\[repr\(C\)\]\s*struct TplErrorDetail \{(.*?)\}", src, flags=re.S)
    c = re.search(r"typedef struct tpl_error_detail \{(.*?)\}", hdr, flags=re.S)
    rust_fields = [tuple(_rust_norm(x) for x in f.split(":")) for f in _split_top(r.group(1))]
    c_fields = []
    for decl in c.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        first, *rest = [d.strip() for d in decl.split(",")]
        m = re.match(r"(.*?)\b([A-Za-z_]\w*)$", first.replace("*", "* "))
        ctype = m.group(1).strip()
        for nm in [m.group(2)] + rest:
            c_fields.append((nm, _rust_norm(_c_type_to_rust(ctype))))
    assert rust_fields == c_fields


def _rust_fns(src):
    """name -> (generics, [(param, type)], return type, where clause) of every `pub fn`."""
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"\bpub fn (\w+)", src):
        i = m.end()
        gen = ""
        if src[i] == "<":
            d, j = 0, i
            while True:
                d += {"<": 1, ">": -1}.get(src[j], 0)
                j += 1
                if d == 0:
                    break
            gen, i = src[i + 1:j - 1], j
        assert src[i] == "(", m.group(1)
        d, j = 0, i
        while True:
            d += {"(": 1, ")": -1}.get(src[j], 0)
            j += 1
            if d == 0:
                break
        params = [(re.sub(r"^mut\s+", "", p.split(":", 1)[0].strip()), p.split(":", 1)[1])
                  if ":" in p else (p, p)  # a `&self` receiver
                  for p in _split_top(src[i + 1:j - 1])]
        tail = src[j:src.index("{", j)]
        rm = re.search(r"->\s*(.*?)\s*(?:\bwhere\b|$)", tail, flags=re.S)
        ret = rm.group(1) if rm else "()"
        where = tail.split("where", 1)[1] if "where" in tail else ""
        out[m.group(1)] = (gen, params, ret, where)
    return out


def _sig_norm(t):
    """The reference's generic scalar and operator read as the shim's concrete ones."""
    t = re.sub(r"\s+", "", t)
    t = re.sub(r"<TasComplexField>::Real|T::Real", "f64", t)
    t = re.sub(r"\bT\b", "f64", t)
    t = re.sub(r"^&(implLinOp<f64>|implHipOperand|O)$", "&OPERAND", t)
    return t


def _closure_bound(gen, where):
    m = re.search(r"F:\s*(FnMut\(.*?\)\s*->\s*Result<[^{]*?anyhow::Error>)", gen + "," + where,
                  flags=re.S)
    return _sig_norm(m.group(1)) if m else None


def test_rust_shim_signatures_match_reference():
    """every public function of src/solvers.rs and
    src/algorithms/{lanczos,lanczos_two_pass}.rs has a same-name counterpart in hip.rs with
    the same parameter names in the same order (`stack: &mut MemStack` included), the same
    parameter, closure-bound and return types once the reference's generic scalar T (and
    T::Real) is read as f64 and its `LinOp<T>` operator as the shim's HipOperand; the
    output structs and the callback type are the crate's own (imported, not redefined);
    and HipCsrOp implements faer's LinOp<f64>."""
    if not os.path.isdir(REF_SRC):
        pytest.skip("reference checkout not present (GPU box)")
    shim_src = open(HIP_RS).read()
    shim = _rust_fns(shim_src)
    ref = {}
    for rel in ("solvers.rs", "algorithms/lanczos.rs", "algorithms/lanczos_two_pass.rs"):
        ref.update(_rust_fns(open(os.path.join(REF_SRC, rel)).read()))
    assert set(ref) == {"lanczos", "lanczos_two_pass", "lanczos_standard", "lanczos_pass_one",
                        "lanczos_pass_two", "lanczos_pass_two_with_basis"}
    for name, (gen, params, ret, where) in ref.items():
        assert name in shim, name
        sgen, sparams, sret, swhere = shim[name]
        assert [p for p, _ in sparams] == [p for p, _ in params], name
        assert [_sig_norm(t) for _, t in sparams] == [_sig_norm(t) for _, t in params], name
        assert _sig_norm(sret) == _sig_norm(ret), name
        assert _closure_bound(sgen, swhere) == _closure_bound(gen, where), name
    for ty in ("LanczosCallback", "LanczosDecomposition", "LanczosOutput",
               "LanczosPassTwoOutput", "TridiagonalSystemView"):
        assert re.search(rf"use crate::algorithms::\{{[^}}]*\b{ty}\b", shim_src), ty
        assert not re.search(rf"\b(struct|type) {ty}\b", shim_src), ty
    assert re.search(r"impl LinOp<f64> for HipCsrOp", shim_src)
    for m in ("apply_scratch", "nrows", "ncols", "apply", "conj_apply"):
        assert re.search(rf"impl LinOp<f64> for HipCsrOp \{{.*?\bfn {m}\(", shim_src, flags=re.S), m
    # the reference's own call sites pass `&a.as_ref()` (a SparseColMatRef)
    assert re.search(r"impl<'a> HipOperand for SparseColMatRef<'a, usize, f64>", shim_src)
