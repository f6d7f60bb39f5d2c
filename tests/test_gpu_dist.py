"""GPU tests of the row-partitioned operator.

* one rank over RCCL, row blocks: the partitioned path reproduces the single-GPU
  result bit for bit (same layout, the rank total of alpha/beta partials is exact);
  replicated long rows: within 1e-10;
* two and three ranks sharing this box's GPU, exchanging through the host transport
  (RCCL refuses two ranks on one device), every partition: identical coefficients on
  every rank, deterministic, x within 1e-10 of the single-GPU solve, SpMV blocks;
* halo-exchange row blocks on a banded matrix without the KKT structure: bitwise the
  plain row blocks' result and the restated partitioned order, moving only the halo.
The ranks run as child processes (tests/dist_worker.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "two-pass-lanczos_amd"))

from conftest import harness_b, load_kkt  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp, world, transport, mode="auto", arcs=5000, k=50, extra_env=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                                       tmp, transport, str(arcs), str(k), mode], env=env))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * world, rcs
    return [np.load(os.path.join(tmp, f"rank{r}.npz")) for r in range(world)]


def _single(kkt_tmp, arcs=5000, k=50):
    import tpl_amd
    a = load_kkt(arcs, kkt_tmp).a
    b = harness_b(a)
    op = tpl_amd.HipCsrOp(a)
    op.set_reorder(False)  # partitioned operators keep the caller's row order
    return (a, tpl_amd.lanczos_two_pass(op, b, k, "inv"),
            tpl_amd.algorithms.lanczos_pass_one(op, b, k), tpl_amd.lanczos(op, b, k, "inv"))


def _assemble(rs, key, n):
    out = np.full(n, np.nan)
    for r in rs:
        out[r["rows"]] = r[key]
    return out


@pytest.mark.parametrize("mode", ["rows", "halo"])
def test_one_rank_rccl_rows_bitwise(kkt_tmp, tmp_path, mode):
    a, x, dec, xs = _single(kkt_tmp)  # same layout as the partition's
    r = _run_ranks(str(tmp_path), 1, "rccl", mode=mode)[0]
    assert str(r["mode"]) == mode
    _check_exchange_profile([r])
    assert np.array_equal(r["x1"], x)
    assert np.array_equal(r["al"], dec.alphas) and np.array_equal(r["be"], dec.betas)
    assert np.array_equal(r["xs"], xs)


def _check_exchange_profile(rs):
    # tpl_profile_kernel's exchange ids: positive times, the bytes one rank receives
    # (pass one: the alpha and beta totals + one vector part per rank; pass two: the part)
    R = len(rs)
    for r in rs:
        assert np.array_equal(r["x3"], r["x1"])
        assert all(t > 0 for t in r["ex_us"])
        b1, b2 = r["ex_bytes"]
        if str(r["mode"]) == "replicated":
            # pass two: one segment of n_long partials + 1 per rank; pass one: the n_long
            # partials + the rank's short-chunk alpha partials (segments as long as the
            # most chunks of any rank, 512 short rows each), then the norm totals
            nl = len(r["s_long"])
            nch = max(-(-(len(q["rows"]) - nl) // 512) for q in rs)
            assert b2 == 8 * R * (nl + 1) and b1 == 8 * R * (nl + nch + 1)
            # tpl_op_flags bit 7: the norm partials travel gathered and pass one's SpMV
            # reduces them (R <= kPbRanks, the 5k KKT's long-row partials fit one block)
            assert int(r["flags"]) & 128
        elif str(r["mode"]) == "halo":  # the halo slots (none with one rank)
            assert b1 - b2 == 16 * R and b2 % (8 * R) == 0 and (b2 > 0) == (R > 1)
        else:
            assert b1 - b2 == 16 * R and b2 > 0


def test_one_rank_rccl_replicated(kkt_tmp, tmp_path):
    a, x, dec, xs = _single(kkt_tmp)
    r = _run_ranks(str(tmp_path), 1, "rccl", mode="replicated")[0]
    assert str(r["mode"]) == "replicated"
    _check_exchange_profile([r])
    xr = _assemble([r], "x1", a.shape[0])
    assert np.linalg.norm(xr - x) <= 1e-10 * np.linalg.norm(x)
    _check_partition_order(a, [r], "replicated", 50)


@pytest.mark.parametrize("mode", ["replicated", "rows"])
def test_one_rank_rccl_capture_refused_falls_back_eager(kkt_tmp, tmp_path, mode):
    """A transport whose exchanges refuse stream capture (forced by the test hook
    TPL_TEST_REFUSE_CAPTURE): the operator switches to eager launches (run_graph's fallback,
    tpl_op_flags bit 1) and produces the same bits as the captured graphs."""
    ref = _run_ranks(str(tmp_path / "g"), 1, "rccl", mode=mode)[0]
    r = _run_ranks(str(tmp_path / "e"), 1, "rccl", mode=mode,
                   extra_env={"TPL_TEST_REFUSE_CAPTURE": "1"})[0]
    assert not int(ref["flags"]) & 2 and int(r["flags"]) & 2
    for key in ("x1", "x2", "x3", "xs", "al", "be", "y"):
        assert np.array_equal(r[key], ref[key]), key


def _check_partition_order(a, rs, mode, k):
    """alphas, betas, ||b|| and x bit for bit against the partitioned order restated on
    the CPU (tests/partition_oracle.py)."""
    from partition_oracle import PartitionOracle
    import tpl_amd
    b = harness_b(a)
    # the host-only plan (tpl_plan_create, what tests/golden/make_parity.py restates the
    # bench's partitioned digests from) is the live rank's rows and layout
    for r, rec in enumerate(rs):
        plan = tpl_amd.HostPlan(a, mode=mode, nranks=len(rs), rank=r)
        ps = plan.schedule()
        assert np.array_equal(plan.local_rows, rec["rows"])
        assert np.array_equal(ps["short_rows"], rec["s_short"])
        assert np.array_equal(ps["long_rows"], rec["s_long"])
        assert (ps["G2"], ps["E"], ps["slices"]) == (int(rec["s_G2"]), int(rec["s_E"]),
                                                     int(rec["s_slices"]))
        plan.close()
    po = PartitionOracle(a, rs, "rows" if mode == "halo" else mode)  # halo: rows' order
    al, be, s, bn = po.pass_one(b, k)
    assert int(rs[0]["steps"]) == s and float(rs[0]["bn"]) == bn
    assert np.array_equal(rs[0]["al"], al) and np.array_equal(rs[0]["be"], be)
    xo = po.pass_two(b, al, be, s, bn, tpl_amd.ftk.INV(al, be) * bn)
    assert np.array_equal(_assemble(rs, "x1", a.shape[0]), xo)


@pytest.mark.parametrize("world,mode", [(2, "rows"), (3, "rows"), (2, "replicated"),
                                        (3, "replicated"), (2, "halo"), (3, "halo")])
def test_ranks_share_gpu_host_transport(kkt_tmp, tmp_path, world, mode):
    a, x, dec, xs = _single(kkt_tmp)
    rs = _run_ranks(str(tmp_path), world, "host", mode=mode)
    assert all(str(r["mode"]) == mode for r in rs)
    for r in rs[1:]:  # every rank holds the same coefficients, bit for bit
        assert np.array_equal(r["al"], rs[0]["al"]) and np.array_equal(r["be"], rs[0]["be"])
    assert int(rs[0]["steps"]) == dec.steps_taken
    np.testing.assert_allclose(rs[0]["al"], dec.alphas, rtol=0, atol=1e-12)
    np.testing.assert_allclose(rs[0]["be"], dec.betas, rtol=1e-12)
    n = a.shape[0]
    xd = _assemble(rs, "x1", n)
    assert np.array_equal(xd, _assemble(rs, "x2", n))  # deterministic
    _check_exchange_profile(rs)
    assert np.linalg.norm(xd - x) <= 1e-10 * np.linalg.norm(x)
    xsd = _assemble(rs, "xs", n)
    assert np.linalg.norm(xsd - xs) <= 1e-10 * np.linalg.norm(xs)
    if mode == "replicated":  # the replicated (long) rows hold identical bits on every rank
        for r in rs[1:]:
            common, i0, i1 = np.intersect1d(rs[0]["rows"], r["rows"], return_indices=True)
            assert len(common) > 0
            assert np.array_equal(rs[0]["x1"][i0], r["x1"][i1])
    _check_partition_order(a, rs, mode, 50)
    # SpMV blocks: +-1 values, exact products
    y = _assemble(rs, "y", n)
    yr = a @ np.cos(np.arange(a.shape[0]))
    np.testing.assert_allclose(y, yr, rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("world", [2, 3])
def test_halo_banded_host_transport(tmp_path, world):
    """tpl_dist_op_create_halo on a matrix without the KKT structure (tests/conftest.py
    banded_hub: band + long hub rows, general values): the same bits as the plain row
    blocks and as the restated partitioned order, every rank receiving only the halo
    (8 H bytes per rank and SpMV, H = dist.halo_width), and "auto" picks it."""
    from conftest import banded_hub
    from tpl_amd.dist import halo_width
    env = {"TPL_TEST_MATRIX": "banded"}
    a = banded_hub()
    rows = _run_ranks(str(tmp_path / "rows"), world, "host", mode="rows", extra_env=env)
    halo = _run_ranks(str(tmp_path / "halo"), world, "host", mode="auto", extra_env=env)
    assert all(str(r["mode"]) == "halo" for r in halo)
    for rr, rh in zip(rows, halo):
        for key in ("rows", "x1", "x2", "x3", "xs", "al", "be", "y"):
            assert np.array_equal(rr[key], rh[key]), key
    H = halo_width(a, halo[0]["starts"])
    assert 0 < H < a.shape[0] // (2 * world)
    for r in halo:
        b1, b2 = r["ex_bytes"]
        assert b2 == 8 * world * H and b1 == 8 * world * (H + 2)
    for r in rows:
        assert r["ex_bytes"][1] > 8 * world * a.shape[0] // world - 1
    _check_partition_order(a, halo, "halo", 50)
    y = _assemble(halo, "y", a.shape[0])
    yr = a @ np.cos(np.arange(a.shape[0]))
    np.testing.assert_allclose(y, yr, rtol=1e-12, atol=1e-12)


def test_halo_without_halo_host_transport(tmp_path):
    """Three independent blocks split at their boundaries (TPL_TEST_STARTS): the halo is
    empty, so no rank packs or exchanges a vector part (pass two moves 0 bytes per step,
    pass one only the two totals) — and the bits are still the plain row blocks' (which
    all-gather every block) and the restated partitioned order's."""
    from conftest import block_diag_spd
    env = {"TPL_TEST_MATRIX": "blockdiag", "TPL_TEST_STARTS": "0,1500,3000,4500"}
    a = block_diag_spd()
    rows = _run_ranks(str(tmp_path / "rows"), 3, "host", mode="rows", extra_env=env)
    halo = _run_ranks(str(tmp_path / "halo"), 3, "host", mode="halo", extra_env=env)
    for rr, rh in zip(rows, halo):
        assert str(rh["mode"]) == "halo"
        assert np.array_equal(rh["starts"], [0, 1500, 3000, 4500])
        for key in ("rows", "x1", "x2", "x3", "xs", "al", "be", "y"):
            assert np.array_equal(rr[key], rh[key]), key
        assert list(rh["ex_bytes"]) == [8 * 3 * 2, 0]
    from partition_oracle import PartitionOracle
    import tpl_amd
    po = PartitionOracle(a, halo, "rows")
    b = harness_b(a)
    al, be, s, bn = po.pass_one(b, 50)
    assert np.array_equal(halo[0]["al"], al) and np.array_equal(halo[0]["be"], be)
    xo = po.pass_two(b, al, be, s, bn, tpl_amd.ftk.INV(al, be) * bn)
    assert np.array_equal(_assemble(halo, "x1", a.shape[0]), xo)


def test_halo_create_rejects_bad_input():
    """tpl_dist_op_create_halo validates before touching the device: a non-increasing or
    short split, fewer rows than ranks and unsorted columns are refused with
    TPL_ERR_INVALID_ARGUMENT and no operator (rank 0 of a two-rank host transport whose
    exchange is never called)."""
    from ctypes import POINTER, byref, c_double, c_int32, c_int64, c_void_p

    import scipy.sparse as sp
    from tpl_amd import _lib

    cb = _lib.ALLGATHER_FN(lambda *args: 1)
    d = c_void_p()
    assert _lib.tpl_dist_create_host(0, 0, 2, cb, None, byref(d)) == _lib.TPL_OK
    try:
        a = sp.identity(6, format="csr") * 2.0
        rp = np.ascontiguousarray(a.indptr, dtype=np.int64)
        ci = np.ascontiguousarray(a.indices, dtype=np.int32)
        v = np.ascontiguousarray(a.data, dtype=np.float64)

        def create(n, starts, rp=rp, ci=ci):
            h = c_void_p()
            st = None if starts is None else np.ascontiguousarray(starts, dtype=np.int64)
            s = _lib.tpl_dist_op_create_halo(
                d.value, n, None if st is None else st.ctypes.data_as(POINTER(c_int64)),
                rp.ctypes.data_as(POINTER(c_int64)), ci.ctypes.data_as(POINTER(c_int32)),
                v.ctypes.data_as(POINTER(c_double)), byref(h))
            if s == _lib.TPL_OK:
                _lib.tpl_op_destroy(h.value)
            return s, h.value

        assert create(6, [0, 4, 3]) == (_lib.TPL_ERR_INVALID_ARGUMENT, None)  # unordered
        assert create(6, [0, 3, 5]) == (_lib.TPL_ERR_INVALID_ARGUMENT, None)  # short
        assert create(1, None, rp=rp[:2]) == (_lib.TPL_ERR_INVALID_ARGUMENT, None)  # 1 row, 2 ranks
        bad = ci.copy()
        bad[0] = 7  # column out of range
        assert create(6, None, ci=bad)[0] == _lib.TPL_ERR_INVALID_ARGUMENT
        assert create(6, [0, 3, 6])[0] == _lib.TPL_OK
    finally:
        _lib.tpl_dist_destroy(d.value)
