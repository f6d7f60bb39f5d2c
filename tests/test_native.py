"""Native drivers (tests/native): the C ABI exercised from C++ and the
engine's host C++ — the untrusted-file loader, the f(T_k) solvers, the SpMV layout
builder — under AddressSanitizer + UndefinedBehaviorSanitizer."""
import lzma
import os
import shutil
import subprocess

import pytest

from conftest import KKT_DIR, ROOT

NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def drivers(tmp_path_factory):
    if shutil.which(os.environ.get("CXX", "g++")) is None:
        pytest.skip("no host C++ compiler")
    subprocess.run(["make", "-s", "-C", NATIVE], check=True, capture_output=True)
    d = tmp_path_factory.mktemp("native")
    dmx = str(d / "5k.dmx")
    with lzma.open(os.path.join(KKT_DIR, "netgen-5000-3.dmx.xz")) as f, open(dmx, "wb") as g:
        g.write(f.read())
    qfc = str(d / "5k.qfc")
    with open(qfc, "w") as f:
        f.write("5000\n1.0 2.0\n3.0 4.0\n")
    return dmx, qfc, str(d)


def _run(args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run(args, capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    assert "OK (0 failures)" in p.stdout
    return p


def test_abi_driver_cpu(drivers):
    dmx, qfc, _ = drivers
    _run([os.path.join(NATIVE, "build", "abi_driver"), dmx, qfc])


def test_host_code_under_asan_ubsan(drivers):
    dmx, qfc, scratch = drivers
    p = _run([os.path.join(NATIVE, "build", "sanitize_driver"), dmx, qfc, scratch])
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


@pytest.mark.gpu
def test_abi_driver_gpu(drivers):
    """Two-pass through a host callback f and through the built-in inv (one device graph):
    bitwise equal; one-pass within 1e-10; error statuses; device footprint."""
    dmx, qfc, _ = drivers
    _run([os.path.join(NATIVE, "build", "abi_driver"), dmx, qfc, "--gpu"])


def test_cpp_api_cpu(drivers):
    """include/tpl.hpp: the reference's error Display tests (src/error.rs:70-127) and the
    StdRng restatement behind its test vectors, no device needed."""
    _run([os.path.join(NATIVE, "build", "cpp_api_test"), "--cpu"])


@pytest.mark.gpu
def test_cpp_api_gpu(drivers):
    """The reference's tests through the C++ host API: tests/correctness.rs (inv / exp / z^2,
    one- and two-pass, diag(1..100), k = 30), src/algorithms/mod.rs's unit tests and its four
    property tests on the 5k KKT instance (TOLERANCE 5e-9), and the solver-closure errors."""
    dmx, qfc, _ = drivers
    _run([os.path.join(NATIVE, "build", "cpp_api_test"), "--gpu", dmx, qfc])


def test_back_substitution_division_is_ieee(tmp_path):
    """k_ftk_inv's back substitution divides with Markstein's correction from a
    precomputed reciprocal (tpl_kernels.hip div_rn); restated on the host with the same
    fused multiply-adds, it gives the IEEE quotient bit for bit on every pair its range
    check lets through (2e7 pairs: wide exponents, near-exact and binade-boundary
    quotients, signed zeros)."""
    cc = os.environ.get("CC", "gcc")
    if shutil.which(cc) is None:
        pytest.skip("no host C compiler")
    exe = str(tmp_path / "div_rn_check")
    subprocess.run([cc, "-O2", "-mfma", "-ffp-contract=off", "-o", exe,
                    os.path.join(NATIVE, "div_rn_check.c"), "-lm"], check=True)
    _run([exe, "20000000"])
