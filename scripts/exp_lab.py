"""Dev tool (GPU): phase timeline of the device exp kernel (k_ftk_exp) on configs[1]'s T_k
(50k arcs, k = 200) and on wider spectra. Run with TPL_LIB_PATH pointing at a TPL_STAMP
variant (scripts/build_variants.sh stamp="-DTPL_STAMP=1"): marks 0..5 = start, loads and
Gershgorin bounds done, Sturm multisection done, term count found, Clenshaw done, end
(s_memrealtime, 100 MHz)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import tpl_amd  # noqa: E402
from tpl_amd import _lib  # noqa: E402
import oracle  # noqa: E402
from conftest import harness_b, load_kkt  # noqa: E402

a = load_kkt(50000, "/tmp").a
al, be, s, bn, _ = oracle.Operator(a).pass_one(harness_b(a), 200)
cases = {"cfg1_k200": (al, be)}
lam = -1000.0 + (999.9 / 9999) * np.arange(10000)
d = sp.diags(lam).tocsr()
from oracle.rng import std_rng_vector  # noqa: E402
al2, be2, *_ = oracle.Operator(d).pass_one(std_rng_vector(10000), 200)
cases["diag_ill_k200"] = (al2, be2)
op = tpl_amd.HipCsrOp(sp.diags(np.arange(1.0, 65.0)).tocsr())
buf = (ctypes.c_ulonglong * 9)()  # kMarks (tpl_lab.h)
nterm = ctypes.c_int()
for name, (x, y) in cases.items():
    for rep in range(3):
        yv, on = op.ftk_device("exp", x, y)
    _lib.lib.tpl_debug_stamps(buf, 1)
    _lib.lib.tpl_debug_exp_terms(ctypes.byref(nterm))
    m = [buf[i] for i in range(6)]
    ph = [round((m[i + 1] - m[i]) * 0.01, 2) for i in range(5)]
    print(f"{name}: on_device={on} terms={nterm.value} phases_us(load+bounds, sturm, "
          f"terms, clenshaw, tail)={ph} total_us={round((m[5] - m[0]) * 0.01, 2)}", flush=True)
