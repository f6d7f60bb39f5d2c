"""Timeline of the pushed-layout launches from a TPL_STAMP build (dev tool). Chunk marks:
[0] start, [1] loads landed (scale known), [2] products staged in LDS, [4] short runs
written, [3] long runs written, [5] end; combiners (pass two): [0], [5]."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd import _lib
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
K = 6
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
op = tpl_amd.HipCsrOp(a)
op.set_push(True)
tpl_amd.lanczos_two_pass(op, b, 50, "inv")
sch = op.schedule()
assert sch["push"], sch["push"]
nch = -(-len(sch["short_rows"]) // sch["chunk_rows"])
ncomb = -(-len(sch["long_rows"]) // 32)  # kCombRows
fn = _lib.lib.tpl_debug_stamps_push
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
def q(x):
    x = x[np.isfinite(x)]
    return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 50, 90, 100])) if len(x) else "-"
for kid, name, comb in [(3, "spmv", 0), (2, "p2", ncomb), (0, "p1", 0)]:
    op.profile_kernel(kid, 20)
    st = np.zeros(K * 65536, dtype=np.uint64)
    fn(st.ctypes.data, 65536)
    G = comb + nch
    m = st[:K * G].reshape(G, K).astype(np.float64)
    m[m == 0] = np.nan
    base = np.nanmin(m[:, 0])
    t = (m - base) / 100.0  # us (100 MHz)
    print(f"== {name}: combiners {comb}, chunks {nch}; us; pct 0/50/90/100")
    for nm, sel, marks in [("comb", slice(0, comb), []), ("chunk", slice(comb, G), [1, 2, 4, 3])]:
        tt = t[sel]
        if len(tt) == 0:
            continue
        print(f"  {nm:5s} start      {q(tt[:,0])}")
        for k in marks:
            print(f"  {nm:5s} mark{k}-start {q(tt[:,k]-tt[:,0])}")
        print(f"  {nm:5s} end        {q(tt[:,5])} | dur {q(tt[:,5]-tt[:,0])}")
