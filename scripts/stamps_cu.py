"""Dev tool (TPL_STAMP variant library): which CUs finish a k_p2_spmv launch last, and
what they hold, on the 500k KKT for several locality-order group counts. Per workgroup
the stamp build records its start / end (s_memrealtime, 100 MHz) and its HW_ID / XCC_ID.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np  # noqa: E402
import tpl_amd  # noqa: E402
from tpl_amd import _lib  # noqa: E402
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line  # noqa: E402

K = 7
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
fn = _lib.lib.tpl_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
for G in [int(x) for x in os.environ.get("GROUPS", "16,15").split(",")]:
    op = tpl_amd.HipCsrOp(a)
    op.tune_order([G], iters=5)
    tpl_amd.lanczos_two_pass(op, b, 50, "inv")
    us = op.profile_kernel(2, 50)[0]
    sch = op.schedule()
    chunk_blocks = 8 * ((sch["G2"] + 7) // 8) * (sch["E"] // 512)
    st = np.zeros(K * 65536, dtype=np.uint64)
    fn(st.ctypes.data, 65536)
    m = st.reshape(-1, K)
    Gt = int(np.count_nonzero(m[:, 0]))
    m = m[:Gt]
    nsb = Gt - chunk_blocks
    t0 = m[:, 0].astype(np.int64)
    base = t0.min()
    start = (t0 - base) / 100.0
    end = (m[:, 5].astype(np.int64) - base) / 100.0
    hw = (m[:, 6] & 0xFFFFFFFF).astype(np.int64)
    xcc = (m[:, 6] >> np.uint64(32)).astype(np.int64)
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    live = end > 0
    print(f"== groups {G}: k_p2_spmv {us:.2f} us isolated; grid {Gt} (bins {nsb}); "
          f"last end {end[live].max():.2f} us, median end {np.median(end[live]):.2f}")
    ukeys = np.unique(key)
    fin = np.array([end[(key == k) & live].max() for k in ukeys])
    busy = np.array([np.sum((end - start)[(key == k) & live]) for k in ukeys])
    print(f"  CUs {len(ukeys)}; CU finish pct 50/90/99/100: "
          + " ".join(f"{v:.2f}" for v in np.percentile(fin, [50, 90, 99, 100])))
    for k in ukeys[np.argsort(-fin)][:4]:
        sel = np.nonzero((key == k))[0]
        desc = ", ".join(f"{'bin' if i < nsb else 'chunk'} {i} [{start[i]:.2f}-{end[i]:.2f}]"
                         for i in sel[np.argsort(start[sel])])
        print(f"  CU xcc{k // 256} se{(k // 32) % 8} cu{k % 16}: {desc}")
    bins = np.arange(Gt) < nsb
    print(f"  bins end pct 50/90/100: " + " ".join(f"{v:.2f}" for v in np.percentile(end[bins & live], [50, 90, 100]))
          + f" | chunks end pct 50/90/100: " + " ".join(f"{v:.2f}" for v in np.percentile(end[~bins & live], [50, 90, 100])))
    op.close()
