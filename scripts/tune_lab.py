"""Dev tool: the engine's default locality order vs tpl_op_tune_order on the 500k KKT
(k_p1_spmv + k_p2_spmv isolated averages, solve time)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
for mode in ("default", "tuned", "off"):
    op = tpl_amd.HipCsrOp(a)
    extra = {}
    if mode == "tuned":
        t0 = time.perf_counter()
        g, us = op.tune_order()
        extra = {"groups": g, "tune_s": round(time.perf_counter() - t0, 2)}
    if mode == "off":
        op.set_reorder(0)
    tpl_amd.lanczos_two_pass(op, b, 500, "inv")
    ts = []
    for _ in range(5):
        t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
    row = {"mode": mode, "solve_ms": round(1000 * min(ts), 3), **extra}
    for kid, nm in [(0, "p1_spmv"), (2, "p2_spmv")]:
        row[nm] = round(op.profile_kernel(kid, 300)[0], 2)
    print(json.dumps(row), flush=True)
    op.close()
