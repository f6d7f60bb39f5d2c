"""Dev tool: k_p1/k_p2_spmv and solve time on the 500k KKT (engine order) per slice count."""
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
for S in [int(x) for x in os.environ.get("SLICES", "8,4,2").split(",")]:
    op = tpl_amd.HipCsrOp(a)
    op.set_slices(S)
    tpl_amd.lanczos_two_pass(op, b, 500, "inv")
    ts = []
    for _ in range(5):
        t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
    row = {"slices": S, "solve_ms": round(1000 * min(ts), 3)}
    for kid, nm in [(0, "p1_spmv"), (2, "p2_spmv")]:
        row[nm] = round(op.profile_kernel(kid, 300)[0], 2)
    print(json.dumps(row), flush=True)
    op.close()
