"""Schedule sweep on the 500k instance: per-kernel HIP-event times for several item
schedules (dev tool; prints a table)."""
import os, sys, json, itertools
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd import _lib
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line

arcs = int(os.environ.get("ARCS", "500000"))
write_qfc_3line("/tmp/t.qfc", arcs)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
op = tpl_amd.HipCsrOp(a)
configs = json.loads(os.environ.get("CONFIGS", "[[2048,1024,4096,1024]]"))
for cfg in configs:
    op.set_schedule(*cfg)
    tpl_amd.lanczos_two_pass(op, b, 50, "inv")
    items, G, E = op.schedule()
    kinds = np.bincount(items[:, 3], minlength=3)
    row = {"cfg": cfg, "items": len(items), "kinds": kinds.tolist(), "G": G, "E": E}
    for kid, nm in [(0, "p1_spmv"), (1, "p1_axpy"), (2, "p2_spmv"), (3, "spmv")]:
        us, by = op.profile_kernel(kid, 300)
        row[nm] = round(us, 2)
    print(json.dumps(row), flush=True)
