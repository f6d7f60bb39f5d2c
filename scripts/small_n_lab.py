"""Dev tool (GPU): solve time, pass-one step and isolated kernel times per element-wise
block size (TPL_ELEM_ROWS, the lab knob of tpl_runtime.cpp rebuild_schedule; read only by a
-DTPL_LAB=1 build, TPL_LIB_PATH pointing at it) at the 50k
(k = 200, f = exp: configs[1]) and 500k (k = 500, f = inv: the headline) instances.
ELEMS (comma list, default 512,1024,2048), ARCS (default 50000,500000), REPS."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tpl_amd  # noqa: E402
from tpl_amd import _lib  # noqa: E402
from tpl_amd.error import check  # noqa: E402
from bench import load_workload, PINNED_ORDER_GROUPS  # noqa: E402

reps = int(os.environ.get("REPS", "20"))
for arcs in [int(a) for a in os.environ.get("ARCS", "50000,500000").split(",")]:
    kkt, _ = load_workload(arcs)
    a = kkt.a
    n = a.shape[0]
    b = torch.from_numpy(a @ np.full(n, 1.0 / np.sqrt(n))).cuda()
    x = torch.empty_like(b)
    k, f = (200, _lib.FTK_EXP_PTR) if arcs == 50000 else (500, _lib.FTK_INV_PTR)
    for e in os.environ.get("ELEMS", "512,1024,2048").split(","):
        os.environ["TPL_ELEM_ROWS"] = e
        op = tpl_amd.HipCsrOp(a)
        if arcs in PINNED_ORDER_GROUPS:
            op.set_order_groups(PINNED_ORDER_GROUPS[arcs])
        sch = op.schedule()

        def solve():
            check(_lib.tpl_lanczos_two_pass(op.handle, b.data_ptr(), n, k, f, None,
                                            x.data_ptr(), _lib.TPL_MEM_DEVICE))
        solve()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            solve()
            ts.append(time.perf_counter() - t0)
        op.enable_timing(True)
        solve()
        p1, p2, n2 = op.pass_timing()
        op.enable_timing(False)
        iso = {name: round(op.profile_kernel(kid, 200)[0], 3) for name, kid in
               (("k_p1_spmv", 0), ("k_p1_axpy", 1), ("k_p2_spmv", 2))}
        print(json.dumps({"arcs": arcs, "elem_rows": int(e), "G2": sch["G2"], "E": sch["E"],
                          "ms_median": round(1000 * float(np.median(ts)), 4),
                          "ms_min": round(1000 * min(ts), 4),
                          "pass1_us_per_step": round(p1 / k, 3),
                          "p2_us_per_launch": round(p2 / n2, 3), "iso": iso,
                          "one_graph": bool(op.flags() & 32)}), flush=True)
        op.close()
