"""Dev tool: configs[4]'s 5M-arc instance on one GPU under element-wise block counts
(max_g2: the norm partials k_p1_spmv reduces — <= 256 takes its one-partial-per-thread
path), alternated; ms per solve and pass one per step."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import torch
import tpl_amd
from tpl_amd import _lib
from tpl_amd.error import check
from tpl_amd.utils.data_loader import generate_kkt
a = generate_kkt(5_000_000, seed=42).a
n = a.shape[0]
b = torch.from_numpy(a @ np.full(n, 1 / np.sqrt(n))).cuda()
x = torch.empty_like(b)
op = tpl_amd.HipCsrOp(a)
op.enable_timing(True)
solve = lambda: check(_lib.tpl_lanczos_two_pass(op.handle, b.data_ptr(), n, 500, _lib.FTK_INV_PTR,
                                                None, x.data_ptr(), _lib.TPL_MEM_DEVICE))
for rep in range(2):
    for g in [int(v) for v in os.environ.get("G2S", "1024,512,256").split(",")]:
        op.set_schedule(0, g)
        solve(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            solve()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 3 * 1e3
        p1, p2, n2 = op.pass_timing()
        s = op.schedule()
        print(json.dumps({"max_g2": g, "G2": s["G2"], "E": s["E"], "ms": round(ms, 3),
                          "p1_us_step": round(p1 / 500, 3), "p2_us": round(p2 / n2, 3)}), flush=True)
