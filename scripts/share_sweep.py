"""Dev tool: layout knobs on the replicated partition's per-rank share at N = 8 (rank 0's
rows of configs[4], scripts/rank_share.py's submatrix), on the single-GPU path: solve time
(two-pass k = 500, inv) in the caller's order and in the locality order at several group
counts, and under each column-slice count."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import torch
import bench
import tpl_amd
from tpl_amd import _lib
from tpl_amd.error import check
N = int(os.environ.get("SHARE_N", "8"))
kkt, _ = bench.load_workload(bench.ARCS_SCALE)
a = kkt.a.tocsr()
plan = tpl_amd.HostPlan(a, mode="replicated", nranks=N, rank=0)
idx = np.asarray(plan.local_rows, dtype=np.int64)
plan.close()
ar = a[idx][:, idx].tocsr()
ar.sort_indices()
n = ar.shape[0]
b = torch.from_numpy(ar @ np.full(n, 1.0 / np.sqrt(n))).cuda()
x = torch.empty_like(b)
op = tpl_amd.HipCsrOp(ar)


def t_solve(reps=5):
    f = lambda: check(_lib.tpl_lanczos_two_pass(op.handle, b.data_ptr(), n, 500, _lib.FTK_INV_PTR,
                                                None, x.data_ptr(), _lib.TPL_MEM_DEVICE))
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return round(1000 * sorted(ts)[len(ts) // 2], 4)


print(json.dumps({"n": n, "nnz": int(ar.nnz), "flags": op.flags(), "groups": op.order_groups(),
                  "slices": op.schedule()["slices"], "ms": t_solve()}), flush=True)
for rep in range(2):
    for g in (8, 12, 13, 16, 20, 24, 32, 48):
        op.set_order_groups(g)
        print(json.dumps({"rep": rep, "groups": g, "ms": t_solve()}), flush=True)
op.set_reorder(0)
print(json.dumps({"order": "caller", "ms": t_solve()}), flush=True)
op.set_reorder(2)
op.set_order_groups(16)
for s in (1, 2, 4, 8):
    op.set_slices(s)
    print(json.dumps({"slices": s, "ms": t_solve()}), flush=True)
op.set_slices(0)
