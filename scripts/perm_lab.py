"""Dev experiment: SpMV-shaped kernel times on the 500k KKT under symmetric arc
permutations (arcs ordered by one endpoint make each node row's out-arcs a contiguous
column run) and slice counts. Prints one JSON line per (ordering, slices)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import scipy.sparse as sp

import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line

arcs = int(os.environ.get("ARCS", "500000"))
write_qfc_3line("/tmp/t.qfc", arcs)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/t.qfc").a
a = sp.csr_matrix(a)
n = a.shape[0]
# arc rows: the rows with 2 entries
deg = np.diff(a.indptr)
arc_rows = np.nonzero(deg == 2)[0]
arc_rows = arc_rows[arc_rows < arcs]
node_rows = np.setdiff1d(np.arange(n), arc_rows)
c0 = a.indices[a.indptr[arc_rows]]
c1 = a.indices[a.indptr[arc_rows] + 1]
v0 = a.data[a.indptr[arc_rows]]
tail = np.where(v0 > 0, c0, c1)
head = np.where(v0 > 0, c1, c0)
orders = {
    "orig": np.arange(len(arc_rows)),
    "tail": np.lexsort((head, tail)),
    "head": np.lexsort((tail, head)),
    "min": np.lexsort((np.maximum(c0, c1), np.minimum(c0, c1))),
}
for name, o in [(k, orders[k]) for k in os.environ.get("ORDERS", "orig,min,tail").split(",")]:
    perm = np.concatenate([arc_rows[o], node_rows])
    ap = sp.csr_matrix(a[perm][:, perm])
    ap.sort_indices()
    b = ap @ np.full(n, 1 / np.sqrt(n))
    for s in [int(v) for v in os.environ.get("SLICES", "2,4").split(",")]:
        op = tpl_amd.HipCsrOp(ap)
        op.set_slices(s)
        tpl_amd.lanczos_two_pass(op, b, 500, "inv")
        import time
        ts = []
        for _ in range(4):
            t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
        row = {"order": name, "slices": s, "solve_ms": round(1000 * min(ts), 3)}
        for kid, nm in [(0, "p1_spmv"), (1, "p1_axpy"), (2, "p2_spmv")]:
            us, _ = op.profile_kernel(kid, 300)
            row[nm] = round(us, 2)
        print(json.dumps(row), flush=True)
        op.close()
