"""Dev tool: k_p2_spmv / solve time of the 500k KKT under internal arc orders
(symmetric permutations of the arc rows/columns; node rows stay last), applied outside
the engine with its own locality order switched off; "engine" = the netgen order with
the engine's locality order (tpl_op_set_reorder) on."""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import scipy.sparse as sp
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
write_qfc_3line("/tmp/t.qfc", 500000)
kkt = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc")
a = kkt.a.tocsr()
m, p = kkt.num_arcs, kkt.num_nodes
n = a.shape[0]
# arc endpoints from the node rows' columns: arc rows are 0..m-1, node rows m..m+p-1
E = a[m:, :m].tocsc()
ep = np.zeros((m, 2), dtype=np.int64)
for c in range(m):
    rows = E.indices[E.indptr[c]:E.indptr[c + 1]]
    vals = E.data[E.indptr[c]:E.indptr[c + 1]]
    ep[c] = rows if len(rows) == 2 else (rows[0], rows[0])
t, h = ep[:, 0], ep[:, 1]
orders = {"netgen": np.arange(m), "engine": None}
lo, hi = np.minimum(t, h), np.maximum(t, h)
sel = os.environ.get("ORDERS", "")
for G in (8, 16, 32):
    g = -(-p // G)
    orders[f"th{G}"] = np.lexsort((h, t, h // g, t // g))
    orders[f"mm{G}"] = np.lexsort((hi, lo, hi // g, lo // g))
    orders[f"ht{G}"] = np.lexsort((t, h, t // g, h // g))
if sel:
    orders = {k: v for k, v in orders.items() if k in sel.split(",")}
for name, order in orders.items():
    if order is None:
        ap = a
        op = tpl_amd.HipCsrOp(ap)
    else:
        perm = np.concatenate([order, np.arange(m, n)])   # new index i <- old perm[i]
        P = sp.csr_matrix((np.ones(n), (np.arange(n), perm)), shape=(n, n))
        ap = (P @ a @ P.T).tocsr()
        ap.sort_indices()
        op = tpl_amd.HipCsrOp(ap)
        op.set_reorder(False)
    b = ap @ np.full(n, 1 / np.sqrt(n))
    tpl_amd.lanczos_two_pass(op, b, 500, "inv")
    ts = []
    for _ in range(5):
        t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
    row = {"order": name, "solve_ms": round(1000 * min(ts), 3)}
    for kid, nm in [(0, "p1_spmv"), (2, "p2_spmv")]:
        row[nm] = round(op.profile_kernel(kid, 300)[0], 2)
    print(json.dumps(row), flush=True)
    op.close()
