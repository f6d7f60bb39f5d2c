"""Dev tool: k_p1_spmv / k_p2_spmv / solve time of a KKT instance under arc orders
(symmetric permutations of the arc rows/columns; node rows stay last), applied outside
the engine with its own locality order switched off.

ARCS=500000 (netgen fixture) or any other count (the synthetic generator).
ORDERS (comma list):
  base     the instance's own order
  engine   the instance's own order, the engine's locality order on (tpl_op_set_reorder)
  engx     tests/conftest.locality_perm (the engine's rule) applied outside the engine
  gsS      arcs by (lo // S, hi // S, lo, hi): node groups of S nodes
  qG       arcs by (lo * G // p, hi * G // p, lo, hi): G node groups
  thS      arcs by (tail // S, head // S, tail, head)
  <order>t the order with the arcs that touch a short node row moved last (so every
           short-row chunk keeps a narrow column span: uint16 columns + LDS window)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import tpl_amd  # noqa: E402
from tpl_amd.utils.data_loader import generate_kkt, load_kkt_system, write_qfc_3line  # noqa: E402

arcs = int(os.environ.get("ARCS", "500000"))
k = int(os.environ.get("K", "500"))
if arcs == 500000:
    write_qfc_3line("/tmp/t.qfc", arcs)
    kkt = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"),
                          "/tmp/t.qfc")
else:
    kkt = generate_kkt(arcs)
a = kkt.a.tocsr()
m, p = kkt.num_arcs, kkt.num_nodes
n = a.shape[0]
# arc endpoints from the node rows' columns: arc rows 0..m-1, node rows m..m+p-1
E = a[m:, :m].tocsc()
E.sort_indices()
cnt = np.diff(E.indptr)
assert np.all(cnt == 2), "every arc has two distinct endpoints"
ep = E.indices.reshape(-1, 2).astype(np.int64)
# tail / head by the sign of E (tail -1, head +1 in the KKT assembly); lo / hi by index
sg = E.data.reshape(-1, 2)
t = np.where(sg[:, 0] < 0, ep[:, 0], ep[:, 1])
h = np.where(sg[:, 0] < 0, ep[:, 1], ep[:, 0])
lo, hi = ep.min(1), ep.max(1)


deg = np.bincount(np.concatenate([lo, hi]), minlength=p)
short_end = (deg[lo] <= 4) | (deg[hi] <= 4)   # arcs touching a short node row


def order_of(name):
    if name.endswith("t"):   # arcs touching a short node row moved last (engine tail rule)
        o = order_of(name[:-1])
        return np.concatenate([o[~short_end[o]], o[short_end[o]]])
    if name in ("base", "engine"):
        return np.arange(m)
    if name.startswith("gs"):
        S = int(name[2:])
        return np.lexsort((hi, lo, hi // S, lo // S))
    if name.startswith("q"):
        G = int(name[1:])
        return np.lexsort((hi, lo, hi * G // p, lo * G // p))
    if name.startswith("th"):
        S = int(name[2:])
        return np.lexsort((h, t, h // S, t // S))
    raise ValueError(name)


for name in os.environ.get("ORDERS", "base,engine").split(","):
    if name == "engx":
        from conftest import locality_perm
        perm = locality_perm(a)
    else:
        perm = np.concatenate([order_of(name), np.arange(m, n)])  # new i <- old perm[i]
    if name == "engine":
        ap = a
    else:
        P = sp.csr_matrix((np.ones(n), (np.arange(n), perm)), shape=(n, n))
        ap = (P @ a @ P.T).tocsr()
        ap.sort_indices()
    op = tpl_amd.HipCsrOp(ap)
    if name != "engine":
        op.set_reorder(False)
    b = ap @ np.full(n, 1 / np.sqrt(n))
    tpl_amd.lanczos_two_pass(op, b, k, "inv")
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        tpl_amd.lanczos_two_pass(op, b, k, "inv")
        ts.append(time.perf_counter() - t0)
    row = {"arcs": arcs, "order": name, "solve_ms": round(1000 * min(ts), 3)}
    for kid, nm in [(0, "p1_spmv"), (2, "p2_spmv")]:
        row[nm] = round(op.profile_kernel(kid, 300)[0], 2)
    print(json.dumps(row), flush=True)
    op.close()
