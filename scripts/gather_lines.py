"""Dev tool (CPU): distinct cache lines the long-row bins gather per SpMV at the 500k-arc
KKT in the engine's locality order, for the gathered vector stored as 8-B values (today)
or as 16-B (w, r_j) pairs (the "form r_{j+1} = w - alpha v_j inside the next gather"
variant of pass one), with 64-B and 128-B lines. A bin = 2,048
consecutive entries of one column slice's pieces, long rows ascending (tpl_layout.cpp)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np  # noqa: E402
import tpl_amd  # noqa: E402
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line  # noqa: E402

groups = int(os.environ.get("GROUPS", "13"))
write_qfc_3line("/tmp/gl.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/gl.qfc").a
perm = tpl_amd.locality_order(a, groups=groups)
iperm = np.empty_like(perm)
iperm[perm] = np.arange(len(perm))
pa = a[perm][:, perm].tocsr()
pa.sort_indices()
n = pa.shape[0]
rl = np.diff(pa.indptr)
long_rows = np.nonzero(rl > 4)[0]
S = 8
bounds = [n * s // S for s in range(S + 1)]
for esize in (8, 16):
    for line in (64, 128):
        total = 0
        for s in range(S):
            cols = []
            for r in long_rows:
                c = pa.indices[pa.indptr[r]:pa.indptr[r + 1]]
                cols.append(c[(c >= bounds[s]) & (c < bounds[s + 1])])
            c = np.concatenate(cols)
            for b0 in range(0, len(c), 2048):
                total += len(np.unique(c[b0:b0 + 2048] * esize // line))
        print(f"groups={groups} element {esize} B, line {line} B: {total} distinct (bin, line) gathers per SpMV")
