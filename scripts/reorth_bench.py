"""One-pass Lanczos with CGS2 full re-orthogonalisation (BASELINE configs[3]: 500k-arc
KKT, k=500, V_k in HBM) — dev timing tool. Prints wall time of tpl_lanczos_standard
(V kept on the device, not copied out) and the re-orthogonalisation traffic rate.
Env: ARCS (500000), K (500), REPS (2)."""
import ctypes, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import torch
import tpl_amd
from tpl_amd import _lib
from tpl_amd.error import check
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
arcs = int(os.environ.get("ARCS", "500000"))
k = int(os.environ.get("K", "500"))
write_qfc_3line("/tmp/rb.qfc", arcs)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/rb.qfc").a
n = a.shape[0]
b = torch.from_numpy(a @ np.full(n, 1 / np.sqrt(n))).cuda()
op = tpl_amd.HipCsrOp(a)
al, be = np.zeros(k), np.zeros(k)
steps, bn = ctypes.c_size_t(0), ctypes.c_double(0)
PD = ctypes.POINTER(ctypes.c_double)
def run(reorth):
    check(_lib.tpl_lanczos_standard(op.handle, b.data_ptr(), n, k, al.ctypes.data_as(PD),
                                    be.ctypes.data_as(PD), ctypes.byref(steps), ctypes.byref(bn),
                                    None, _lib.TPL_MEM_DEVICE, reorth, None, None))
    torch.cuda.synchronize()
for reorth in (0, 1):
    run(reorth)
    ts = []
    for _ in range(int(os.environ.get("REPS", "2"))):
        t0 = time.perf_counter(); run(reorth); ts.append(time.perf_counter() - t0)
    s = int(steps.value)
    # CGS2: per step j (1..s-1), two sweeps of (h = V_j^T r: 8 n j + 8 n) + (r -= V_j h: 8 n j + 16 n)
    byts = sum(2 * (16.0 * n * j + 24.0 * n) for j in range(1, s)) if reorth else 0.0
    print(json.dumps({"reorth": reorth, "k": k, "steps": s, "s": round(min(ts), 4),
                      "reorth_TB": round(byts / 1e12, 3)}), flush=True)
