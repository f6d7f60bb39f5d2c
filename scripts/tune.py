"""Per-kernel HIP-event times on the 500k instance (dev tool). Env: ARCS, LIBS (list of
library paths to compare, loaded one per subprocess)."""
import os, sys, json, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("TPL_CHILD") != "1":
    libs = json.loads(os.environ.get("LIBS", "[\"\"]"))
    for spec in libs:  # "path[;KEY=VALUE...]"
        lib, *kv = spec.split(";")
        env = dict(os.environ, TPL_CHILD="1", **dict(x.split("=", 1) for x in kv))
        if lib:
            env["TPL_LIB_PATH"] = lib
        subprocess.run([sys.executable, __file__], env=env, check=False)
    sys.exit(0)
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
arcs = int(os.environ.get("ARCS", "500000"))
write_qfc_3line("/tmp/t.qfc", arcs)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
op = tpl_amd.HipCsrOp(a)
op.set_slices(int(os.environ.get("SLICES", "0")))
tpl_amd.lanczos_two_pass(op, b, 50, "inv")
row = {"lib": os.path.basename(tpl_amd.LIB_PATH), "own": os.environ.get("TPL_OWNER_SLICES", ""), "slices": op.schedule()["slices"]}
if os.environ.get("SOLVE", "1") == "1":  # full two-pass k=500 solves (ms, best of 5)
    import time
    tpl_amd.lanczos_two_pass(op, b, 500, "inv")
    ts = []
    for _ in range(5):
        t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
    row["solve_ms"] = round(1000 * min(ts), 3)
for kid, nm in [(0, "p1_spmv"), (1, "p1_axpy"), (2, "p2_spmv"), (3, "spmv")]:
    us, by = op.profile_kernel(kid, 300)
    row[nm] = round(us, 2)
print(json.dumps(row), flush=True)
