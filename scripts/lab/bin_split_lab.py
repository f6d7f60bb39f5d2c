"""Lab (TPL_LAB build): bin packing caps vs the SpMV tail at 500k, pinned order 13.
Configs from CONFIGS="segs:lines,..." (0 = no cap); per config: pass-one step, k_p1_spmv,
k_p2_spmv (isolated, profile_kernel), solve ms (median of 7) and the x digest (packing is
speed only: the digest must not change). Rounds alternate the configs."""
import hashlib, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
cfgs = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("CONFIGS", "0:0,128:0,64:0,0:256").split(",")]
ops = {}
for segs, lines in cfgs:
    os.environ["TPL_BIN_SEGS"] = str(segs)
    os.environ["TPL_BIN_LINES"] = str(lines)
    op = tpl_amd.HipCsrOp(a)
    op.set_order_groups(13)
    x = tpl_amd.lanczos_two_pass(op, b, 500, "inv")
    G = op.schedule()["G2"]
    ops[(segs, lines)] = op
    print(json.dumps({"segs": segs, "lines": lines, "x": hashlib.sha256(x.tobytes()).hexdigest()[:16]}), flush=True)
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for key, op in ops.items():
        ts = []
        for _ in range(7):
            t0 = time.perf_counter(); tpl_amd.lanczos_two_pass(op, b, 500, "inv"); ts.append(time.perf_counter() - t0)
        row = {"round": rnd, "segs": key[0], "lines": key[1], "solve_ms": round(1000 * float(np.median(ts)), 3)}
        for kid, nm in [(6, "pass1_step"), (0, "p1_spmv"), (2, "p2_spmv")]:
            row[nm] = round(op.profile_kernel(kid, 300)[0], 3)
        print(json.dumps(row), flush=True)
