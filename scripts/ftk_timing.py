"""Dev tool: per-solve time of lanczos_two_pass with the built-in inv evaluated on the
device (one graph) vs on the host between two graphs, configs[0] (5k, k = 50) and the
500k headline (k = 500). Args: arcs:k pairs (default 5000:50 50000:200 500000:500), e.g.
5000:1000 5000:1365 50000:1000 50000:1365 for the top of auto mode's device range."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import torch
import tpl_amd
from tpl_amd import _lib, ftk
from tpl_amd.error import check
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
PAIRS = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or \
    [(5000, 50), (50000, 200), (500000, 500)]
for arcs, k in PAIRS:
    write_qfc_3line("/tmp/t.qfc", arcs)
    a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/t.qfc").a
    n = a.shape[0]
    b = torch.from_numpy(a @ np.full(n, 1 / np.sqrt(n))).cuda()
    x = torch.empty_like(b)
    op = tpl_amd.HipCsrOp(a)
    row = {"arcs": arcs, "k": k}
    for dev in (True, False, True, False):
        op.set_device_ftk(dev)
        solve = lambda: check(_lib.tpl_lanczos_two_pass(op.handle, b.data_ptr(), n, k, _lib.FTK_INV_PTR, None, x.data_ptr(), _lib.TPL_MEM_DEVICE))
        solve(); torch.cuda.synchronize()
        reps = 20 if arcs < 500000 else 5
        t = time.perf_counter()
        for _ in range(reps):
            solve()
        torch.cuda.synchronize()
        row[("dev" if dev else "host") + "_ms"] = round((time.perf_counter() - t) / reps * 1e3, 4)
        row[("dev" if dev else "host") + "_flag"] = op.flags() & 32
    row["steps"] = tpl_amd.algorithms.lanczos_pass_one(op, a @ np.full(n, 1 / np.sqrt(n)), k).steps_taken
    print(json.dumps(row), flush=True)
