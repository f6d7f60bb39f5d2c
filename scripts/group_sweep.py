"""Dev tool: k_p1_spmv + k_p2_spmv time (tpl_op_tune_order's objective) of the locality
order at each group count, on the 500k KKT; twice per count to show the noise."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
op = tpl_amd.HipCsrOp(a)
for g in list(range(6, 33)) + [40, 48, 64]:
    us = [round(op.tune_order([g], iters=100)[1], 3) for _ in range(2)]
    print(json.dumps({"groups": g, "group_rows": -(-1154 // g), "p1+p2_us": us}), flush=True)
op.close()
