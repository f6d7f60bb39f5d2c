"""Workload for rocprofv3 --pmc passes (dev tool): a few two-pass solves on the 500k
KKT instance with graphs disabled (TPL_NO_GRAPH=1, set by the caller) so each kernel
is its own dispatch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
arcs = int(os.environ.get("ARCS", "500000"))
write_qfc_3line("/tmp/pmc.qfc", arcs)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt", f"netgen-{arcs}-3.dmx.xz"), "/tmp/pmc.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
op = tpl_amd.HipCsrOp(a)
for _ in range(int(os.environ.get("REPS", "2"))):
    tpl_amd.lanczos_two_pass(op, b, int(os.environ.get("K", "40")), "inv")
print("done")
