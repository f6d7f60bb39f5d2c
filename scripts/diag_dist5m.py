"""Diagnostic: replicated partition at 5M arcs over 1-2 ranks sharing one GPU (host
transport), for several long-row slice counts, against the single-GPU betas."""
import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "two-pass-lanczos_amd")]
import numpy as np
import tpl_amd
from conftest import load_kkt, harness_b
from test_gpu_dist import _run_ranks
arcs = int(sys.argv[1]) if len(sys.argv) > 1 else 5000000
k = 30
tmp = tempfile.mkdtemp()
a = load_kkt(arcs, tmp).a
b = harness_b(a)
op = tpl_amd.HipCsrOp(a)
dec = tpl_amd.algorithms.lanczos_pass_one(op, b, k)
op.close()
for world, mode, sl in [(1, "replicated", ""), (2, "replicated", "1"), (2, "replicated", "8"),
                        (2, "replicated", ""), (2, "rows", "")]:
    os.environ["TPL_TEST_SLICES"] = sl
    d = tempfile.mkdtemp()
    try:
        rs = _run_ranks(d, world, "host", mode=mode, arcs=arcs, k=k)
    except AssertionError as e:
        print(world, mode, sl, "FAILED", e, flush=True)
        continue
    be = rs[0]["be"]
    rel = np.abs(be - dec.betas) / np.abs(dec.betas)
    bad = np.nonzero(rel > 1e-12)[0]
    same = all(np.array_equal(r["be"], be) for r in rs)
    print(world, mode, sl or "auto", "first bad beta", bad[:5], "max rel", rel.max(),
          "ranks agree", same, flush=True)
