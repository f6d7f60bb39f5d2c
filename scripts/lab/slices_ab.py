"""Lab A/B of the long rows' column-slice count S on the headline (GPU).

The headline operator (500k-arc KKT, pinned locality order) is solved with
lanczos_two_pass k = 500 under each S given (tpl_op_set_slices rebuilds the layout on
the same operator), alternated REPS times; prints the median ms of SOLVES calls and x's
digest (S is part of the reduction order, so the digests differ by S).

    python scripts/lab/slices_ab.py 8 4 2
"""
import hashlib
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))


def main():
    import numpy as np
    import torch

    import bench
    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.error import check
    variants = [int(v) for v in sys.argv[1:]] or [8, 4]
    reps = int(os.environ.get("REPS", "3"))
    solves = int(os.environ.get("SOLVES", "7"))
    kkt, _ = bench.load_workload(500000)
    a = kkt.a
    n = a.shape[0]
    b = a @ np.full(n, 1.0 / np.sqrt(n))
    op = tpl_amd.HipCsrOp(a)
    op.set_order_groups(bench.PINNED_ORDER_GROUPS[500000])
    bd = torch.from_numpy(np.ascontiguousarray(b)).cuda()
    xd = torch.empty_like(bd)

    def solve():
        check(_lib.tpl_lanczos_two_pass(op.handle, bd.data_ptr(), n, 500, _lib.FTK_INV_PTR,
                                        None, xd.data_ptr(), _lib.TPL_MEM_DEVICE))
    res = {s: [] for s in variants}
    for rep in range(reps):
        for s in variants:
            op.set_slices(s)
            solve()
            torch.cuda.synchronize()
            per = []
            for _ in range(solves):
                t0 = time.perf_counter()
                solve()
                torch.cuda.synchronize()
                per.append(1000.0 * (time.perf_counter() - t0))
            x = xd.cpu().numpy()
            dig = hashlib.sha256(x.tobytes()).hexdigest()[:16]
            med = statistics.median(per)
            res[s].append(med)
            print(f"rep {rep} S={s} slices={op.schedule()['slices']} median {med:.4f} ms min {min(per):.4f} x {dig}",
                  flush=True)
    for s in variants:
        print(f"S={s}: medians {['%.4f' % v for v in res[s]]}")
    op.close()


if __name__ == "__main__":
    main()
