"""Per-rank share of BASELINE configs[4]'s replicated-long-row partition at N = 2, 4, 8,
timed on ONE GPU through one RCCL rank (a prediction to hold the first
8-GPU number against).

Rank r of the replicated partition holds its block of short (arc) rows and every long
(node) row, and its node rows keep only the entries in its own columns: its local
operator IS the KKT of its arc block with all the nodes. So the submatrix A[idx][:, idx]
(idx = rank r's local rows from the runtime's own host plan, tpl_plan_create) solved as
a one-rank replicated partition runs exactly the kernels, grid sizes and bytes one rank
runs at N — the partition's own launches included — with collectives that move nothing.
What the N-rank run adds is the collectives' latency: per pass-one step two all-gathers
(the long-row partials + chunk alpha partials, then the beta totals), per pass-two step
one. So

    predicted_ms(N, L) = max over ranks of ms_per_solve(1-rank share) + (2 k + (k - 1)) L / 1000,

L = one small all-gather over xGMI at N ranks, the unknown (never measured here: one GPU
per box). bench.py --gpus N (N > 1) prints this next to its measured line and the L
the measurement implies.

    python scripts/rank_share.py [--k 500] [--ranks 8 4 2 1] [--arcs 500000] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=500)
    ap.add_argument("--ranks", type=int, nargs="*", default=[8, 4, 2, 1])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--all-ranks", type=int, default=1,
                    help="1: every rank's share (the N-rank solve waits for the slowest); "
                         "0: rank 0's only")
    ap.add_argument("--single", type=int, default=1,
                    help="1: also solve rank 0's share on the single-GPU path (0: the "
                         "one-rank partition only, e.g. under rocprofv3)")
    ap.add_argument("--arcs", type=int, default=0,
                    help="workload (bench.load_workload): default BASELINE configs[4] (5M "
                         "arcs); 500000 for the headline's shares (profiles/rank_share_500k.json)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rank_share.json"))
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import bench
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    import numpy as np
    import torch
    import torch.distributed as dist

    from tpl_amd.dist import DistContext
    dist.init_process_group("gloo", rank=0, world_size=1)
    torch.cuda.set_device(0)
    kkt, data = bench.load_workload(args.arcs or bench.ARCS_SCALE)
    a = kkt.a.tocsr()
    ctx = DistContext(0, 1, device=0, transport="rccl")
    name = "configs[2] (the headline)" if args.arcs == 500000 else "configs[4]"
    out = {"workload": f"{name}: {data}", "k": args.k, "arcs": args.arcs or bench.ARCS_SCALE,
           "shares": {}}
    for N in args.ranks:
        res = share(a, N, 0, args, ctx, single=bool(args.single))
        if args.all_ranks and N > 1:
            # every other rank's share through one RCCL rank (its kernels only): the N-rank
            # solve runs at the pace of the slowest
            per = [res["one_rank_replicated"]["ms_per_solve"]]
            for r in range(1, N):
                per.append(share(a, N, r, args, ctx, single=False)["one_rank_replicated"]["ms_per_solve"])
            res["ms_per_solve_every_rank"] = per
            res["slowest_rank"] = int(np.argmax(per))
        res["collectives_per_step"] = {"pass1": 2, "pass2": 1}
        res["collectives_per_solve"] = 2 * args.k + (args.k - 1)
        out["shares"][str(N)] = res
        print(N, json.dumps(res), flush=True)
    ctx.close()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    dist.destroy_process_group()


def share(a, N, rank, args, ctx, single=True):
    """Rank `rank`'s share at N ranks, solved as a one-rank replicated partition (and, with
    `single`, on the single-GPU path beside it)."""
    import numpy as np
    import torch

    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.dist import DistHipCsrOp
    from tpl_amd.error import check
    plan = tpl_amd.HostPlan(a, mode="replicated", nranks=N, rank=rank)
    idx = np.asarray(plan.local_rows, dtype=np.int64)
    plan.close()
    ar = a[idx][:, idx].tocsr()
    ar.sort_indices()
    n = ar.shape[0]
    b = ar @ np.full(n, 1.0 / np.sqrt(n))
    res = {"rank": rank, "rank0_rows": int(n), "rank0_nnz": int(ar.nnz)}
    for kind in (("one_rank_replicated", "single_gpu") if single else ("one_rank_replicated",)):
        op = (DistHipCsrOp(ar, ctx, mode="replicated") if kind == "one_rank_replicated"
              else tpl_amd.HipCsrOp(ar, device=0))
        bl = op.local(b) if kind == "one_rank_replicated" else b
        bd = torch.from_numpy(np.ascontiguousarray(bl)).cuda()
        xd = torch.empty_like(bd)

        def solve():
            check(_lib.tpl_lanczos_two_pass(op.handle, bd.data_ptr(), int(bd.shape[0]),
                                            args.k, _lib.FTK_INV_PTR, None, xd.data_ptr(),
                                            _lib.TPL_MEM_DEVICE))
        op.enable_timing(True)
        solve()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            solve()
            ts.append(time.perf_counter() - t)
        p1, p2, n2 = op.pass_timing()
        dec = tpl_amd.algorithms.lanczos_pass_one(op, bl, args.k)
        st = dec.steps_taken
        r = {"ms_per_solve": round(1000 * min(ts), 4), "steps": st,
             "pass1_us_per_step": round(p1 / st, 3), "pass2_us_per_step": round(p2 / n2, 3)}
        if kind == "one_rank_replicated":
            e1 = op.profile_kernel(_lib.TPL_KERNEL_EXCHANGE_P1, 200)
            e2 = op.profile_kernel(_lib.TPL_KERNEL_EXCHANGE_P2, 200)
            r["exchange_1rank_us"] = {"pass1_step": round(e1[0], 3), "pass2_step": round(e2[0], 3)}
            r["exchange_bytes_per_rank"] = {"pass1_step": int(e1[1]), "pass2_step": int(e2[1])}
        res[kind] = r
        op.close()
        del bd, xd
        torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    main()
