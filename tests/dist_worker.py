"""One rank of a partitioned GPU solve, started as a child process by
tests/test_gpu_dist.py (RANK / WORLD_SIZE / MASTER_* in the environment; all ranks
may share one GPU with the host transport). Writes rank<r>.npz into argv[1]."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "two-pass-lanczos_amd"))

import numpy as np  # noqa: E402


def main():
    os.makedirs(sys.argv[1], exist_ok=True)
    out, transport, arcs, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else "auto"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    import tpl_amd
    from tpl_amd.dist import DistContext, DistHipCsrOp
    from conftest import banded_hub, block_diag_spd, harness_b, load_kkt
    # TPL_TEST_MATRIX=banded / blockdiag: tests/conftest.py banded_hub / block_diag_spd (no
    # KKT structure) instead; TPL_TEST_STARTS: the row split ("0,1500,...")
    kind = os.environ.get("TPL_TEST_MATRIX")
    a = (banded_hub() if kind == "banded" else block_diag_spd() if kind == "blockdiag"
         else load_kkt(arcs, out).a)
    st = os.environ.get("TPL_TEST_STARTS")
    starts = None if not st else np.array([int(v) for v in st.split(",")], dtype=np.int64)
    b = harness_b(a)
    ctx = DistContext(rank, world, device=int(os.environ.get("TPL_DEVICE", "0")), transport=transport)
    op = DistHipCsrOp(a, ctx, starts=starts, mode=mode)
    if os.environ.get("TPL_TEST_SLICES"):  # diagnostics: force the long-row slice count
        op.set_slices(int(os.environ["TPL_TEST_SLICES"]))
    bl = op.local(b)
    x1 = tpl_amd.lanczos_two_pass(op, bl, k, "inv")
    x2 = tpl_amd.lanczos_two_pass(op, bl, k, "inv")
    dec = tpl_amd.algorithms.lanczos_pass_one(op, bl, k)
    xs = tpl_amd.lanczos(op, bl, k, "inv")
    y = op.apply(op.local(np.cos(np.arange(a.shape[0]))))
    sch = op.schedule()  # this rank's layout: the partition oracle's reduction order
    # the exchange timing ids (collective; bench.py's comm fraction), then a solve again:
    # profiling leaves nothing behind that changes the next solve
    ex = [op.profile_kernel(k_id, 5) for k_id in (4, 5)]
    x3 = tpl_amd.lanczos_two_pass(op, bl, k, "inv")
    np.savez(os.path.join(out, f"rank{rank}.npz"), x1=x1, x2=x2, x3=x3, ex_us=[e[0] for e in ex], ex_bytes=[e[1] for e in ex], xs=xs, y=y,
             al=dec.alphas, be=dec.betas, steps=dec.steps_taken, bn=dec.b_norm,
             rows=op.local_rows, mode=op.mode, s_short=sch["short_rows"],
             s_long=sch["long_rows"], s_G2=sch["G2"], s_E=sch["E"], s_slices=sch["slices"],
             starts=getattr(op, "starts", np.zeros(0, dtype=np.int64)), flags=op.flags())
    torch.cuda.synchronize()
    tdist.barrier()
    op.close()
    ctx.close()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
