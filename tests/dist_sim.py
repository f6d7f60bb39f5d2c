"""Host simulation of the row-partitioned two-pass Lanczos exchange protocol (the one
tpl_runtime.cpp runs over RCCL): test infrastructure for the world_size > 1 CPU tests.

Each rank owns rows [starts[r], starts[r+1]) (tpl_dist_partition), keeps only its
block of every vector, all-gathers the vector before each SpMV, and forms alpha and
beta from the per-rank totals all-gathered and summed in rank order — so every rank
computes identical coefficients. With ``halo=True`` the vector exchange is
tpl_dist_op_create_halo's instead: each rank packs the rows of its block that another
rank's rows reference (B_r) into a slot of H = max_q |B_q| doubles, the slots are
all-gathered, and the SpMV reads remote columns through the remapped positions
[own block | R x H slots]; entries no rank sent are NaN, so a wrong map shows. Row sums follow the reference order (sequential,
ascending columns); the recurrence follows src/algorithms/mod.rs:167-212 op by op.
"""
from __future__ import annotations

import numpy as np


def allgather(tdist, local: np.ndarray, world: int) -> np.ndarray:
    import torch
    t = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64))
    parts = [torch.empty_like(t) for _ in range(world)]
    tdist.all_gather(parts, t)
    return torch.cat(parts).numpy()


def rank_sum(tdist, value: float, world: int) -> float:
    vals = allgather(tdist, np.array([value]), world)
    s = 0.0
    for v in vals:  # rank order
        s = s + float(v)
    return s


def local_spmv(rp, ci, v, x_full):
    n = len(rp) - 1
    y = np.empty(n)
    for i in range(n):
        s = 0.0
        for q in range(rp[i], rp[i + 1]):
            s = s + v[q] * x_full[ci[q]]
        y[i] = s
    return y


def seq_dot(a, b):
    s = 0.0
    for x, y in zip(a, b):
        s = s + x * y
    return s


def halo_plan(a, starts, rank):
    """(send: local indices of B_rank, H, column map of rank's block: global column ->
    position in [own block | R x H slots]) — the host half of tpl_dist_op_create_halo."""
    n = a.shape[0]
    R = len(starts) - 1
    owner = np.searchsorted(starts, np.arange(n), "right") - 1
    row_owner = np.repeat(owner, np.diff(a.indptr))
    need = np.zeros(n, dtype=bool)
    need[a.indices[row_owner != owner[a.indices]]] = True
    pos = np.full(n, -1, dtype=np.int64)
    H = 0
    for q in range(R):
        idx = np.nonzero(need[starts[q]:starts[q + 1]])[0] + starts[q]
        pos[idx] = np.arange(len(idx))
        H = max(H, len(idx))
    r0, r1 = int(starts[rank]), int(starts[rank + 1])
    ld = r1 - r0
    cmap = np.full(n, -1, dtype=np.int64)
    cmap[r0:r1] = np.arange(ld)
    rem = (owner != rank) & (pos >= 0)
    cmap[rem] = ld + owner[rem] * H + pos[rem]
    send = np.nonzero(need[r0:r1])[0]
    return send, H, cmap


def two_pass(tdist, rank, world, a, starts, b_full, k, ftk, halo=False):
    """-> (x block, alphas, betas) of lanczos_two_pass on this rank."""
    r0, r1 = int(starts[rank]), int(starts[rank + 1])
    rp = a.indptr[r0:r1 + 1] - a.indptr[r0]
    ci = a.indices[a.indptr[r0]:a.indptr[r1]]
    vv = a.data[a.indptr[r0]:a.indptr[r1]]
    counts = np.diff(starts)

    def gather_rows(loc):
        # ranks contribute blocks of different lengths: pad to the widest, then cut
        ld = int(counts.max())
        buf = np.zeros(ld)
        buf[:len(loc)] = loc
        g = allgather(tdist, buf, world).reshape(world, ld)
        return np.concatenate([g[r, :counts[r]] for r in range(world)])

    if halo:
        send, H, cmap = halo_plan(a, starts, rank)
        ci = cmap[ci]
        assert (ci >= 0).all()

        def gather(loc):  # [own block | every rank's halo slot]
            buf = np.full(H, np.nan)
            buf[:len(send)] = loc[send]
            return np.concatenate([loc, allgather(tdist, buf, world)]) if H else loc
    else:
        gather = gather_rows

    b = b_full[r0:r1].copy()
    bn = np.sqrt(rank_sum(tdist, seq_dot(b, b), world))
    tol = 1000 * np.finfo(np.float64).eps
    # pass one (src/algorithms/lanczos_two_pass.rs:65-110)
    v = b * (1.0 / bn)
    v_prev = np.zeros_like(v)
    beta_prev = 0.0
    alphas, betas = [], []
    for j in range(k):
        w = local_spmv(rp, ci, vv, gather(v))
        if j > 0:
            w = w - beta_prev * v_prev
        alpha = rank_sum(tdist, seq_dot(v, w), world)
        w = w - alpha * v
        beta = np.sqrt(rank_sum(tdist, seq_dot(w, w), world))
        alphas.append(alpha)
        if beta <= tol:
            break
        if j + 1 < k:
            betas.append(beta)
        v_prev, v = v, w * (1.0 / beta)
        beta_prev = beta
    steps = len(alphas)
    y = np.asarray(ftk(np.array(alphas), np.array(betas[:steps - 1])), dtype=np.float64) * bn
    # pass two (src/algorithms/lanczos_two_pass.rs:176-312)
    v = b * (1.0 / bn)
    v_prev = np.zeros_like(v)
    x = v * y[0]
    for j in range(steps - 1):
        w = local_spmv(rp, ci, vv, gather(v))
        if j > 0:
            w = w - betas[j - 1] * v_prev
        w = w - alphas[j] * v
        v_prev, v = v, w * (1.0 / betas[j])
        x = x + y[j + 1] * v
    return x, np.array(alphas), np.array(betas[:steps - 1])
