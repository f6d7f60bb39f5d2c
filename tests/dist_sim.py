"""Host simulation of the row-partitioned two-pass Lanczos exchange protocol (the one
tpl_runtime.cpp runs over RCCL): test infrastructure for the world_size > 1 CPU tests.

Each rank owns rows [starts[r], starts[r+1]) (tpl_dist_partition), keeps only its
block of every vector, all-gathers the vector before each SpMV, and forms alpha and
beta from the per-rank totals all-gathered and summed in rank order — so every rank
computes identical coefficients. Row sums follow the reference order (sequential,
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


def two_pass(tdist, rank, world, a, starts, b_full, k, ftk):
    """-> (x block, alphas, betas) of lanczos_two_pass on this rank."""
    r0, r1 = int(starts[rank]), int(starts[rank + 1])
    rp = a.indptr[r0:r1 + 1] - a.indptr[r0]
    ci = a.indices[a.indptr[r0]:a.indptr[r1]]
    vv = a.data[a.indptr[r0]:a.indptr[r1]]
    counts = np.diff(starts)

    def gather(loc):
        # ranks contribute blocks of different lengths: pad to the widest, then cut
        ld = int(counts.max())
        buf = np.zeros(ld)
        buf[:len(loc)] = loc
        g = allgather(tdist, buf, world).reshape(world, ld)
        return np.concatenate([g[r, :counts[r]] for r in range(world)])

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
