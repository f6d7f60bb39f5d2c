"""Partitioned reduction orders of the multi-GPU operator, restated on the CPU — TEST
INFRASTRUCTURE (composes the C oracle's primitives; never on the product path).

The row-partitioned solve (tpl_runtime.cpp) keeps alpha, beta and x
bitwise identical on every rank because each rank reduces its own partials in the
single-GPU canonical order and the R rank totals are combined in rank order. This
module replays exactly that, given each rank's layout (HipCsrOp.schedule() on that rank),
so the partitioned GPU results can be checked BIT FOR BIT, not only within a tolerance
of the single-GPU order (at 5M arcs the Krylov process reaches its summation-order chaos
onset within ~20 steps, so a tolerance against another order stops meaning anything).

Orders restated (reference recurrence src/algorithms/mod.rs:167-212 unchanged in
between — the element-wise steps are the same IEEE operations on every rank):

* "rows" (tpl_dist_op_create_csr): rank r owns rows [starts[r], starts[r+1]) and
  gathers the whole vector; its SpMV is the canonical one over its block (long-row
  slices cut on global columns); alpha = partials([T_0 .. T_{R-1}]) with T_r = rank r's
  partials() of its alpha partials; beta^2 likewise over the norm totals.
* "replicated" (tpl_dist_op_create_replicated): rank r's vector is [its short rows |
  all long rows]; its local CSR (local indices) restricts each long row to the columns
  it owns; a long row = 0 + P_0 + P_1 + ... (rank order) of the ranks' restricted sums;
  alpha = partials([T_0 .. T_{R-1}, LB_0 .. LB_{nb-1}]) (short-row chunk totals, then the
  long rows' fma blocks of 256 (one row per thread), k_long_epi_p1); the norm of rank r covers its local
  elements [0, norm_n) (rank 0: all, others: short rows only: replicated rows once).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

import oracle


class _Rank:
    """One rank's operator(s) and its view of the global vectors."""

    def __init__(self, a, rec, mode):
        sched = {"short_rows": rec["s_short"], "long_rows": rec["s_long"], "G2": int(rec["s_G2"]),
                 "E": int(rec["s_E"]), "slices": int(rec["s_slices"])}
        self.rows = np.asarray(rec["rows"], dtype=np.int64)
        self.n = self.rows.shape[0]
        if mode == "rows":
            block = sp.csr_matrix(a[self.rows[0]:self.rows[-1] + 1])  # n_local x n_global
            self.op = oracle.Operator(block, sched)
            self.op_alpha = self.op
            self.ns = self.n
            self.norm_n = self.n
        else:
            local = self._local_csr(a, rec)
            self.op = oracle.Operator(local, sched)
            short_only = dict(sched, long_rows=np.zeros(0, dtype=np.int32))
            self.op_alpha = oracle.Operator(local, short_only)
            self.ns = len(rec["s_short"])
        self.sched = sched

    def _local_csr(self, a, rec):
        """tpl_dist_op_create_replicated's local CSR: own short rows whole, long rows
        restricted to the columns this rank owns (its short rows; long columns only on
        rank 0 — none for the KKT matrices), in local column indices."""
        m = sp.csr_matrix(a)
        n = m.shape[0]
        ns = len(rec["s_short"])
        g2l = np.full(n, -1, dtype=np.int64)
        g2l[self.rows] = np.arange(self.n)
        sub = m[self.rows]                       # local rows, global columns
        coo = sub.tocoo()
        lc = g2l[coo.col]
        keep = lc >= 0
        is_long_row = coo.row >= ns
        owned = np.where(lc >= ns, bool(rec["rank0"]), lc >= 0)
        keep &= np.where(is_long_row, owned, True)
        loc = sp.csr_matrix((coo.data[keep], (coo.row[keep], lc[keep])), shape=(self.n, self.n))
        loc.sort_indices()
        return loc


def _combine(totals):
    """partials() over the rank totals (+ further partials), as finish_partials does."""
    return oracle.reduce_partials(np.asarray(totals, dtype=np.float64))


class PartitionOracle:
    """Restated partitioned solve. recs: the ranks' records (rank order) with keys
    rows, s_short, s_long, s_G2, s_E, s_slices; mode: "rows" or "replicated"."""

    def __init__(self, a, recs, mode):
        self.a = sp.csr_matrix(a)
        self.n = self.a.shape[0]
        self.mode = mode
        self.ranks = []
        for r, rec in enumerate(recs):
            rec = dict(rec)
            rec["rank0"] = r == 0
            self.ranks.append(_Rank(self.a, rec, mode))
        if mode == "replicated":
            r0 = self.ranks[0]
            self.long_rows = r0.rows[r0.ns:]      # global indices, identical on every rank
            for rk in self.ranks[1:]:
                assert np.array_equal(rk.rows[rk.ns:], self.long_rows)
        # norm coverage: rank 0 counts the replicated rows, the others only their own
        for r, rk in enumerate(self.ranks):
            rk.norm_n = rk.n if (mode == "rows" or r == 0) else rk.ns

    # -- primitives over global vectors --------------------------------------------------
    def spmv(self, x):
        y = np.empty(self.n)
        if self.mode == "rows":
            for rk in self.ranks:
                y[rk.rows] = rk.op.apply(x)
            return y
        acc = None
        for rk in self.ranks:
            yl = rk.op.apply(x[rk.rows])
            y[rk.rows[:rk.ns]] = yl[:rk.ns]
            part = yl[rk.ns:]
            acc = 0.0 + part if acc is None else acc + part   # k_long_epi_*: y = 0; y += P_r
        if acc is not None:
            y[self.long_rows] = acc
        return y

    def alpha(self, v, w):
        tot = [rk.op_alpha.dot(v[rk.rows], w[rk.rows]) for rk in self.ranks]
        if self.mode == "replicated" and len(self.long_rows):
            tot += list(oracle.long_alpha_blocks(v[self.long_rows], w[self.long_rows]))
        return _combine(tot)

    def sumsq(self, x):
        return _combine([rk.op.sumsq(x[rk.rows][:rk.norm_n]) for rk in self.ranks])

    # -- the reference's passes in this order ---------------------------------------------
    def pass_one(self, b, k):
        """-> (alphas, betas, steps, b_norm); no breakdown handling beyond the reference's
        (src/algorithms/mod.rs:206-208)."""
        tol = 1000.0 * np.finfo(np.float64).eps
        b = np.asarray(b, dtype=np.float64)
        bn = float(np.sqrt(self.sumsq(b)))
        vc = b * (1.0 / bn)
        vp = np.zeros(self.n)
        bprev = 0.0
        al, be = [], []
        for it in range(k):
            w = self.spmv(vc)
            w = w - bprev * vp
            a_ = self.alpha(vc, w)
            al.append(a_)
            if it + 1 == k:
                break
            w = w - a_ * vc
            beta = float(np.sqrt(self.sumsq(w)))
            if beta <= tol:
                break
            be.append(beta)
            vp, vc = vc, w * (1.0 / beta)
            bprev = beta
        return np.array(al), np.array(be), len(al), bn

    def pass_two(self, b, alphas, betas, steps, b_norm, y):
        b = np.asarray(b, dtype=np.float64)
        vc = b * (1.0 / b_norm)
        x = vc * y[0]
        vp = np.zeros(self.n)
        for j in range(steps - 1):
            w = self.spmv(vc)
            w = w - (betas[j - 1] if j > 0 else 0.0) * vp
            w = w - alphas[j] * vc
            w = w * (1.0 / betas[j])
            x = x + y[j + 1] * w
            vp, vc = vc, w
        return x
