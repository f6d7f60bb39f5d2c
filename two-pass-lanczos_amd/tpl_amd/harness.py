"""Experiment harness on the MI355X engine — the callers of the hot path in the
reference's binaries, with the same inputs, sweeps and CSV schemas:

  tradeoff      src/bin/tradeoff.rs      variant,k,time_s,rss_kb          (KKT instance, f = inv)
  scalability   src/bin/scalability.rs   variant,n,k,time_s,rss_kb        (several instances, f = inv)
  accuracy      src/bin/stability.rs     k,relative_error_standard,relative_error_two_pass,
                                         relative_solution_deviation      (diagonal spectra)
  orthogonality src/bin/orthogonality.rs k,ortho_loss_standard,ortho_loss_regenerated,
                                         basis_drift_fro,solution_deviation_l2

    python -m tpl_amd.harness tradeoff --arcs 500000 --output tradeoff.csv
    python -m tpl_amd.harness accuracy --function inv --scenario well-conditioned --output a.csv

time_s is the wall time of one solver call with b and x in host memory (the
reference's window, src/bin/tradeoff.rs:265-288); rss_kb is the process's peak host
RSS (the basis lives in HBM here, so it does not show in RSS). f(T_k) uses the engine's
built-in solvers: inv = tridiagonal LU (the harness's sp_lu), exp = symmetric
tridiagonal eigensolver (self_adjoint_eigen).
"""
from __future__ import annotations

import argparse
import csv
import os
import resource
import time

import numpy as np
import scipy.sparse as sp

from . import algorithms, solvers
from .operator import HipCsrOp
from .utils.data_loader import generate_kkt, load_kkt_system, write_qfc_3line
from .utils.rng import std_rng_f64

VARIANTS = ("standard", "two-pass")


def _rss_kb() -> int:
    return int(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss)


def _solve(variant, op, b, k, f):
    fn = solvers.lanczos if variant == "standard" else solvers.lanczos_two_pass
    return fn(op, b, k, f)


def kkt_instance(arcs: int | None = None, dmx: str | None = None, qfc: str | None = None,
                 fixtures: str | None = None):
    """KKT operator A and the harness b = A (1/sqrt(n)) 1 (src/bin/tradeoff.rs:235-236)."""
    if dmx:
        kkt = load_kkt_system(dmx, qfc)
    elif arcs in (5000, 50000, 500000) and fixtures:
        q = os.path.join("/tmp", f"tpl_harness_{arcs}_{os.getpid()}.qfc")
        write_qfc_3line(q, arcs)
        kkt = load_kkt_system(os.path.join(fixtures, f"netgen-{arcs}-3.dmx.xz"), q)
        os.unlink(q)
    else:
        kkt = generate_kkt(int(arcs))
    a = kkt.a
    return a, a @ np.full(a.shape[0], 1.0 / np.sqrt(a.shape[0]))


def tradeoff(a, b, ks, device: int = 0):
    """Rows (variant, k, time_s, rss_kb) for every k (src/bin/tradeoff.rs:262-300)."""
    op = HipCsrOp(a, device=device)
    _solve("two-pass", op, b, min(ks), "inv")  # warm-up: layout, graphs, clocks
    rows = []
    for k in ks:
        for v in VARIANTS:
            t0 = time.perf_counter()
            _solve(v, op, b, k, "inv")
            rows.append({"variant": v, "k": k, "time_s": time.perf_counter() - t0,
                         "rss_kb": _rss_kb()})
    return rows


def scalability(instances, k: int = 500, device: int = 0):
    """Rows (variant, n, k, time_s, rss_kb), one instance after another
    (src/bin/scalability.rs)."""
    rows = []
    for a, b in instances:
        op = HipCsrOp(a, device=device)
        _solve("two-pass", op, b, min(k, 10), "inv")
        for v in VARIANTS:
            t0 = time.perf_counter()
            _solve(v, op, b, k, "inv")
            rows.append({"variant": v, "n": a.shape[0], "k": k,
                         "time_s": time.perf_counter() - t0, "rss_kb": _rss_kb()})
        op.close()
    return rows


def diagonal_problem(n: int, function: str, scenario: str):
    """Diagonal test matrix and its spectrum (src/bin/stability.rs:98-157,
    src/bin/orthogonality.rs create_diagonal_problem)."""
    i = np.arange(n, dtype=np.float64)
    d = max(n - 1, 1)
    if function == "exp" and scenario == "well-conditioned":
        eigs = -10.0 + (9.9 / d) * i
    elif function == "exp":
        eigs = -1000.0 + (999.9 / d) * i
    elif scenario == "well-conditioned":
        eigs = 0.1 + (99.9 / d) * i
    else:
        mid = n // 2
        lo = 0.1 + (0.9 / max(mid - 1, 1)) * i[:mid]
        hi = -1.0 + (0.9 / max(n - mid - 1, 1)) * (i[mid:] - mid)
        eigs = np.concatenate([lo, hi])
        eigs[mid] = 1e-8
    return sp.diags(eigs).tocsr(), eigs


def accuracy(function: str, scenario: str, n: int = 10000, k_min: int = 10, k_max: int = 200,
             k_step: int = 10, device: int = 0):
    """Rows of results/accuracy_*.csv (src/bin/stability.rs:250-312)."""
    a, eigs = diagonal_problem(n, function, scenario)
    b = std_rng_f64(n, 42)
    f = np.exp if function == "exp" else (lambda z: 1.0 / z)
    x_true = f(eigs) * b
    xn = np.linalg.norm(x_true)
    op = HipCsrOp(a, device=device)
    rows = []
    for k in range(k_min, k_max + 1, k_step):
        xs = solvers.lanczos(op, b, k, function)
        xt = solvers.lanczos_two_pass(op, b, k, function)
        rows.append({"k": k, "relative_error_standard": np.linalg.norm(xs - x_true) / xn,
                     "relative_error_two_pass": np.linalg.norm(xt - x_true) / xn,
                     "relative_solution_deviation": np.linalg.norm(xs - xt) / np.linalg.norm(xs)})
    return rows


def orthogonality(function: str, scenario: str, n: int = 10000, k_min: int = 20,
                  k_max: int = 500, k_step: int = 20, device: int = 0):
    """Rows of results/orthogonality_*.csv (src/bin/orthogonality.rs:171-225)."""
    a, _ = diagonal_problem(n, function, scenario)
    b = std_rng_f64(n, 42)
    op = HipCsrOp(a, device=device)
    rows = []
    for k in range(k_min, k_max + 1, k_step):
        out = algorithms.lanczos_standard(op, b, k)
        steps = out.decomposition.steps_taken
        if steps == 0:
            continue
        v = np.asarray(out.v_k)
        y = np.zeros(steps)
        p2 = algorithms.lanczos_pass_two_with_basis(op, b, out.decomposition, y)
        vr = np.asarray(p2.v_k)
        eye = np.eye(steps)
        rows.append({"k": steps,
                     "ortho_loss_standard": np.linalg.norm(eye - v.T @ v),
                     "ortho_loss_regenerated": np.linalg.norm(eye - vr.T @ vr),
                     "basis_drift_fro": np.linalg.norm(v - vr),
                     "solution_deviation_l2": np.linalg.norm(v @ y - vr @ y)})
    return rows


def write_csv(path: str, rows) -> None:
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else [])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def main(argv=None):
    p = argparse.ArgumentParser(prog="tpl_amd.harness")
    sub = p.add_subparsers(dest="cmd", required=True)
    fixtures = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "tests", "golden", "kkt")
    t = sub.add_parser("tradeoff")
    t.add_argument("--arcs", type=int, default=50000)
    t.add_argument("--dmx")
    t.add_argument("--qfc")
    t.add_argument("--k-start", type=int, default=50)
    t.add_argument("--k-end", type=int, default=1000)
    t.add_argument("--k-step", type=int, default=50)
    t.add_argument("--output", required=True)
    s = sub.add_parser("scalability")
    s.add_argument("--arcs", type=int, nargs="+", default=[5000, 50000, 500000])
    s.add_argument("--k", type=int, default=500)
    s.add_argument("--output", required=True)
    for name in ("accuracy", "orthogonality"):
        q = sub.add_parser(name)
        q.add_argument("--function", choices=["inv", "exp"], required=True)
        q.add_argument("--scenario", choices=["well-conditioned", "ill-conditioned"],
                       required=True)
        q.add_argument("--n", type=int, default=10000)
        q.add_argument("--k-min", type=int, default=10 if name == "accuracy" else 20)
        q.add_argument("--k-max", type=int, default=200 if name == "accuracy" else 500)
        q.add_argument("--k-step", type=int, default=10 if name == "accuracy" else 20)
        q.add_argument("--output", required=True)
    a = p.parse_args(argv)
    if a.cmd == "tradeoff":
        A, b = kkt_instance(a.arcs, a.dmx, a.qfc, fixtures)
        rows = tradeoff(A, b, list(range(a.k_start, a.k_end + 1, a.k_step)))
    elif a.cmd == "scalability":
        rows = scalability([kkt_instance(m, fixtures=fixtures) for m in a.arcs], a.k)
    elif a.cmd == "accuracy":
        rows = accuracy(a.function, a.scenario, a.n, a.k_min, a.k_max, a.k_step)
    else:
        rows = orthogonality(a.function, a.scenario, a.n, a.k_min, a.k_max, a.k_step)
    write_csv(a.output, rows)


if __name__ == "__main__":
    main()
