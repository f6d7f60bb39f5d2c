"""Experiment harness on the MI355X engine — the callers of the hot path in the
reference's binaries, with the same inputs, sweeps and CSV schemas:

  tradeoff      src/bin/tradeoff.rs      variant,k,time_s,rss_kb,device_kb   (KKT instance, f = inv)
  scalability   src/bin/scalability.rs   variant,n,k,time_s,rss_kb,device_kb (several instances)
  accuracy      src/bin/stability.rs     k,relative_error_standard,relative_error_two_pass,
                                         relative_solution_deviation      (diagonal spectra)
  orthogonality src/bin/orthogonality.rs k,ortho_loss_standard,ortho_loss_regenerated,
                                         basis_drift_fro,solution_deviation_l2

    python -m tpl_amd.harness tradeoff --arcs 500000 --output tradeoff.csv
    python -m tpl_amd.harness accuracy --function inv --scenario well-conditioned --output a.csv

tradeoff / scalability follow the reference's orchestrator (src/bin/tradeoff.rs:160-214,
src/bin/scalability.rs:120-215): every variant runs in a FRESH worker process (this
module re-run with TPL_HARNESS_VARIANT set) that prints its CSV rows, so one variant's
allocations never show in the other's numbers. Per k the worker first makes one
untimed call (the engine's one-time work at a new k: growing the state / basis,
capturing and instantiating the k-step graphs), then times one call with b and x in
host memory (the reference's window, src/bin/tradeoff.rs:265-288).
  rss_kb    : VmPeak of the worker (/proc/self/status), exactly the reference's
              get_peak_rss_kb (src/utils/perf.rs:16-31) — host memory;
  device_kb : device memory the operator holds after the call (tpl_op_device_bytes):
              layout + recurrence vectors + state, plus V_k (8 n k bytes) for the
              standard variant. This is where the reference's memory trade-off lives on
              this engine (results/scalability_k500_rho3.csv: 2,090,524 vs 194,472 KB).
f(T_k) uses the engine's built-in solvers: inv = tridiagonal LU (the harness's sp_lu),
exp = symmetric tridiagonal eigensolver (self_adjoint_eigen).
"""
from __future__ import annotations

import argparse
import csv
import io
import os
import subprocess
import sys
import time

import numpy as np
import scipy.sparse as sp

from . import algorithms, solvers
from .operator import HipCsrOp
from .utils.data_loader import generate_kkt, load_kkt_system, write_qfc_3line
from .utils.rng import std_rng_f64

VARIANTS = ("standard", "two-pass")


def _rss_kb() -> int:
    """VmPeak (kB) of this process, as src/utils/perf.rs:16-31 reads it (0 if unreadable)."""
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("VmPeak:"):
                    return int(line.split()[1])
    except OSError:
        pass
    return 0


VARIANT_ENV = "TPL_HARNESS_VARIANT"


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


def _timed(variant, op, b, k):
    """One untimed call at k (one-time work), then one timed call -> (time_s, rss_kb,
    device_kb)."""
    _solve(variant, op, b, k, "inv")
    t0 = time.perf_counter()
    _solve(variant, op, b, k, "inv")
    dt = time.perf_counter() - t0
    return dt, _rss_kb(), op.device_bytes() // 1024


def tradeoff_worker(variant, a, b, ks, device: int = 0):
    """Rows (variant, k, time_s, rss_kb, device_kb) of ONE variant, k ascending
    (src/bin/tradeoff.rs:222-300, run_worker)."""
    op = HipCsrOp(a, device=device)
    rows = []
    for k in ks:
        t, rss, dev = _timed(variant, op, b, k)
        rows.append({"variant": variant, "k": k, "time_s": t, "rss_kb": rss, "device_kb": dev})
    op.close()
    return rows


def scalability_worker(variant, instances, k: int = 500, device: int = 0):
    """Rows (variant, n, k, time_s, rss_kb, device_kb) of ONE variant over the instances."""
    rows = []
    for a, b in instances:
        op = HipCsrOp(a, device=device)
        t, rss, dev = _timed(variant, op, b, k)
        rows.append({"variant": variant, "n": a.shape[0], "k": k, "time_s": t, "rss_kb": rss,
                     "device_kb": dev})
        op.close()
    return rows


def run_workers(argv, fields):
    """Orchestrator: this module once per variant in a fresh process (env VARIANT_ENV),
    each printing headerless CSV rows; returns the rows in variant order."""
    rows = []
    for v in VARIANTS:
        env = dict(os.environ, **{VARIANT_ENV: v})
        out = subprocess.run([sys.executable, "-m", "tpl_amd.harness"] + list(argv), env=env,
                             check=True, capture_output=True, text=True,
                             cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        for rec in csv.reader(io.StringIO(out.stdout)):
            if rec:
                rows.append(dict(zip(fields, rec)))
    return rows


TRADEOFF_FIELDS = ["variant", "k", "time_s", "rss_kb", "device_kb"]
SCALABILITY_FIELDS = ["variant", "n", "k", "time_s", "rss_kb", "device_kb"]


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
    argv = list(sys.argv[1:] if argv is None else argv)
    worker = os.environ.get(VARIANT_ENV)
    if a.cmd in ("tradeoff", "scalability") and worker:
        if a.cmd == "tradeoff":
            A, b = kkt_instance(a.arcs, a.dmx, a.qfc, fixtures)
            rows = tradeoff_worker(worker, A, b, list(range(a.k_start, a.k_end + 1, a.k_step)))
        else:
            rows = scalability_worker(worker, [kkt_instance(m, fixtures=fixtures) for m in a.arcs],
                                      a.k)
        w = csv.writer(sys.stdout)
        for r in rows:
            w.writerow(list(r.values()))
        return
    if a.cmd == "tradeoff":
        rows = run_workers(argv, TRADEOFF_FIELDS)
    elif a.cmd == "scalability":
        rows = run_workers(argv, SCALABILITY_FIELDS)
    elif a.cmd == "accuracy":
        rows = accuracy(a.function, a.scenario, a.n, a.k_min, a.k_max, a.k_step)
    else:
        rows = orthogonality(a.function, a.scenario, a.n, a.k_min, a.k_max, a.k_step)
    write_csv(a.output, rows)


if __name__ == "__main__":
    main()
