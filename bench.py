#!/usr/bin/env python3
"""Headline benchmark: two-pass Lanczos f(A)b on the 500k-arc rho=3 netgen KKT instance,
k = 500, f = inv (BASELINE.json configs[2]; metric "Lanczos iterations/sec + SpMV GB/s
(vs HBM roofline), 500k-arc KKT k=500").

A "step" = one full ``solvers::lanczos_two_pass`` call (pass one, f(T_k) solve, pass
two), the window the reference times (src/bin/tradeoff.rs:265-288). Inputs (A, b) are
resident in HBM before the timed region; x stays in HBM.

    python bench.py [--gpus N --steps K --warmup W]

N > 1: when started without torch.distributed.run's environment (no WORLD_SIZE), this
process launches ``python -m torch.distributed.run --nproc-per-node N ... bench.py`` as
a CHILD (it never touches the GPU itself) and exits with its status. Each rank drives
one GPU; `value` is ONE row-partitioned solve of the SAME headline workload over the N
GPUs (replicated long rows, RCCL all-gathers in the pass graphs), timed
between barriers, max over ranks — strong scaling, so value_N / value_1 is the
partition's speed-up; rank 0 checks the assembled x against configs2_replicated_N<N> and
times the same workload on its GPU alone (single_gpu_same_workload). Then BASELINE
configs[4] (5M arcs) partitioned (`partitioned_configs4`; the N = 1 line carries it on
one GPU, configs4_5m_1gpu) and the headline on every GPU independently (`replicas`).
A failed or hung partitioned headline prints `value: null` with its status and exits
non-zero. Rehearsal on a one-GPU box: TPL_DEVICE=0 TPL_DIST_TRANSPORT=host (all ranks
share GPU 0, exchanges through host memory).

Extra JSON fields: ``roofline`` for the dominant kernel — SURVEY.md §8(d)'s B_spmv
= 12 nnz + 4 (n+1) + 16 n per launch over the live HIP-event average launch time of
k_p2_spmv, vs 8 TB/s (``frac``), with the fused-epilogue byte count, pass one and the
whole solve beside it; ``cpu_baseline`` (the oracle's reference-order restatement, one
pinned core, bounded sample on the host of the GPU box); ``pcie_inclusive`` (host b and
x: one H2D and one D2H per solve); ``one_pass_reorth`` (BASELINE configs[3]).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "Lanczos iterations/sec + SpMV GB/s (vs HBM roofline), 500k-arc KKT k=500"
ARCS_SCALE = 5000000   # BASELINE configs[4]
# Locality-order group count per netgen instance, pinned (not tuned on the box) so every
# run of the headline solve holds the same order and gives bit-identical x: 13 groups was
# the fastest of 6..64 at 500k arcs in two repeated sweeps (profiles/r02_group_sweep.txt:
# 15.3 us p1 + p2 SpMV against 15.5 at the default 16); tests/test_gpu_parity.py
# test_headline_pinned_order_bitwise checks that exact operator against the oracle.
PINNED_ORDER_GROUPS = {500000: 13}
ORACLE_CFLAGS = "gcc 11 -O2 -mfma -ffp-contract=off -fno-fast-math (oracle/Makefile)"
# Expected digests of every timed workload, computed on the CPU by the oracle in the
# device's reduction order (tests/golden/make_parity.py; pinned by
# tests/test_parity_digests.py): the `parity` block compares the GPU's results with them
PARITY_FILE = os.path.join(ROOT, "tests", "golden", "parity.json")
# configs[1] (f = exp on the device: a tolerance, not bits) against the reference-order
# oracle with LAPACK's exp (SURVEY.md §0.5 measured 1.2e-14 between orders)
EXP_TOL = 1e-10
# N > 1: the parent's limit on the whole torchrun child (then it kills the child's
# process group and reports the last stage every rank reached)
CHILD_TIMEOUT_S = 900


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--k", type=int, default=500)
    p.add_argument("--f", choices=("inv", "exp"), default="inv",
                   help="built-in f(T_k) of the timed solve (inv: the headline, configs[2]; "
                        "exp: configs[1]'s function)")
    p.add_argument("--arcs", type=int, default=0,
                   help="5000/50000/500000 (netgen fixtures) or any other count (synthetic); "
                        "default 500000 (the headline; row-partitioned at N > 1)")
    p.add_argument("--partition", type=int, default=-1,
                   help="1: row-partitioned operator even at N=1 (default: N>1)")
    p.add_argument("--single-ref", type=int, default=1,
                   help="N>1: also time the same workload on rank 0's GPU alone")
    p.add_argument("--scale-ref", type=int, default=1,
                   help="N=1: also time BASELINE configs[4] (5M arcs) on this GPU")
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the CPU leg")
    p.add_argument("--cpu-k", type=int, default=500, help="k of the bounded CPU sample")
    p.add_argument("--cpu-reps", type=int, default=3,
                   help="CPU sample repetitions (the baseline is the fastest of them)")
    p.add_argument("--order-groups", type=int, default=-1,
                   help="locality-order group count: -1 (default) the pinned count of the "
                        "instance (PINNED_ORDER_GROUPS, else 16), 0 the engine default (16), "
                        ">0 explicit")
    p.add_argument("--tune-order", type=int, default=0,
                   help="1: tpl_op_tune_order before the warm-up (times group counts on this "
                        "GPU; the chosen order, and so the bits of x, may differ between "
                        "boxes); 0 (default): the pinned group count")
    p.add_argument("--headline-only", type=int, default=0,
                   help="1: only the headline solves (no isolated kernel timings, other "
                        "configs, PCIe, one-pass, 5M or CPU legs) — for rocprofv3 runs whose "
                        "per-kernel averages must cover the timed workload alone")
    p.add_argument("--profile-iters", type=int, default=200)
    p.add_argument("--other-configs", type=int, default=1,
                   help="N=1: also time BASELINE configs[0] and [1] (5k inv k=50, 50k exp k=200)")
    p.add_argument("--one-pass", type=int, default=1,
                   help="N=1: also time BASELINE configs[3] (one-pass k with CGS2 "
                        "re-orthogonalisation, V_k in HBM); 0 to skip")
    p.add_argument("--pcie", type=int, default=1, help="N=1: also time host b / x (PCIe)")
    p.add_argument("--parity", type=int, default=1,
                   help="0 to skip the parity block (digests vs tests/golden/parity.json)")
    p.add_argument("--configs4", type=int, default=1,
                   help="N > 1: after the partitioned headline, also BASELINE configs[4] (5M "
                        "arcs) partitioned over the N GPUs (`partitioned_configs4`)")
    p.add_argument("--replicas", type=int, default=1,
                   help="N > 1: also the headline solved independently on every GPU (the "
                        "`replicas` sub-block; never `value`)")
    p.add_argument("--rank-timeout", type=float, default=600.0,
                   help="N > 1: seconds after which every rank gives up (a hung collective); "
                        "rank 0 then prints a line with no value (the headline hung) or with "
                        "the phase that hung named")
    p.add_argument("--dist-mode", choices=("auto", "replicated", "rows", "halo"),
                   default="auto",
                   help="partition of the N > 1 solve: replicated long rows (auto: when the "
                        "matrix allows it), row blocks with the whole vector all-gathered, "
                        "or row blocks exchanging only their halo (same bits as rows)")
    p.add_argument("--child-timeout", type=float, default=CHILD_TIMEOUT_S,
                   help="N>1: seconds the parent waits for the torchrun child")
    return p.parse_args(argv)


def launch_command(argv, nproc: int, port: int) -> list:
    """torch.distributed.run command line of the N-rank bench (one rank per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.join(ROOT, "bench.py")] + list(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def host_info() -> dict:
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "allowed_cpus": len(os.sched_getaffinity(0)),
            "cpu_model": model}


def cpu_threads_allowed() -> int:
    """CPU threads this process may really use: the affinity mask, capped by the cgroup's
    cpu.max quota (a GPU box shows the whole machine's CPUs in the mask but grants one GPU's
    share) and by OMP_NUM_THREADS when set."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def load_workload(arcs: int):
    from tpl_amd.utils.data_loader import generate_kkt, load_kkt_system, write_qfc_3line
    if arcs in (5000, 50000, 500000):
        dmx = os.path.join(ROOT, "tests", "golden", "kkt", f"netgen-{arcs}-3.dmx.xz")
        qfc = os.path.join("/tmp", f"tpl_bench_{arcs}_{os.getpid()}.qfc")
        write_qfc_3line(qfc, arcs)
        kkt = load_kkt_system(dmx, qfc)
        os.unlink(qfc)
        data = (f"netgen {arcs}-arc rho=3 instance regenerated from the reference's netgen "
                "(tests/golden/kkt), b = A(1/sqrt(n))1, qfc 3-line (D empty)")
    else:
        kkt = generate_kkt(arcs, seed=42)
        data = (f"synthetic {arcs}-arc rho=3 KKT (tpl_generate_kkt seed 42, "
                f"{kkt.num_nodes} nodes), b = A(1/sqrt(n))1, D empty")
    return kkt, data


def time_solves(solve, reps: int, sync) -> float:
    """Seconds per solve over `reps` calls after one untimed call."""
    solve()
    sync()
    t = time.perf_counter()
    for _ in range(reps):
        solve()
    sync()
    return (time.perf_counter() - t) / reps


def time_each(solve, reps: int, sync) -> list:
    """Seconds of each of `reps` calls (each synchronised) after one untimed call."""
    solve()
    sync()
    out = []
    for _ in range(reps):
        t = time.perf_counter()
        solve()
        sync()
        out.append(time.perf_counter() - t)
    return out


def x_digest(*arrays) -> str:
    """First 16 hex digits of sha256 over the fp64 bytes of the arrays, in order (bit
    identity across runs; the rule of tests/golden/make_parity.py)."""
    import hashlib

    import numpy as np
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()[:16]


def expected_parity() -> dict:
    try:
        with open(PARITY_FILE) as f:
            return json.load(f)["workloads"]
    except (OSError, ValueError, KeyError):
        return {}


def parity_entry(expected: dict, name: str, **got) -> dict:
    """One workload's verdict: each digest `got` (x / coef) against the committed one."""
    exp = expected.get(name)
    if exp is None:
        return {"ok": False, "error": f"no committed expectation for {name!r}"}
    ent = {}
    ok = True
    for key, val in got.items():
        ent[key] = val
        ent[key + "_expected"] = exp.get(key)
        ok = ok and val == exp.get(key)
    ent["ok"] = ok
    return ent


KERNEL_SOURCES = ("tpl_kernels.hip", "tpl_kcommon.h", "tpl_device.h", "tpl_lab.h")


def kernel_src_digest() -> str:
    """sha256 (16 hex digits) of the device-code sources in this tree: ties a committed
    profile to the kernels it measured (scripts/update_profiles.py stores the same)."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "two-pass-lanczos_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def rocprof_spmv(steps: int, b_spmv: float):
    """COMMITTED profile, not this run: in-graph durations of both SpMV kernels from the
    rocprofv3 summary of the headline (profiles/rocprof_headline.json, written by
    scripts/update_profiles.py): their fractions of the HBM roofline by B_spmv, and the
    time-weighted one over all 2k - 1 SpMV launches of a solve (k of k_p1_spmv, k - 1 of
    k_p2_spmv). `matches_build` says whether that profile measured this tree's kernels."""
    path = os.path.join(ROOT, "profiles", "rocprof_headline.json")
    try:
        with open(path) as f:
            rj = json.load(f)
    except (OSError, ValueError):
        return None
    frac = lambda ns: round(b_spmv / (ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
    out = {"source": rj.get("source"), "kernel_src_sha16": rj.get("kernel_src_sha16"),
           "matches_build": rj.get("kernel_src_sha16") == kernel_src_digest()}
    # mean (rocprofv3 --stats) and median ("median per-kernel time")
    for stat, key in (("mean", "avg_ns"), ("median", "median_ns")):
        try:
            t1, t2 = float(rj[key]["k_p1_spmv"]), float(rj[key]["k_p2_spmv"])
        except (KeyError, TypeError, ValueError):
            continue
        tw = (2 * steps - 1) * b_spmv / ((steps * t1 + (steps - 1) * t2) * 1e-9) / 1e9
        out[stat] = {"k_p1_spmv_us": round(t1 / 1000, 3), "k_p1_spmv_frac": frac(t1),
                     "k_p2_spmv_us": round(t2 / 1000, 3), "k_p2_spmv_frac": frac(t2),
                     "all_spmv_time_weighted_frac": round(tw / HBM_PEAK_GBS, 4)}
    return out if len(out) > 3 else None


def roofline_committed(b_spmv: float, live: dict):
    """The N = 1 line's `roofline`, every number recomputable from files under profiles/
    (VERDICT r05 #2): the DOMINANT SpMV kernel by its share of GPU time in the committed
    rocprofv3 --kernel-trace --stats profile of the headline (profiles/rocprof_headline.json,
    scripts/update_profiles.py), SURVEY.md §8(d)'s B_spmv over that profile's MEAN launch
    duration vs 8 TB/s (`frac`; the median beside it), and its PMC bytes per launch from the
    committed FETCH_SIZE / WRITE_SIZE passes (`traffic`). The same kernel measured live in
    this run's timed solves rides along as `frac_live` / `avg_launch_us_live` (the rest of
    the live measurement is the line's `roofline_live`). None when the committed profile
    measured other kernel sources than this tree's (then the live block stands in)."""
    try:
        with open(os.path.join(ROOT, "profiles", "rocprof_headline.json")) as f:
            rj = json.load(f)
    except (OSError, ValueError):
        return None
    if rj.get("kernel_src_sha16") != kernel_src_digest():
        return None
    try:
        share = {k: float(rj["percentage_of_gpu_time"][k]) for k in ("k_p1_spmv", "k_p2_spmv")}
        dom = max(share, key=share.get)
        avg_us = float(rj["avg_ns"][dom]) / 1000.0
    except (KeyError, TypeError, ValueError):
        return None
    gbs = lambda t_us: b_spmv / (t_us * 1e-6) / 1e9
    pmc_file = "pmc_pass_one.json" if dom == "k_p1_spmv" else "pmc_k_p2_spmv.json"
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", pmc_file)) as f:
            pj = json.load(f)
        traffic = (pj["traffic_bytes_per_launch"] if dom == "k_p2_spmv" else
                   next(v["traffic_bytes_per_launch"] for k, v in pj["kernels"].items()
                        if k.split("::")[-1].startswith(dom + "<")))
    except (OSError, ValueError, KeyError, StopIteration):
        pass
    lk = live.get("kernels", {}).get(dom, {})
    out = {"bound": "hbm", "kernel": dom, "achieved": round(gbs(avg_us), 1),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs(avg_us) / HBM_PEAK_GBS, 4),
           "traffic": traffic,
           "frac_counter_bytes": None if traffic is None else round(
               traffic / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
           "bytes_per_launch": b_spmv,
           "bytes_rule": "SURVEY.md §8(d) B_spmv = 12 nnz + 4 (n+1) + 16 n",
           "avg_launch_us": round(avg_us, 3),
           "calls_in_profile": rj.get("calls", {}).get(dom),
           "share_of_gpu_time_pct": share[dom],
           "dominant_by": "share of GPU time in the committed rocprofv3 profile",
           "source": {"avg_launch_us": "profiles/rocprof_headline.json avg_ns (from "
                                        + str(rj.get("source")) + ")",
                      "traffic": f"profiles/{pmc_file} (2 x FETCH_SIZE + WRITE_SIZE per launch)"},
           "profile_kernel_src_sha16": rj.get("kernel_src_sha16"), "matches_build": True,
           "frac_live": lk.get("frac"), "avg_launch_us_live": lk.get("avg_launch_us_events")}
    med = (rj.get("median_ns") or {}).get(dom)
    if med:
        out["median"] = {"avg_launch_us": round(float(med) / 1000.0, 3),
                         "frac": round(gbs(float(med) / 1000.0) / HBM_PEAK_GBS, 4)}
    return out


def roofline_block(b_spmv, b_fused, p2_us, p1s_us, p1a_us, n_samp, steps, p1_step_us,
                   solve_s, p2_traffic, p2_traffic_src, p1_traffic, p1_traffic_src, iso,
                   partitioned):
    """The line's `roofline`: the DOMINANT kernel by live time share (k_p1_spmv: k launches
    per solve; k_p2_spmv: k - 1; both measured live with HIP events in the timed solves —
    k_p2_spmv over the whole pass-two graph, k_p1_spmv over 8 sampled steps of pass one),
    SURVEY.md §8(d)'s B_spmv over its average launch time vs 8 TB/s (`frac`), its PMC
    counter bytes (`traffic`) and the fraction those bytes make of peak in the same time
    (`frac_counter_bytes`); the other SpMV and the time-weighted figure over all 2k - 1
    SpMV launches beside it."""
    gbs = lambda byts, t_us: byts / (t_us * 1e-6) / 1e9
    frac = lambda byts, t_us: round(gbs(byts, t_us) / HBM_PEAK_GBS, 4)
    kern = {"k_p2_spmv": {"avg_launch_us_events": round(p2_us, 3), "launches_per_solve": steps - 1,
                          "events": "one pair around the graph of the pass-two step launches",
                          "achieved": round(gbs(b_spmv, p2_us), 1), "frac": frac(b_spmv, p2_us),
                          "traffic": p2_traffic, "traffic_source": p2_traffic_src,
                          "fused_bytes_per_launch": b_fused,
                          "frac_fused_bytes": frac(b_fused, p2_us)}}
    if p1s_us:
        t1 = (p1_traffic or {}).get("k_p1_spmv")
        kern["k_p1_spmv"] = {"avg_launch_us_events": round(p1s_us, 3), "launches_per_solve": steps,
                             "events": f"start-to-start, GPU real-time clock stamps of {n_samp} middle steps' launches in the last timed solve's pass-one graph",
                             "achieved": round(gbs(b_spmv, p1s_us), 1), "frac": frac(b_spmv, p1s_us),
                             "traffic": t1, "traffic_source": p1_traffic_src}
        kern["k_p1_axpy"] = {"avg_launch_us_events": round(p1a_us, 3), "launches_per_solve": steps,
                             "traffic": (p1_traffic or {}).get("k_p1_axpy")}
    for name, kd in kern.items():
        if kd.get("traffic"):
            kd["frac_counter_bytes"] = frac(kd["traffic"], kd["avg_launch_us_events"])
    spmv = [n for n in ("k_p1_spmv", "k_p2_spmv") if n in kern]
    dom = max(spmv, key=lambda n: kern[n]["avg_launch_us_events"] * kern[n]["launches_per_solve"])
    d = kern[dom]
    out = {"bound": "hbm", "kernel": dom + ("" if not partitioned else " (+ exchange, rank 0)"),
           "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["frac"],
           "traffic": d.get("traffic"), "traffic_source": d.get("traffic_source"),
           "frac_counter_bytes": d.get("frac_counter_bytes"),
           "bytes_per_launch": b_spmv,
           "bytes_rule": "SURVEY.md §8(d) B_spmv = 12 nnz + 4 (n+1) + 16 n",
           "avg_launch_us_events": d["avg_launch_us_events"],
           "dominant_by": "live time share: avg launch (events) x launches per solve",
           "kernels": kern,
           "pass1_us_per_step": round(p1_step_us, 3),
           "frac_pass1_step": frac(b_spmv, p1_step_us),
           "frac_whole_solve": round((2 * steps - 1) * b_spmv / solve_s / 1e9 / HBM_PEAK_GBS, 4),
           "kernels_us_isolated": iso}
    if p1s_us:
        out["all_spmv_time_weighted_frac"] = round(
            (2 * steps - 1) * b_spmv / ((steps * p1s_us + (steps - 1) * p2_us) * 1e-6) / 1e9
            / HBM_PEAK_GBS, 4)
    return out


RANK_SHARE_FILE = os.path.join(ROOT, "profiles", "rank_share.json")  # configs[4], 5M arcs
# the headline's shares (configs[2], 500k arcs: scripts/rank_share.py --arcs 500000)
RANK_SHARE_500K_FILE = os.path.join(ROOT, "profiles", "rank_share_500k.json")


def rank_share_file(arcs: int) -> str:
    return RANK_SHARE_500K_FILE if arcs == 500000 else RANK_SHARE_FILE


def predicted_block(world: int, k: int, steps: int, solve_s: float, path: str = None):
    """The prediction an N-rank line is held against (scripts/rank_share.py, committed as
    profiles/rank_share.json for configs[4] and profiles/rank_share_500k.json for the
    headline): rank 0's share of the replicated partition at this N, solved on one GPU
    through one RCCL rank — every kernel one rank runs per step, with collectives that move
    nothing — plus (2 k + k - 1) all-gathers per solve at an unknown latency L each. Beside
    the measured time: the L it implies."""
    path = path or RANK_SHARE_FILE
    try:
        with open(path) as f:
            rs = json.load(f)
        sh = rs["shares"][str(world)]
    except (OSError, ValueError, KeyError):
        return None
    one = sh["one_rank_replicated"]
    if rs.get("k") != k or one.get("steps") != steps:
        return {"error": f"profile is for k={rs.get('k')}, steps={one.get('steps')}"}
    c = 2 * steps + (steps - 1)
    # the N-rank solve runs at the pace of its slowest rank's share
    t0 = max(sh.get("ms_per_solve_every_rank") or [one["ms_per_solve"]])
    kern = None
    try:  # the per-step kernels of the share (rocprofv3 trace medians; 5M, N = 8 only)
        if path == RANK_SHARE_FILE:
            with open(os.path.join(ROOT, "profiles", f"rank_share_n{world}_kernels.json")) as f:
                kern = json.load(f)
    except (OSError, ValueError):
        pass
    return {"source": f"{os.path.relpath(path, ROOT)} ({rs.get('source', 'scripts/rank_share.py')})",
            "rank0_rows": sh["rank0_rows"], "rank0_nnz": sh["rank0_nnz"],
            "ms_every_rank_share": sh.get("ms_per_solve_every_rank"),
            "per_step_us_1rank": {"pass1": one["pass1_us_per_step"],
                                  "pass2": one["pass2_us_per_step"]},
            "exchange_1rank_us": one.get("exchange_1rank_us"),
            "per_step_kernels_trace_us": None if kern is None else {
                "pass1": kern.get("pass1_step"), "pass2": kern.get("pass2_step"),
                "source": f"profiles/rank_share_n{world}_kernels.json", "note": kern.get("note")},
            "single_gpu_same_share_ms": sh.get("single_gpu", {}).get("ms_per_solve"),
            "collectives_per_step": sh["collectives_per_step"], "collectives_per_solve": c,
            "model": "ms = slowest rank's share (ms_1rank) + collectives_per_solve * L / 1000",
            "ms_1rank": t0,
            "ms_at_L_us": {str(L): round(t0 + c * L / 1000.0, 3) for L in (5, 10, 20, 40)},
            "measured_ms": round(1000.0 * solve_s, 3),
            "implied_L_us": round((1000.0 * solve_s - t0) * 1000.0 / c, 2)}


def predicted_curve(k: int, single_ms: float, path: str = None):
    """predicted_block's model for N = 2, 4, 8 at a few all-gather latencies L: ms per
    solve and the speed-up over the one-GPU solve measured in this run."""
    path = path or RANK_SHARE_FILE
    try:
        with open(path) as f:
            rs = json.load(f)
    except (OSError, ValueError):
        return None
    if rs.get("k") != k:
        return None
    out = {"source": f"{os.path.relpath(path, ROOT)} (scripts/rank_share.py): the slowest "
                     "rank's share of the replicated partition through one RCCL rank + "
                     "(3k - 1) all-gathers of latency L", "one_gpu_ms": round(single_ms, 3),
           "N": {}}
    for n in ("2", "4", "8"):
        sh = rs.get("shares", {}).get(n)
        if not sh:
            continue
        t0 = max(sh.get("ms_per_solve_every_rank") or [sh["one_rank_replicated"]["ms_per_solve"]])
        c = sh["collectives_per_solve"]
        out["N"][n] = {"ms_1rank_share": t0, "kernels_only_speedup": round(single_ms / t0, 2),
                       **{f"L{L}us": {"ms": round(t0 + c * L / 1000.0, 2),
                                      "speedup": round(single_ms / (t0 + c * L / 1000.0), 2)}
                          for L in (5, 10, 20)}}
    return out


def run_replicas(args, rank: int, world: int, dist, device: int) -> dict:
    """N > 1, the `replicas` sub-block (context, never `value`): the headline workload
    (BASELINE configs[2]: 500k-arc KKT, two-pass k = 500, f = inv) solved independently on
    every rank's GPU — no collective — K timed solves between barriers, max over ranks.
    Every rank's x must carry the headline's committed digest (the same bits on every GPU:
    the order is pinned)."""
    import numpy as np
    import torch

    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.error import check
    stage_marker("replicas: operator")
    kkt, data = load_workload(500000)
    a = kkt.a
    n = a.shape[0]
    b = a @ np.full(n, 1.0 / np.sqrt(n))
    op = tpl_amd.HipCsrOp(a, device=device)
    if op.flags() & 64:
        op.set_order_groups(PINNED_ORDER_GROUPS[500000])
    bd = torch.from_numpy(np.ascontiguousarray(b)).cuda(device)
    xd = torch.empty_like(bd)

    def solve():
        check(_lib.tpl_lanczos_two_pass(op.handle, bd.data_ptr(), n, args.k, _lib.FTK_INV_PTR,
                                        None, xd.data_ptr(), _lib.TPL_MEM_DEVICE))
    for _ in range(max(args.warmup, 1)):
        solve()
    torch.cuda.synchronize()
    dist.barrier()
    stage_marker("replicas: timed_loop")
    t0 = time.perf_counter()
    per = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        solve()
        per.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    stage_marker("replicas: timed_done")
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    steps = tpl_amd.algorithms.lanczos_pass_one(op, b, args.k).steps_taken
    mine = {"rank": rank, "device": device, "x": x_digest(xd.cpu().numpy()),
            "ms_per_solve_median": round(1000.0 * sorted(per)[len(per) // 2], 4)}
    every = [None] * world
    dist.all_gather_object(every, mine)
    expected = expected_parity().get("headline", {}).get("x")
    op.close()
    del bd, xd
    torch.cuda.empty_cache()
    return {"what": f"the headline solved independently on each of the {world} GPUs (no "
                    "collective; context for the partitioned `value`, never `value` itself)",
            "iterations_per_s_all_gpus": round(world * args.steps * steps / dt, 2),
            "ms_per_step": round(1000.0 * dt / args.steps, 4), "steps_taken": steps,
            "ranks": every,
            "parity": {"ok": expected is not None and all(e["x"] == expected for e in every),
                       "x_expected": expected, "x_every_rank": [e["x"] for e in every]}}


def partitioned_solve(args, arcs: int, rank: int, world: int, dist, dctx, device: int) -> dict:
    """ONE row-partitioned lanczos_two_pass (k = args.k, f = args.f) of the `arcs` workload
    over the `world` ranks (DistHipCsrOp, --dist-mode; RCCL all-gathers inside the pass
    graphs): K timed solves between barriers, max over ranks (strong
    scaling: the total work is the workload's, whatever N). Rank 0 assembles x from every
    rank's block and checks its digest against tests/golden/parity.json
    (configs2_<mode>_N<world> for the headline, configs4_<mode>_N<world> for configs[4]),
    times the same workload on its GPU alone (single_gpu_same_workload) and prints the
    exchange timing and the rank-share prediction beside it."""
    import numpy as np
    import torch

    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.dist import DistHipCsrOp
    from tpl_amd.error import check
    tag = f"partitioned {arcs}"
    stage_marker(f"{tag}: operator")
    kkt, data = load_workload(arcs)
    a = kkt.a
    n = a.shape[0]
    b = a @ np.full(n, 1.0 / np.sqrt(n))  # src/bin/tradeoff.rs:235-236
    op = DistHipCsrOp(a, dctx, mode=args.dist_mode)
    b_loc = op.local(b)
    b_dev = torch.from_numpy(np.ascontiguousarray(b_loc)).cuda(device)
    x_dev = torch.empty_like(b_dev)
    torch.cuda.synchronize()
    nloc = int(b_dev.shape[0])
    f_ptr = _lib.FTK_EXP_PTR if args.f == "exp" else _lib.FTK_INV_PTR

    def solve():
        check(_lib.tpl_lanczos_two_pass(op.handle, b_dev.data_ptr(), nloc, args.k, f_ptr, None,
                                        x_dev.data_ptr(), _lib.TPL_MEM_DEVICE))

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
    op.enable_timing(True)
    stage_marker(f"{tag}: first_solve (graph capture)")
    for _ in range(max(args.warmup, 0)):
        solve()
    stage_marker(f"{tag}: warmup_done")
    steps_taken = tpl_amd.algorithms.lanczos_pass_one(op, b_loc, args.k).steps_taken
    barrier()
    stage_marker(f"{tag}: timed_loop")
    t0 = time.perf_counter()
    per_solve = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        solve()
        per_solve.append(time.perf_counter() - ts)
    barrier()
    dt = time.perf_counter() - t0
    stage_marker(f"{tag}: timed_done")
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    solve_s = dt / args.steps
    p1_us, p2_us, p2_n = op.pass_timing()
    b_spmv = op.algo_bytes(_lib.TPL_KERNEL_SPMV)
    b_fused = op.algo_bytes(_lib.TPL_KERNEL_PASS2_SPMV)
    x_host = x_dev.cpu().numpy()
    parts = [None] * world if dist is not None else None
    mine = (np.asarray(op.local_rows), x_host)
    if dist is not None:
        dist.all_gather_object(parts, mine)
    else:
        parts = [mine]
    per_ms = sorted(1000.0 * t for t in per_solve)
    med_ms = float(np.median(per_ms))
    mode = op.mode
    res = {"value": round(args.steps * steps_taken / dt, 2),
           "unit": "Lanczos iterations/s",
           "ms_per_step": round(1000.0 * solve_s, 4),
           "ms_per_solve_median": round(med_ms, 4), "ms_per_solve_min": round(per_ms[0], 4),
           "iterations_per_s_median": round(steps_taken / (med_ms * 1e-3), 2),
           "scaling": "strong", "data": data, "mode": mode, "steps_taken": steps_taken,
           "config": {"workload": f"lanczos_two_pass k={args.k} f={args.f}, {arcs}-arc rho=3 "
                                  f"KKT (n={n}, nnz={a.nnz}), rows partitioned over {world} GPUs",
                      "k": args.k, "n": n, "nnz": int(a.nnz), "steps_taken": steps_taken,
                      "graphs": op.uses_graphs, "rank0_rows": nloc,
                      "parallelism": f"{mode}{world} (" + {
                          "replicated": "long-row partials all-gathered per SpMV",
                          "halo": "halo rows all-gathered per SpMV"}.get(
                              mode, "vector all-gathered per SpMV") + f", {dctx.transport})"},
           # rank 0's share, measured live: k_p2_spmv between events around its pass-two
           # graph (exchanges included); B_spmv of this rank's rows
           "roofline": roofline_block(b_spmv, b_fused, p2_us / p2_n, None, None, 0, steps_taken,
                                      p1_us / steps_taken, solve_s, None, None, None, None, {},
                                      True)}
    res["roofline"]["rank"] = 0
    x_full = None
    if rank == 0:
        x_full = np.zeros(n)
        for rows, xs in parts:
            x_full[rows] = xs
        res["config"]["x_sha256_16"] = x_digest(x_full)
        prefix = {500000: "configs2", ARCS_SCALE: "configs4"}.get(arcs)
        if args.parity and prefix and (args.k, args.f) == (500, "inv"):
            # halo row blocks reduce in the plain row blocks' order: the same digest
            key = f"{prefix}_{'rows' if mode == 'halo' else mode}_N{world}"
            res["parity"] = {key: parity_entry(expected_parity(), key, x=x_digest(x_full))}
    if args.single_ref:
        if rank == 0:
            # the same workload on rank 0's GPU alone (the headline's operator: pinned
            # order), for the speed-up of the partition and x checked against it
            op1 = tpl_amd.HipCsrOp(a, device=device)
            if op1.flags() & 64 and arcs in PINNED_ORDER_GROUPS:
                op1.set_order_groups(PINNED_ORDER_GROUPS[arcs])
            bd = torch.from_numpy(b).cuda(device)
            xd = torch.empty_like(bd)

            def solve1():
                check(_lib.tpl_lanczos_two_pass(op1.handle, bd.data_ptr(), n, args.k, f_ptr,
                                                None, xd.data_ptr(), _lib.TPL_MEM_DEVICE))
            d1 = time_solves(solve1, args.steps, torch.cuda.synchronize)
            x1 = xd.cpu().numpy()
            nb = float(np.linalg.norm(b))
            res["single_gpu_same_workload"] = {
                "value": round(steps_taken / d1, 2), "ms_per_step": round(1000.0 * d1, 4),
                "speedup_of_partition": round(d1 / solve_s, 3),
                # the partition's reduction order differs from one GPU's (rank totals), so
                # x agrees to rounding before the Krylov process turns chaotic and both
                # solve A x = b to the same residual after
                "x_rel_diff_vs_partitioned": float(np.linalg.norm(x_full - x1)
                                                   / max(np.linalg.norm(x1), 1e-300)),
                "residual_partitioned": float(np.linalg.norm(a @ x_full - b) / nb),
                "residual_single": float(np.linalg.norm(a @ x1 - b) / nb)}
            op1.close()
            del bd, xd
        barrier()
    # SURVEY.md §8(e) "comm fraction": the exchanges of one pass-one / pass-two step (rank
    # totals + all-gathers, as the pass graphs issue them) timed alone, every rank together
    try:  # a diagnostic: its failure must not cost the measured line
        ex1 = op.profile_kernel(_lib.TPL_KERNEL_EXCHANGE_P1, args.profile_iters)
        ex2 = op.profile_kernel(_lib.TPL_KERNEL_EXCHANGE_P2, args.profile_iters)
        comm_ms = (steps_taken * ex1[0] + (steps_taken - 1) * ex2[0]) / 1000.0
        res["exchange"] = {"pass1_us_per_step": round(ex1[0], 3),
                           "pass2_us_per_step": round(ex2[0], 3),
                           "bytes_received_per_step": [int(ex1[1]), int(ex2[1])],
                           "ms_per_solve": round(comm_ms, 3),
                           "comm_frac": round(comm_ms / (1000.0 * solve_s), 4)}
    except Exception as e:  # noqa: BLE001
        res["exchange"] = {"error": str(e)}
    if world > 1 and mode == "replicated" and rank == 0:
        pred = predicted_block(world, args.k, steps_taken, solve_s, rank_share_file(arcs))
        if pred is not None:
            res["predicted"] = pred
    op.close()
    del b_dev, x_dev
    torch.cuda.empty_cache()
    return res


PARITY_SOURCE = ("tests/golden/parity.json: the CPU oracle in the device's reduction order "
                 "(tests/golden/make_parity.py, pinned by tests/test_parity_digests.py)")


def parity_block(workloads: dict) -> dict:
    return {"all_ok": bool(workloads) and all(v.get("ok") is True for v in workloads.values()),
            "checked": len(workloads), "source": PARITY_SOURCE, "workloads": workloads}


def multi_line(head: dict, world: int, args) -> dict:
    """The N > 1 line (and bench.py --partition 1 at N = 1): `value` is ONE partitioned solve
    of the headline (BASELINE configs[2], 500k arcs, k = 500, f = inv) over the N GPUs —
    strong scaling of the N = 1 line's own workload, so value_N / value_1 is its speed-up."""
    keep = ("ms_per_step", "ms_per_solve_median", "ms_per_solve_min", "iterations_per_s_median",
            "data", "config", "roofline", "exchange", "predicted", "single_gpu_same_workload")
    line = {"metric": METRIC, "value": head["value"], "unit": "Lanczos iterations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "status": "ok"}
    line.update({k: head[k] for k in keep if k in head})
    line["parity"] = parity_block(dict(head.get("parity", {})))
    return line


def sub_phase_failed(line: dict, name: str, status: str, detail: str) -> dict:
    """A phase after the measured `value` (configs[4] partitioned, replicas) failed or hung:
    the line keeps its value and names the phase, and its parity verdict is no longer
    all_ok (the phase's digest was never checked)."""
    line[name] = {"status": status, "detail": detail, "last_stage_rank0": _PROGRESS["stage"],
                  "after_s": round(time.time() - _PROGRESS["t0"], 1)}
    line["status"] = f"{name}: {status}"
    line["parity"]["all_ok"] = False
    return line


def failed_line(world: int, status: str, detail: str) -> dict:
    """The N > 1 line when the partitioned headline itself failed or hung: no `value`."""
    return {"metric": METRIC, "value": None, "unit": "Lanczos iterations/s", "n_gpus": world,
            "higher_is_better": True, "status": status, "detail": detail,
            "last_stage_rank0": _PROGRESS["stage"],
            "after_s": round(time.time() - _PROGRESS["t0"], 1)}


def rank_watchdog(rank: int, world: int, args):
    """N > 1 under the driver's torchrun (no bench parent to time the ranks out): if the
    run has not finished `args.rank_timeout` s after start — a hung collective — rank 0
    prints the line it has and every rank exits, instead of the job dying silently. Before
    the partitioned headline was measured that line has NO value (status "timeout", exit
    124); after it, the value stands and the phase that hung is named (exit 0)."""
    import threading

    def fire():
        measured = _PROGRESS["line"]
        if rank == 0:
            detail = f"not finished after {args.rank_timeout} s"
            out = (failed_line(world, "timeout", detail) if measured is None else
                   sub_phase_failed(measured, _PROGRESS["phase"] or "report", "timeout", detail))
            print(json.dumps(out), flush=True)
        os._exit(0 if measured is not None else 124)
    t = threading.Timer(args.rank_timeout, fire)
    t.daemon = True
    t.start()
    return t


def run_multi(args, rank: int, world: int, dist, device: int) -> None:
    """N > 1 (and --partition 1): the partitioned headline (the line's `value`), then
    configs[4] partitioned (`partitioned_configs4`) and the replicas (`replicas`)."""
    from tpl_amd.dist import DistContext
    if dist is None:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
    dctx = DistContext(rank, world, device=device,
                       transport=os.environ.get("TPL_DIST_TRANSPORT", "rccl"))
    stage_marker("comm_init")
    arcs = args.arcs or 500000
    head = partitioned_solve(args, arcs, rank, world, dist, dctx, device)
    line = multi_line(head, world, args)
    _PROGRESS["line"] = line
    if args.configs4 and world > 1 and arcs != ARCS_SCALE:
        _PROGRESS["phase"] = "partitioned_configs4"
        try:
            c4 = partitioned_solve(args, ARCS_SCALE, rank, world, dist, dctx, device)
            line["partitioned_configs4"] = {k: v for k, v in c4.items() if k != "parity"}
            line["parity"] = parity_block(dict(line["parity"]["workloads"], **c4.get("parity", {})))
        except Exception as e:  # noqa: BLE001
            sub_phase_failed(line, "partitioned_configs4", "failed", f"{type(e).__name__}: {e}")
    if args.replicas and world > 1:
        _PROGRESS["phase"] = "replicas"
        try:
            rep = run_replicas(args, rank, world, dist, device)
            line["replicas"] = {k: v for k, v in rep.items() if k != "parity"}
            wl = dict(line["parity"]["workloads"], headline_replicas=rep["parity"])
            line["parity"] = parity_block(wl)
        except Exception as e:  # noqa: BLE001
            sub_phase_failed(line, "replicas", "failed", f"{type(e).__name__}: {e}")
    if rank == 0:
        stage_marker("report")
        print(json.dumps(line), flush=True)
    dctx.close()


# ---- N > 1: the parent process (never touches the GPU) ------------------------------
# this rank's progress, for the N > 1 watchdog (rank_watchdog): the stage it reached, the
# line once the partitioned headline is measured, and the phase running after it
_PROGRESS = {"stage": "start", "t0": time.time(), "line": None, "phase": None}


def stage_marker(stage: str) -> None:
    """Append this rank's progress to its marker file (TPL_BENCH_STAGE_DIR, set by the
    parent), so a hung or failed N-rank run still reports where every rank stopped."""
    _PROGRESS["stage"] = stage
    d = os.environ.get("TPL_BENCH_STAGE_DIR")
    if not d:
        return
    try:
        with open(os.path.join(d, f"rank{os.environ.get('RANK', '0')}.stage"), "a") as f:
            f.write(f"{time.time():.3f} {os.getpid()}:{proc_start(os.getpid())} {stage}\n")
    except OSError:
        pass


def proc_start(pid: int) -> str:
    """The process's start time in clock ticks since boot (/proc/PID/stat field 22): with
    the pid it names one process, so a recorded rank is never confused with a later
    process that reuses its pid. "" when unreadable."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        return ""


def read_stages(d: str) -> dict:
    """rank -> {"stage": last stage, "t": seconds since the parent started it}."""
    out = {}
    try:
        names = sorted(os.listdir(d))
    except OSError:
        return out
    for fn in names:
        if not fn.endswith(".stage"):
            continue
        try:
            with open(os.path.join(d, fn)) as f:
                lines = [ln.split(" ", 2) for ln in f.read().splitlines() if ln.strip()]
        except OSError:
            continue
        if lines and all(len(ln) == 3 for ln in lines):
            pid, _, start = lines[-1][1].partition(":")
            out[fn[len("rank"):-len(".stage")]] = {"stage": lines[-1][2], "stages": len(lines),
                                                   "t": float(lines[-1][0]),
                                                   "pid": int(pid), "start": start}
    return out


def run_parent(argv, nproc: int, timeout: float, cmd=None) -> int:
    """Launch the N-rank child (torchrun; `cmd` overrides it for tests) in its own process
    group, wait at most `timeout` s; on a time-out or a failure kill the whole group and
    print ONE JSON line naming the last stage each rank reached. Returns the exit status.
    That line is the LAST line of the run and the authoritative one: a rank of a failing
    child may have printed its own line before it (tests/test_bench_cli.py).
    A rank recorded in the markers is killed only while its pid still names the same
    process (its start time, /proc/PID/stat), never a later process reusing the pid."""
    import signal
    import tempfile
    d = tempfile.mkdtemp(prefix="tpl_bench_stages_")
    env = dict(os.environ, TPL_BENCH_STAGE_DIR=d)
    cmd = cmd or launch_command(argv, nproc, _free_port())
    t0 = time.time()
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    status, rc = "ok", 0
    try:
        rc = p.wait(timeout=timeout)
        if rc != 0:
            status = "failed"
    except subprocess.TimeoutExpired:
        status, rc = "timeout", 124
    if status != "ok":
        # torchrun forwards SIGTERM to its workers (each in a session of its own); then
        # SIGKILL the launcher's group and every rank pid the markers recorded
        for sig in (signal.SIGTERM, signal.SIGKILL):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=30)
                break
            except subprocess.TimeoutExpired:
                continue
        stages = read_stages(d)
        for st in stages.values():
            if st["start"] and proc_start(st["pid"]) == st["start"]:
                try:
                    os.kill(st["pid"], signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
            st["t"] = round(st["t"] - t0, 1)
            del st["pid"], st["start"]
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Lanczos iterations/s",
                          "n_gpus": nproc, "higher_is_better": True, "status": status,
                          "exit_code": rc, "child_timeout_s": timeout,
                          "wall_s": round(time.time() - t0, 1),
                          "ranks_reporting": len(stages), "last_stage": stages}), flush=True)
    return rc


def main():
    args = parse()
    if args.headline_only:
        args.other_configs = args.one_pass = args.pcie = args.scale_ref = 0
        args.cpu_baseline = args.single_ref = 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # parent of the N ranks: no GPU call here, no exec — a child under a time limit,
        # then its status (or a JSON line naming where every rank stopped)
        sys.exit(run_parent(sys.argv[1:], args.gpus, args.child_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    stage_marker("start")
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")  # barriers / max-reduce of host timings only
        stage_marker("process_group")

    import ctypes

    import numpy as np
    import torch

    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.error import check

    device = int(os.environ.get("TPL_DEVICE", local_rank))  # rehearsal: ranks sharing one GPU
    torch.cuda.set_device(device)
    partitioned = (world > 1) if args.partition < 0 else bool(args.partition)
    if partitioned:
        # the row-partitioned headline over the N GPUs
        run_multi(args, rank, world, dist, device)
        if dist is not None and world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    # ---- N = 1: the headline on one GPU, and the other configs beside it
    arcs = args.arcs or 500000
    kkt, data = load_workload(arcs)
    a = kkt.a
    n = a.shape[0]
    b = a @ np.full(n, 1.0 / np.sqrt(n))  # src/bin/tradeoff.rs:235-236

    tuned = None
    op = tpl_amd.HipCsrOp(a, device=device)
    b_loc = b
    groups = (PINNED_ORDER_GROUPS.get(arcs, 0) if args.order_groups < 0
              else args.order_groups)
    if op.flags() & 64:
        op.set_order_groups(groups)
    if args.tune_order and op.flags() & 64:
        # 30 launches per candidate: enough to separate the group counts (0.2-0.8 us
        # apart), few enough that a rocprofv3 run of this command stays dominated by
        # the solves' launches
        tuned = op.tune_order(iters=30)
    stage_marker("operator")
    b_dev = torch.from_numpy(np.ascontiguousarray(b_loc)).cuda(device)
    x_dev = torch.empty_like(b_dev)
    torch.cuda.synchronize()
    nloc = int(b_dev.shape[0])

    f_ptr = _lib.FTK_EXP_PTR if args.f == "exp" else _lib.FTK_INV_PTR

    def solve():
        check(_lib.tpl_lanczos_two_pass(op.handle, b_dev.data_ptr(), nloc, args.k,
                                        f_ptr, None, x_dev.data_ptr(),
                                        _lib.TPL_MEM_DEVICE))

    op.enable_timing(True)  # event records inside the captured passes (live timing)
    stage_marker("first_solve (graph capture)")
    for _ in range(max(args.warmup, 0)):
        solve()
    stage_marker("warmup_done")
    dec = tpl_amd.algorithms.lanczos_pass_one(op, b_loc, args.k)
    steps_taken = dec.steps_taken

    def barrier():
        torch.cuda.synchronize()

    barrier()
    stage_marker("timed_loop")
    t0 = time.perf_counter()
    per_solve = []
    for _ in range(args.steps):
        # every call returns after its own stream synchronisation (x is complete), so the
        # per-call clock adds nothing to the timed region
        ts = time.perf_counter()
        solve()
        per_solve.append(time.perf_counter() - ts)
    barrier()
    dt = time.perf_counter() - t0
    stage_marker("timed_done")

    # ---- roofline of the dominant kernel, measured live: HIP events recorded inside the
    # last timed solve's pass two (on the operator's stream) bracket its steps_taken - 1
    # k_p2_spmv launches (launch gaps included). Bytes: SURVEY.md §8(d)'s B_spmv.
    p1_us, p2_us, p2_n = op.pass_timing()
    us = p2_us / p2_n
    b_spmv = op.algo_bytes(_lib.TPL_KERNEL_SPMV)
    b_fused = op.algo_bytes(_lib.TPL_KERNEL_PASS2_SPMV)
    achieved = b_spmv / (us * 1e-6) / 1e9
    p1_step_us = p1_us / steps_taken
    # pass one's kernels, live in the pass-one graph: start stamps (GPU real-time clock)
    # of k_p1_spmv and k_p1_axpy on 8 consecutive middle steps of the last timed solve
    try:
        s1_us, a1_us, n_samp = op.step_samples()
    except Exception:  # noqa: BLE001 - partitioned / host f: no sampled pass one
        s1_us = a1_us = None
        n_samp = 0
    solve_s = dt / args.steps
    # isolated per-kernel event timings (graph of back-to-back launches), diagnostics only
    names = {_lib.TPL_KERNEL_PASS1_SPMV: "k_p1_spmv", _lib.TPL_KERNEL_PASS1_AXPY: "k_p1_axpy",
             _lib.TPL_KERNEL_PASS2_SPMV: "k_p2_spmv",
             _lib.TPL_KERNEL_PASS1_STEP: "pass1_step"}
    iso = ({} if args.headline_only else
           {names[kk]: round(op.profile_kernel(kk, args.profile_iters)[0], 3) for kk in names})
    # HBM-side traffic of the same kernel from the committed PMC profile (rocprofv3 --pmc
    # FETCH_SIZE and WRITE_SIZE in separate passes, gfx950 correction applied there)
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_k_p2_spmv.json")
    if os.path.exists(pmc) and arcs == 500000:
        with open(pmc) as f:
            pj = json.load(f)
        traffic, traffic_src = pj["traffic_bytes_per_launch"], pj["source"]

    p1_traffic, p1_traffic_src = None, None
    pmc1 = os.path.join(ROOT, "profiles", "pmc_pass_one.json")
    if os.path.exists(pmc1) and arcs == 500000 and args.k == 500:
        with open(pmc1) as f:
            pj1 = json.load(f)
        p1_traffic = {k.split("::")[-1].split("<")[0]: v["traffic_bytes_per_launch"]
                      for k, v in pj1["kernels"].items()}
        p1_traffic_src = pj1.get("source")
    iters = args.steps * steps_taken
    value = iters / dt
    x_host = x_dev.cpu().numpy()
    # parity: every timed workload's result against the digest the CPU oracle computed
    # in the device's reduction order (tests/golden/parity.json), outside the timed region
    expected = expected_parity() if args.parity else {}
    parity = {}
    if args.parity and (arcs, args.k, args.f) == (500000, 500, "inv") \
            and op.order_groups() == PINNED_ORDER_GROUPS[500000]:
        parity["headline"] = parity_entry(expected, "headline", x=x_digest(x_host),
                                          coef=x_digest(dec.alphas, dec.betas))
    per_ms = sorted(1000.0 * t for t in per_solve)
    med_ms = per_ms[len(per_ms) // 2] if len(per_ms) % 2 else 0.5 * (per_ms[len(per_ms) // 2 - 1]
                                                                      + per_ms[len(per_ms) // 2])
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Lanczos iterations/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * solve_s, 4),
        # SURVEY.md §8(d) timing protocol: median and min of the timed calls beside the mean
        "ms_per_solve_median": round(med_ms, 4),
        "ms_per_solve_min": round(per_ms[0], 4),
        "iterations_per_s_median": round(steps_taken / (med_ms * 1e-3), 2),
        "higher_is_better": True,
        # the same total work at every N: the N > 1 lines partition this solve
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data,
        "config": {"workload": f"lanczos_two_pass k={args.k} f={args.f}, {arcs}-arc rho=3 KKT "
                               f"(n={n}, nnz={a.nnz})",
                   "k": args.k, "n": n, "nnz": int(a.nnz), "steps_taken": steps_taken,
                   "graphs": op.uses_graphs,
                   "one_graph_solve": bool(op.flags() & 32),  # f(T_k) on the device
                   # tpl_op_flags bit 6: the device holds the rows in the locality order
                   "row_order": "locality" if op.flags() & 64 else "caller",
                   "order_groups": op.order_groups(),
                   **({} if tuned is None else
                      {"order_tuned": {"groups": tuned[0], "best_us": round(tuned[1], 3)}}),
                   # bits of the last timed solve's x: equal across runs of one
                   # configuration (P0, include/tpl.h tpl_op_set_order_groups)
                   "x_sha256_16": x_digest(x_host),
                   "parallelism": "single"},
        "roofline": roofline_block(b_spmv, b_fused, us, s1_us, a1_us, n_samp, steps_taken,
                                   p1_step_us, solve_s, traffic, traffic_src, p1_traffic,
                                   p1_traffic_src, iso, False),
    }

    if (arcs, args.k) == (500000, 500):
        # the 1 -> 8 curve of the N > 1 lines (the same solve partitioned), predicted from
        # the headline's committed rank shares against this run's one-GPU solve
        curve = predicted_curve(args.k, 1000.0 * solve_s, RANK_SHARE_500K_FILE)
        if curve is not None:
            out["predicted_scaling"] = curve
    rp = rocprof_spmv(steps_taken, b_spmv) if arcs == 500000 else None
    if rp is not None:
        out["roofline"]["committed_profile"] = rp
    # `roofline` from the committed profiles (recomputable), the live measurement beside it
    committed = roofline_committed(b_spmv, out["roofline"]) if (arcs, args.k) == (500000, 500) else None
    if committed is not None:
        out["roofline_live"] = out["roofline"]
        out["roofline"] = committed
    else:
        out["roofline"]["frac_source"] = "live (no committed profile of this tree's kernels)"
    if not args.headline_only:
        # the instrumentation's cost: the timed solves ran with live timing on (pass one
        # stamped, the passes in three graphs with events between them); the same solve
        # untimed is ONE graph
        op.enable_timing(False)
        tu = time_solves(solve, max(args.steps, 5), torch.cuda.synchronize)
        op.enable_timing(True)
        out["untimed_one_graph"] = {"ms_per_solve": round(1000.0 * tu, 4),
                                    "iterations_per_s": round(steps_taken / tu, 2),
                                    "note": "the same solve with live timing off (one device "
                                            "graph, no events or stamps); not `value`"}
    if args.pcie:
        # PCIe-inclusive rate (never `value`): host b in, host x out, one H2D + one D2H
        xh = np.empty(n)
        bh = np.ascontiguousarray(b)

        def solve_h():
            check(_lib.tpl_lanczos_two_pass(op.handle, bh.ctypes.data, n, args.k,
                                            _lib.FTK_INV_PTR, None, xh.ctypes.data,
                                            _lib.TPL_MEM_HOST))
        th = time_solves(solve_h, max(args.steps, 3), torch.cuda.synchronize)
        out["pcie_inclusive"] = {"iterations_per_s": round(steps_taken / th, 1),
                                 "ms_per_solve": round(1000 * th, 4),
                                 "note": "b and x in host memory (TPL_MEM_HOST)"}
    if args.one_pass:
        # BASELINE configs[3]: lanczos_standard (one pass, V_k in HBM) with CGS2 full
        # re-orthogonalisation, same instance and k; V stays on the device. The sweep
        # rate counts the algorithmic bytes of the re-orthogonalisation (per step j, two
        # passes of h = V_j^T r and r -= V_j h: 2 (16 n j + 24 n) bytes) over the time the
        # solve spends beyond the plain one-pass solve.
        PD = ctypes.POINTER(ctypes.c_double)
        al, be = np.zeros(args.k), np.zeros(args.k)
        st, bn = ctypes.c_size_t(0), ctypes.c_double(0.0)

        def one_pass(reorth):
            check(_lib.tpl_lanczos_standard(op.handle, b_dev.data_ptr(), nloc, args.k,
                                            al.ctypes.data_as(PD), be.ctypes.data_as(PD),
                                            ctypes.byref(st), ctypes.byref(bn), None,
                                            _lib.TPL_MEM_DEVICE, reorth, None, None))
        tm, second, coef = {}, {}, {}
        for r in (0, 1, 2):
            tm[r] = time_solves(lambda: one_pass(r), 2, torch.cuda.synchronize)
            second[r] = op.reorth_second_passes()
            coef[r] = x_digest(al[:st.value], be[:max(int(st.value) - 1, 0)])
        s1 = int(st.value)
        if args.parity and args.k == 500 and op.order_groups() == PINNED_ORDER_GROUPS.get(arcs):
            # configs[3]: solvers::lanczos (x = ||b|| V_k y') bit for bit; the CGS2 and
            # selective runs by their coefficients, plus ||I - V^T V||_F of the basis
            # (computed on the device: the north star's orthonormality check)
            x1p = torch.empty_like(b_dev)
            check(_lib.tpl_lanczos(op.handle, b_dev.data_ptr(), nloc, args.k, _lib.FTK_INV_PTR,
                                   None, x1p.data_ptr(), _lib.TPL_MEM_DEVICE))
            parity["configs3_one_pass"] = parity_entry(expected, "configs3_one_pass",
                                                       x=x_digest(x1p.cpu().numpy()))
            del x1p
            for r, name in ((1, "configs3_cgs2"), (2, "configs3_selective")):
                V = torch.empty((args.k, nloc), dtype=torch.float64, device=b_dev.device)
                check(_lib.tpl_lanczos_standard(op.handle, b_dev.data_ptr(), nloc, args.k,
                                                al.ctypes.data_as(PD), be.ctypes.data_as(PD),
                                                ctypes.byref(st), ctypes.byref(bn), V.data_ptr(),
                                                _lib.TPL_MEM_DEVICE, r, None, None))
                sv = int(st.value)
                V = V[:sv]
                loss = float(torch.linalg.norm(torch.eye(sv, dtype=torch.float64, device=V.device)
                                               - V @ V.T))
                ent = parity_entry(expected, name, coef=coef[r])
                ent["ortho_loss_fro"] = loss
                ent["ortho_ok"] = loss < 1e-12  # 1.9e-14 measured in numpy
                ent["ok"] = ent["ok"] and ent["ortho_ok"]
                parity[name] = ent
                del V
                torch.cuda.empty_cache()
        rb = sum(2.0 * (16.0 * n * j + 24.0 * n) for j in range(1, s1))
        rate = rb / max(tm[1] - tm[0], 1e-9) / 1e9
        out["one_pass_reorth"] = {
            "config": f"lanczos_standard k={args.k} + CGS2, V_k in HBM ({8 * n * args.k / 1e9:.2f} GB)",
            "ms_per_solve": round(1000 * tm[1], 2), "iterations_per_s": round(s1 / tm[1], 1),
            "plain_one_pass_ms": round(1000 * tm[0], 3),
            "reorth_bytes": rb, "reorth_GBs": round(rate, 1),
            "reorth_frac_of_hbm": round(rate / HBM_PEAK_GBS, 4)}
        # the selective (Kahan–Parlett) variant: the second pass only where needed; its
        # bytes: one pass per step plus a second pass on `second_passes` steps
        rb2 = sum(16.0 * n * j + 24.0 * n for j in range(1, s1)) * (1.0 + second[2] / max(s1 - 1, 1))
        rate2 = rb2 / max(tm[2] - tm[0], 1e-9) / 1e9
        out["one_pass_reorth_selective"] = {
            "config": f"lanczos_standard k={args.k} + selective CGS (Kahan-Parlett twice-is-enough)",
            "ms_per_solve": round(1000 * tm[2], 2), "iterations_per_s": round(s1 / tm[2], 1),
            "second_passes": second[2], "steps": s1,
            "reorth_GBs": round(rate2, 1), "reorth_frac_of_hbm": round(rate2 / HBM_PEAK_GBS, 4)}
    exp_case = None  # configs[1]: (A, b, device x), checked in the CPU leg
    if args.other_configs:
        # BASELINE configs[0] and [1] on the same GPU (parity-test sizes; reported, not `value`)
        others = {}
        for arcs_o, k_o, f_o, ptr in ((5000, 50, "inv", _lib.FTK_INV_PTR),
                                      (50000, 200, "exp", _lib.FTK_EXP_PTR)):
            ko, _ = load_workload(arcs_o)
            ao = ko.a
            no = ao.shape[0]
            opo = tpl_amd.HipCsrOp(ao, device=device)
            bo = torch.from_numpy(ao @ np.full(no, 1.0 / np.sqrt(no))).cuda(device)
            xo = torch.empty_like(bo)

            def solve_o():
                check(_lib.tpl_lanczos_two_pass(opo.handle, bo.data_ptr(), no, k_o, ptr, None,
                                                xo.data_ptr(), _lib.TPL_MEM_DEVICE))
            dto = time_solves(solve_o, 10, torch.cuda.synchronize)
            others[f"{arcs_o}-arc k={k_o} f={f_o}"] = {
                "ms_per_solve": round(1000 * dto, 3), "iterations_per_s": round(k_o / dto, 1),
                "n": no, "nnz": int(ao.nnz)}
            if args.parity and f_o == "inv":
                parity["configs0"] = parity_entry(expected, "configs0", x=x_digest(xo.cpu().numpy()))
            elif args.parity:
                exp_case = (ao, bo.cpu().numpy(), xo.cpu().numpy(), k_o)
            opo.close()
        out["other_configs"] = others
    if args.scale_ref:
        # BASELINE configs[4]'s workload on this one GPU: the N = 1 point of the 1 -> N curve
        # that the N > 1 lines measure (their `value` is this same solve, partitioned)
        k5, _ = load_workload(ARCS_SCALE)
        a5 = k5.a
        n5 = a5.shape[0]
        op5 = tpl_amd.HipCsrOp(a5, device=device)
        b5 = torch.from_numpy(a5 @ np.full(n5, 1.0 / np.sqrt(n5))).cuda(device)
        x5 = torch.empty_like(b5)

        def solve5():
            check(_lib.tpl_lanczos_two_pass(op5.handle, b5.data_ptr(), n5, args.k,
                                            _lib.FTK_INV_PTR, None, x5.data_ptr(),
                                            _lib.TPL_MEM_DEVICE))
        op5.enable_timing(True)
        # five calls, each timed: at 5M the run-to-run spread is several %,
        # so the line carries every call and the median is the figure
        t5 = time_each(solve5, 5, torch.cuda.synchronize)
        d5 = float(np.median(t5))
        if args.parity and args.k == 500:
            parity["configs4_1gpu"] = parity_entry(expected, "configs4_1gpu",
                                                   x=x_digest(x5.cpu().numpy()))
        q1, q2, qn = op5.pass_timing()
        u5 = q2 / qn
        out["configs4_5m_1gpu"] = {
            "workload": f"lanczos_two_pass k={args.k} f=inv, {ARCS_SCALE}-arc synthetic KKT "
                        f"(n={n5}, nnz={a5.nnz}), one GPU",
            "iterations_per_s": round(args.k / d5, 1), "ms_per_solve": round(1000 * d5, 3),
            "ms_per_solve_each": [round(1000 * t, 3) for t in t5],
            "k_p2_spmv_us": round(u5, 3),
            "frac": round(op5.algo_bytes(_lib.TPL_KERNEL_SPMV) / (u5 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        op5.close()
        # the 1 -> 8 curve the driver's node would measure, predicted from the committed
        # per-rank shares (scripts/rank_share.py) against this GPU's one-GPU solve
        curve = predicted_curve(args.k, 1000.0 * d5)
        if curve is not None:
            out["configs4_5m_1gpu"]["predicted_scaling"] = curve
    if args.cpu_baseline:
        import oracle  # CPU baseline only (reference-order restatement, single thread)
        from oracle import ftk_ref
        o = oracle.Operator(a)
        kc = min(args.cpu_k, args.k)
        reps = max(1, args.cpu_reps)
        mask = os.sched_getaffinity(0)
        core = min(mask)
        os.sched_setaffinity(0, {core})  # one pinned core, as the reference's Par::Seq
        oracle.set_threads(1)
        load0 = os.getloadavg()
        times = []
        try:
            for _ in range(reps):
                t1 = time.perf_counter()
                o.lanczos_two_pass(b, kc, ftk_ref.inv)
                times.append(time.perf_counter() - t1)
        finally:
            os.sched_setaffinity(0, mask)
        load1 = os.getloadavg()
        tc = min(times)  # the fastest call: the least disturbed by other load on the host
        out["cpu_baseline"] = {
            "value": round(kc / tc, 2), "unit": "Lanczos iterations/s", "cores": 1,
            "kind": "port",
            "sample": f"oracle C restatement (reference order, 1 thread pinned to cpu {core}) "
                      f"lanczos_two_pass k={kc} f=inv on the same instance, fastest of {reps} "
                      f"calls ({', '.join(f'{t:.2f}' for t in times)} s)",
            "calls_s": [round(t, 3) for t in times],
            "median_value": round(kc / sorted(times)[len(times) // 2], 2),
            "loadavg_before_after": [round(load0[0], 2), round(load1[0], 2)],
            "compiler": ORACLE_CFLAGS, **host_info()}
        out["speedup_vs_cpu"] = round(value / (kc / tc), 1)
        # beside it, the same restatement on every core this process may use (SURVEY.md
        # §8(d)): the SpMV and the vector updates split over OpenMP
        # threads, the dot products and norms serial in the reference's order (bits equal to
        # the one-thread run's, oracle/lanczos_oracle.c)
        nthr = cpu_threads_allowed()
        oracle.set_threads(nthr)
        load2 = os.getloadavg()
        times_all = []
        for _ in range(reps):
            t1 = time.perf_counter()
            o.lanczos_two_pass(b, kc, ftk_ref.inv)
            times_all.append(time.perf_counter() - t1)
        oracle.set_threads(1)
        ta = min(times_all)
        out["cpu_baseline"]["all_cores"] = {
            "value": round(kc / ta, 2), "unit": "Lanczos iterations/s", "cores": nthr,
            "sample": f"the same restatement and call on {nthr} OpenMP threads (SpMV and "
                      f"vector updates parallel, dot products serial), fastest of {reps} calls",
            "calls_s": [round(t, 3) for t in times_all],
            "median_value": round(kc / sorted(times_all)[len(times_all) // 2], 2),
            "loadavg_before": round(load2[0], 2),
            "threads_rule": "min(sched_getaffinity, cgroup cpu.max quota, OMP_NUM_THREADS)"}
        out["speedup_vs_cpu_all_cores"] = round(value / (kc / ta), 1)
        if (arcs, args.k, args.f) == (500000, 500, "inv"):
            # context only (not vs_baseline: BASELINE.md publishes times, not this metric):
            # the reference's own CPU times for this solve on its Xeon, one thread
            out["reference_published_cpu"] = {
                "two_pass_k500_s": {"results/tradeoff_arcs500k_rho3.csv:31": 7.539755,
                                    "results/scalability_k500_rho3.csv:21": 5.27505},
                "derived_iterations_per_s": [66.3, 94.8],
                "ratio_of_value": [round(value / 66.3, 1), round(value / 94.8, 1)],
                "hardware": "2x Xeon Gold 5318Y, parallelism disabled (BASELINE.md)"}
        if exp_case is not None:
            # configs[1]: the device exp is held to a tolerance (an EVD-class evaluation,
            # not the host QL's bits): x against the reference-order oracle with LAPACK's
            # exp
            ae, be_, xe, ke = exp_case
            oracle.set_threads(min(16, len(mask)))
            xf = oracle.Operator(ae).lanczos_two_pass(be_, ke, ftk_ref.exp)
            rel = float(np.linalg.norm(xe - xf) / np.linalg.norm(xf))
            parity["configs1_exp"] = {"rel_err_vs_reference_order": rel, "tol": EXP_TOL,
                                      "ok": rel <= EXP_TOL}
    elif exp_case is not None:
        parity["configs1_exp"] = {"ok": None, "skipped": "needs the CPU leg (--cpu-baseline 1)"}
    if parity:
        out["parity"] = parity_block(parity)
    stage_marker("report")
    print(json.dumps(out), flush=True)
    op.close()


def run():
    """main() with the N > 1 safety net: a rank-local watchdog against hangs, and — when a
    rank raises — rank 0's line instead of no line at all: with no `value` and a non-zero
    exit when the partitioned headline itself failed; with the value and the failed phase
    named when a later phase (configs[4] partitioned, replicas) failed."""
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1 or "WORLD_SIZE" not in os.environ:
        return main()
    dog = rank_watchdog(rank, world, args)
    try:
        main()
    except Exception as e:  # noqa: BLE001
        line = _PROGRESS["line"]
        detail = f"{type(e).__name__}: {e}"
        if rank == 0:
            out = (failed_line(world, "failed", detail) if line is None else
                   sub_phase_failed(line, _PROGRESS["phase"] or "report", "failed", detail))
            print(json.dumps(out), flush=True)
        # peers blocked in a collective are ended by their own watchdogs
        os._exit(1 if line is None else 0)
    finally:
        dog.cancel()


if __name__ == "__main__":
    run()
