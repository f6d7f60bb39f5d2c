"""Expected results of every workload bench.py times, computed on the CPU by the oracle
in the device's reduction order — TEST INFRASTRUCTURE (writes tests/golden/parity.json,
read by bench.py's `parity` block and pinned by tests/test_parity_digests.py).

The device's reduction order of a run is a function of the matrix and of the operator's
host-side plan (row order, short / long rows, slices, element-wise blocks; for a
partition also each rank's rows): tpl_plan_create computes exactly that plan with the
runtime's own code and no GPU (tpl_amd.HostPlan), the C oracle (oracle/lanczos_oracle.c,
canonical mode) restates the arithmetic of the reference recurrence in that order, and
tests/partition_oracle.py the partitioned orders. The GPU run is bitwise this result
(SURVEY.md §8(c) P2), so a bench line can carry a parity verdict of its own even when no
GPU test runs beside it.

Digests: first 16 hex digits of sha256 over the fp64 bytes — x in the caller's row
order (`x`), or alphas then betas (`coef`, for the runs that return no x).

    python tests/golden/make_parity.py [--only NAME ...] [--check]

--check recomputes and compares with the committed file instead of writing it.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "two-pass-lanczos_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

OUT = os.path.join(HERE, "parity.json")

# name -> workload (bench.py times each of these; order_groups as bench.py pins them:
# PINNED_ORDER_GROUPS for the headline instance, the engine default elsewhere)
WORKLOADS = {
    # BASELINE configs[2], the headline: bench.py's `value`
    "headline": dict(arcs=500000, k=500, f="inv", solver="two_pass", order_groups=13),
    # configs[0]
    "configs0": dict(arcs=5000, k=50, f="inv", solver="two_pass", order_groups=0),
    # configs[3]: solvers::lanczos (standard pass + x = ||b|| V_k y'), and the
    # re-orthogonalised standard passes (no x: alphas / betas)
    "configs3_one_pass": dict(arcs=500000, k=500, f="inv", solver="lanczos", order_groups=13),
    "configs3_cgs2": dict(arcs=500000, k=500, solver="standard", reorth="cgs2", order_groups=13),
    "configs3_selective": dict(arcs=500000, k=500, solver="standard", reorth="selective",
                               order_groups=13),
    # configs[4] on one GPU (the N = 1 point of the 1 -> N curve)
    "configs4_1gpu": dict(arcs=5000000, k=500, f="inv", solver="two_pass", order_groups=0),
    # configs[4] partitioned (bench.py --gpus N: the replicated-long-row partition; N = 1
    # is bench.py --gpus 1 --partition 1, one RCCL rank)
    "configs4_replicated_N1": dict(arcs=5000000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=1),
    "configs4_replicated_N2": dict(arcs=5000000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=2),
    "configs4_replicated_N4": dict(arcs=5000000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=4),
    "configs4_replicated_N8": dict(arcs=5000000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=8),
    # the headline partitioned (bench.py --gpus N, N > 1: the line's `value`, strong
    # scaling of configs[2]; --dist-mode auto takes the replicated long rows for the KKT)
    "configs2_replicated_N1": dict(arcs=500000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=1),
    "configs2_replicated_N2": dict(arcs=500000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=2),
    "configs2_replicated_N4": dict(arcs=500000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=4),
    "configs2_replicated_N8": dict(arcs=500000, k=500, f="inv", solver="partition",
                                   mode="replicated", nranks=8),
    # the row-block partition (bench.py --gpus N with TPL_DIST_MODE=rows): every SpMV
    # all-gathers the whole vector
    "configs4_rows_N2": dict(arcs=5000000, k=500, f="inv", solver="partition", mode="rows",
                             nranks=2),
    "configs4_rows_N4": dict(arcs=5000000, k=500, f="inv", solver="partition", mode="rows",
                             nranks=4),
    "configs4_rows_N8": dict(arcs=5000000, k=500, f="inv", solver="partition", mode="rows",
                             nranks=8),
}
# quick cases the CPU suite recomputes every run (the same code paths at a small k)
QUICK = {
    "configs2_replicated_N2_k20": dict(arcs=500000, k=20, f="inv", solver="partition",
                                       mode="replicated", nranks=2),
    "configs2_replicated_N8_k20": dict(arcs=500000, k=20, f="inv", solver="partition",
                                       mode="replicated", nranks=8),
    "configs4_replicated_N2_k20": dict(arcs=5000000, k=20, f="inv", solver="partition",
                                       mode="replicated", nranks=2),
    "configs4_replicated_N8_k20": dict(arcs=5000000, k=20, f="inv", solver="partition",
                                       mode="replicated", nranks=8),
    "configs4_rows_N2_k20": dict(arcs=5000000, k=20, f="inv", solver="partition",
                                 mode="rows", nranks=2),
    "configs4_rows_N4_k20": dict(arcs=5000000, k=20, f="inv", solver="partition",
                                 mode="rows", nranks=4),
    "configs4_rows_N8_k20": dict(arcs=5000000, k=20, f="inv", solver="partition",
                                 mode="rows", nranks=8),
}


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()[:16]


def plan_records(a, mode: str, nranks: int):
    """Every rank's record for tests/partition_oracle.py, from the runtime's own plan."""
    import tpl_amd
    recs = []
    for r in range(nranks):
        p = tpl_amd.HostPlan(a, mode=mode, nranks=nranks, rank=r)
        s = p.schedule()
        assert s["perm"] is None  # partitioned operators hold no device permutation
        recs.append({"rows": p.local_rows.copy(), "s_short": s["short_rows"],
                     "s_long": s["long_rows"], "s_G2": s["G2"], "s_E": s["E"],
                     "s_slices": s["slices"]})
        p.close()
    return recs


def compute(w: dict, tmp: str = "/tmp") -> dict:
    import oracle
    import tpl_amd
    from conftest import harness_b, load_kkt
    from tpl_amd import ftk
    a = load_kkt(w["arcs"], tmp).a
    b = harness_b(a)
    k = w["k"]
    f = {"inv": ftk.INV, "exp": ftk.EXP}.get(w.get("f"))
    out = {}
    if w["solver"] == "partition":
        from partition_oracle import PartitionOracle
        po = PartitionOracle(a, plan_records(a, w["mode"], w["nranks"]), w["mode"])
        al, be, s, bn = po.pass_one(b, k)
        x = po.pass_two(b, al, be, s, bn, f(al, be) * bn)
        out.update(x=digest(x), coef=digest(al, be), steps=int(s))
    else:
        plan = tpl_amd.HostPlan(a, order_groups=w.get("order_groups", 0))
        o = oracle.Operator(a, plan.schedule())
        plan.close()
        if w["solver"] == "two_pass":
            al, be, s, bn, _ = o.pass_one(b, k)
            x, _ = o.pass_two(b, al, be, s, bn, f(al, be) * bn)
            out.update(x=digest(x), coef=digest(al, be), steps=int(s))
        elif w["solver"] == "lanczos":
            x = o.lanczos(b, k, f)
            out.update(x=digest(x))
        elif w["solver"] == "standard":
            al, be, s, bn, V = o.pass_one(b, k, reorth=w["reorth"])
            del V
            out.update(coef=digest(al, be), steps=int(s))
        else:
            raise ValueError(w["solver"])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args(argv)
    import oracle
    oracle.set_threads(os.cpu_count() or 1)  # bitwise the same for any thread count
    old = json.load(open(OUT)) if os.path.exists(OUT) else {"workloads": {}, "quick": {}}
    res = {"generator": "tests/golden/make_parity.py", "workloads": dict(old.get("workloads", {})),
           "quick": dict(old.get("quick", {}))}
    bad = []
    for group, table in (("workloads", WORKLOADS), ("quick", QUICK)):
        for name, w in table.items():
            if args.only is not None and name not in args.only:
                continue
            t = time.time()
            got = dict(w, **compute(w))
            dt = time.time() - t
            print(f"{name}: {got} ({dt:.1f} s)", flush=True)
            if args.check and old.get(group, {}).get(name) != got:
                bad.append(name)
            res[group][name] = got
    if args.check:
        if bad:
            print("MISMATCH:", bad)
            sys.exit(1)
        return
    with open(OUT, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
        fh.write("\n")


if __name__ == "__main__":
    main()
