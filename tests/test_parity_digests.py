"""The parity fixtures bench.py checks every run against (tests/golden/parity.json, made by
tests/golden/make_parity.py): the expected digests of every timed workload, computed by
the CPU oracle in the device's reduction order from the runtime's own host plan
(tpl_plan_create, tpl_amd.HostPlan — no GPU).

* the fixture covers every workload the bench times, and its specs are the script's;
* the host plan is the layout rule conftest restates independently (single GPU, the
  headline's pinned order included), and refuses every device call;
* the digests recompute: the small and medium workloads, the headline partitioned over 2
  and 8 ranks (the N > 1 bench lines' `value`, ≈15 s each) and the k = 20 partition cases
  on every run (about two minutes on 8 cores); the other k = 500 partitioned and
  re-orthogonalised ones (minutes each) with TPL_PARITY_FULL=1.
The headline's digest is also the one every round-3 driver bench printed
(BENCH_r03 config.x_sha256_16 = 7bf2409fbbfac620)."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_parity  # noqa: E402
from conftest import canon_schedule, load_kkt, locality_perm  # noqa: E402

FULL = os.environ.get("TPL_PARITY_FULL") == "1"


@pytest.fixture(scope="module")
def fixture():
    with open(make_parity.OUT) as f:
        return json.load(f)


def test_fixture_covers_the_bench_workloads(fixture):
    assert set(fixture["workloads"]) == set(make_parity.WORKLOADS)
    assert set(fixture["quick"]) == set(make_parity.QUICK)
    for group, table in (("workloads", make_parity.WORKLOADS), ("quick", make_parity.QUICK)):
        for name, spec in table.items():
            got = fixture[group][name]
            assert {k: got[k] for k in spec} == spec, name
            assert "x" in got or "coef" in got
    # the bench's own names (bench.py parity_entry calls)
    import bench
    assert bench.PINNED_ORDER_GROUPS[500000] == fixture["workloads"]["headline"]["order_groups"]
    assert fixture["workloads"]["headline"]["x"] == "7bf2409fbbfac620"


@pytest.mark.parametrize("arcs,groups", [(5000, 0), (500000, 13), (500000, 0)])
def test_host_plan_is_the_restated_layout_rule(kkt_tmp, arcs, groups):
    import tpl_amd
    a = load_kkt(arcs, kkt_tmp).a
    p = tpl_amd.HostPlan(a, order_groups=groups)
    s = p.schedule()
    perm = locality_perm(a, groups=groups or 16)
    c = canon_schedule(a.tocsr()[perm][:, perm].tocsr())
    assert np.array_equal(s["perm"], perm)
    for key in ("short_rows", "long_rows"):
        assert np.array_equal(s[key], c[key]), key
    assert (s["G2"], s["E"], s["slices"]) == (c["G2"], c["E"], c["slices"])
    assert p.order_groups() == (groups or 16) and p.flags() & 64


def test_host_plan_partitions_and_refusals(kkt5k):
    import tpl_amd
    from tpl_amd import _lib
    from tpl_amd.error import TplError
    a = kkt5k.a
    n = a.shape[0]
    for mode in ("replicated", "rows"):
        rows = []
        for r in range(3):
            p = tpl_amd.HostPlan(a, mode=mode, nranks=3, rank=r)
            rows.append(p.local_rows)
            assert p.schedule()["perm"] is None and p.flags() & 1
        allr = np.concatenate(rows)
        # every row owned once (replicated: the long rows on every rank)
        if mode == "rows":
            assert np.array_equal(np.sort(allr), np.arange(n))
        else:
            u, c = np.unique(allr, return_counts=True)
            assert np.array_equal(u, np.arange(n)) and set(c) <= {1, 3}
    p = tpl_amd.HostPlan(a)
    x = np.ones(n)
    assert _lib.tpl_op_apply(p.handle, x.ctypes.data,
                             x.ctypes.data, _lib.TPL_MEM_HOST) == _lib.TPL_ERR_INVALID_ARGUMENT
    assert "plan" in _lib.last_error()
    with pytest.raises(TplError):
        tpl_amd.HostPlan(a, mode="replicated", nranks=2, rank=2)


def _check(name, spec, expected, kkt_tmp):
    got = dict(spec, **make_parity.compute(spec, kkt_tmp))
    assert got == expected, (name, got, expected)


@pytest.mark.parametrize("name", ["configs0", "headline", "configs3_one_pass", "configs4_1gpu",
                                  "configs2_replicated_N2", "configs2_replicated_N8"])
def test_digests_recompute(fixture, kkt_tmp, name):
    _check(name, make_parity.WORKLOADS[name], fixture["workloads"][name], kkt_tmp)


@pytest.mark.parametrize("name", sorted(make_parity.QUICK))
def test_partition_digests_recompute_k20(fixture, kkt_tmp, name):
    _check(name, make_parity.QUICK[name], fixture["quick"][name], kkt_tmp)


@pytest.mark.skipif(not FULL, reason="minutes per case: TPL_PARITY_FULL=1")
@pytest.mark.parametrize("name", [n for n in make_parity.WORKLOADS
                                  if n.startswith(("configs3_cgs2", "configs3_selective",
                                                   "configs4_replicated", "configs4_rows",
                                                   "configs2_replicated_N4"))])
def test_full_digests_recompute(fixture, kkt_tmp, name):
    _check(name, make_parity.WORKLOADS[name], fixture["workloads"][name], kkt_tmp)
