"""World-size-2 (gloo, CPU) coverage of the row-partitioned path:
the partition rule of the C ABI (tpl_dist_partition, host-only) and the exchange
protocol the runtime runs over RCCL, simulated on host memory (tests/dist_sim.py),
against the single-process reference-order oracle."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "two-pass-lanczos_amd"))

from conftest import banded_hub, harness_b, load_kkt  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 8])
def test_partition_rule(kkt5k, nranks):
    from tpl_amd.dist import partition
    a = kkt5k.a
    st = partition(a, nranks)
    assert st[0] == 0 and st[-1] == a.shape[0]
    assert np.all(np.diff(st) >= 1)
    cost = 12.0 * a.indptr + 40.0 * np.arange(a.shape[0] + 1)
    per = np.diff(cost[st])
    # every block within one row's cost of the ideal share
    rowmax = (12.0 * np.diff(a.indptr) + 40.0).max()
    assert np.all(np.abs(per - cost[-1] / nranks) <= rowmax + 1e-9)


def test_partition_errors():
    from tpl_amd.dist import partition
    from tpl_amd.error import TplError
    with pytest.raises(TplError):
        partition((2, np.array([0, 1, 2]), np.array([0, 1]), np.ones(2)), 3)


def _worker(rank, world, port, tmp, arcs, halo=False):
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, HERE)
        import dist_sim
        from tpl_amd.dist import partition
        from oracle import ftk_ref
        a = load_kkt(arcs, tmp).a
        b = harness_b(a)
        st = partition(a, world)
        x, al, be = dist_sim.two_pass(tdist, rank, world, a, st, b, 50, ftk_ref.inv, halo=halo)
        np.savez(os.path.join(tmp, f"{'halo' if halo else 'rows'}{rank}.npz"), x=x, al=al, be=be,
                 st=st)
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("halo", [False, True])
def test_dist_protocol_two_ranks(kkt_tmp, halo):
    """The row-block exchange (whole vector all-gathered) and the halo exchange
    (tpl_dist_op_create_halo: only the referenced rows, packed into per-rank slots; NaN
    anywhere else) over gloo, world 2, against the single-process oracle."""
    import torch.multiprocessing as mp
    import oracle
    from oracle import ftk_ref
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), kkt_tmp, 5000, halo), nprocs=world, join=True)
    r = [np.load(os.path.join(kkt_tmp, f"{'halo' if halo else 'rows'}{i}.npz"))
         for i in range(world)]
    # identical coefficients on every rank
    assert np.array_equal(r[0]["al"], r[1]["al"]) and np.array_equal(r[0]["be"], r[1]["be"])
    x = np.concatenate([r[i]["x"] for i in range(world)])
    a = load_kkt(5000, kkt_tmp).a
    b = harness_b(a)
    xo = oracle.Operator(a).lanczos_two_pass(b, 50, ftk_ref.inv)
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)


def _banded_worker(rank, world, port, tmp, halo):
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, HERE)
        import dist_sim
        from tpl_amd.dist import partition
        from oracle import ftk_ref
        a = banded_hub(n=3000, hub_every=499)
        st = partition(a, world)
        x, al, be = dist_sim.two_pass(tdist, rank, world, a, st, harness_b(a), 30, ftk_ref.inv,
                                      halo=halo)
        np.savez(os.path.join(tmp, f"banded_{int(halo)}_{rank}.npz"), x=x, al=al, be=be)
    finally:
        tdist.destroy_process_group()


def test_halo_protocol_banded_three_ranks(tmp_path):
    """World 3 over gloo on a matrix without the KKT structure (band + long hub rows): the
    halo exchange gives the row-block exchange's bits (the same arithmetic, only the
    referenced rows moved) and agrees with the single-process oracle."""
    import torch.multiprocessing as mp
    import oracle
    from oracle import ftk_ref
    world = 3
    res = {}
    for halo in (False, True):
        mp.spawn(_banded_worker, args=(world, _free_port(), str(tmp_path), halo), nprocs=world,
                 join=True)
        r = [np.load(os.path.join(tmp_path, f"banded_{int(halo)}_{i}.npz")) for i in range(world)]
        res[halo] = (np.concatenate([q["x"] for q in r]), r[0]["al"], r[0]["be"])
    for u, v in zip(res[False], res[True]):
        assert np.array_equal(u, v)
    a = banded_hub(n=3000, hub_every=499)
    xo = oracle.Operator(a).lanczos_two_pass(harness_b(a), 30, ftk_ref.inv)
    assert np.linalg.norm(res[True][0] - xo) <= 1e-12 * np.linalg.norm(xo)


def _plan_worker(rank, world, port, tmp, arcs, mode):
    """One rank of a gloo world: ITS plan from the C++ runtime (tpl_plan_create — the
    code an RCCL rank runs before capturing its graphs), exchanged with the other ranks'."""
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import tpl_amd
        a = load_kkt(arcs, tmp).a
        p = tpl_amd.HostPlan(a, mode=mode, nranks=world, rank=rank)
        s = p.schedule()
        mine = {"rows": p.local_rows.copy(), "s_short": s["short_rows"], "s_long": s["long_rows"],
                "s_G2": s["G2"], "s_E": s["E"], "s_slices": s["slices"], "perm": s["perm"]}
        p.close()
        recs = [None] * world
        tdist.all_gather_object(recs, mine)
        if rank == 0:
            import pickle
            with open(os.path.join(tmp, f"plans_{mode}_{world}.pkl"), "wb") as f:
                pickle.dump(recs, f)
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("mode", ["replicated", "rows"])
def test_rank_plans_over_gloo(kkt_tmp, mode):
    """World 2 over gloo, each rank its own process: the runtime's per-rank plans cover
    every row exactly once (replicated mode: the long rows on every rank), hold no device
    permutation, and drive the partition oracle (tests/partition_oracle.py — the order the
    GPU ranks reduce in) to the same bits as plans made in one process."""
    import pickle

    import torch.multiprocessing as mp
    from partition_oracle import PartitionOracle
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_parity import digest, plan_records
    world, arcs = 2, 50000
    mp.spawn(_plan_worker, args=(world, _free_port(), kkt_tmp, arcs, mode), nprocs=world, join=True)
    with open(os.path.join(kkt_tmp, f"plans_{mode}_{world}.pkl"), "rb") as f:
        recs = pickle.load(f)  # written by this test's own rank 0 above
    a = load_kkt(arcs, kkt_tmp).a
    n = a.shape[0]
    assert all(r["perm"] is None for r in recs)
    rows = np.concatenate([r["rows"] for r in recs])
    if mode == "rows":
        assert np.array_equal(np.sort(rows), np.arange(n))
    else:
        assert np.array_equal(np.unique(rows), np.arange(n))
    local = plan_records(a, mode, world)
    for r, l in zip(recs, local):
        for key in ("rows", "s_short", "s_long"):
            assert np.array_equal(r[key], l[key]), key
        assert (r["s_G2"], r["s_E"], r["s_slices"]) == (l["s_G2"], l["s_E"], l["s_slices"])
    b = harness_b(a)
    po = PartitionOracle(a, [{k: v for k, v in r.items() if k != "perm"} for r in recs], mode)
    al, be, s, bn = po.pass_one(b, 20)
    po1 = PartitionOracle(a, local, mode)
    al1, be1, s1, bn1 = po1.pass_one(b, 20)
    assert s == s1 and digest(al, be) == digest(al1, be1)
