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

from conftest import harness_b, load_kkt  # noqa: E402


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


def _worker(rank, world, port, tmp, arcs):
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
        x, al, be = dist_sim.two_pass(tdist, rank, world, a, st, b, 50, ftk_ref.inv)
        np.savez(os.path.join(tmp, f"rank{rank}.npz"), x=x, al=al, be=be, st=st)
    finally:
        tdist.destroy_process_group()


def test_dist_protocol_two_ranks(kkt_tmp):
    import torch.multiprocessing as mp
    import oracle
    from oracle import ftk_ref
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), kkt_tmp, 5000), nprocs=world, join=True)
    r = [np.load(os.path.join(kkt_tmp, f"rank{i}.npz")) for i in range(world)]
    # identical coefficients on every rank
    assert np.array_equal(r[0]["al"], r[1]["al"]) and np.array_equal(r[0]["be"], r[1]["be"])
    x = np.concatenate([r[i]["x"] for i in range(world)])
    a = load_kkt(5000, kkt_tmp).a
    b = harness_b(a)
    xo = oracle.Operator(a).lanczos_two_pass(b, 50, ftk_ref.inv)
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)
