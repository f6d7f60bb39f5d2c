"""bench.py's driver contract on the CPU: argument plumbing and the N-GPU launcher
(the parent starts torch.distributed.run as a child — never an exec, never a GPU call —
and exits with its status)."""
import json
import time
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults():
    a = bench.parse([])
    assert (a.gpus, a.steps, a.warmup, a.k) == (1, 5, 1, 500)


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3", "--warmup", "1"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


@pytest.mark.parametrize("rc", [0, 3])
def test_parent_launches_ranks_as_child(monkeypatch, rc):
    """--gpus N without WORLD_SIZE: bench.main() runs the launcher as a child (run_parent)
    and exits with the child's status before importing torch.cuda / touching a GPU."""
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])

    def fake_parent(argv, nproc, timeout, cmd=None):
        seen.update(cmd=bench.launch_command(argv, nproc, 1), timeout=timeout)
        return rc
    monkeypatch.setattr(bench, "run_parent", fake_parent)
    monkeypatch.setattr(bench.os, "execv", lambda *a: pytest.fail("exec"), raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == rc
    assert "--nproc-per-node=2" in seen["cmd"]
    assert seen["cmd"][-4:] == ["--gpus", "2", "--steps", "1"]
    assert seen["timeout"] == bench.CHILD_TIMEOUT_S


# a stub of the N-rank child: two "ranks" that write stage markers as bench.main() does,
# then either finish, fail, or hang past the parent's limit
_STUB = r"""
import os, subprocess, sys, time
mode = sys.argv[1]
if len(sys.argv) == 2:  # the launcher: start two ranks in sessions of their own (torchrun)
    if os.environ.get("FAKE_PID"):  # a marker whose pid now names another process
        with open(os.path.join(os.environ["TPL_BENCH_STAGE_DIR"], "rank9.stage"), "w") as f:
            f.write(f"{time.time():.3f} {os.environ['FAKE_PID']}:1 start\n")
    ps = [subprocess.Popen([sys.executable, __file__, mode, str(r)], start_new_session=True,
                           env=dict(os.environ, RANK=str(r))) for r in range(2)]
    sys.exit(max(p.wait() for p in ps))
sys.path.insert(0, os.environ["BENCH_ROOT"])
import bench
r = int(sys.argv[2])
bench.stage_marker("start")
bench.stage_marker("comm_init")
if mode == "ok":
    sys.exit(0)
if mode == "fail":
    sys.exit(3 if r == 1 else 0)
if r == 0:
    bench.stage_marker("timed_loop")
time.sleep(600)  # hang (the parent kills it)
"""


@pytest.mark.parametrize("mode,rc,status", [("ok", 0, None), ("fail", 3, "failed"),
                                            ("hang", 124, "timeout")])
def test_parent_timeout_and_stage_report(tmp_path, capsys, monkeypatch, mode, rc, status):
    """run_parent on a stub child: a clean child passes its status through silently; a
    failing or hung child is killed (its process group and every rank pid) and the parent
    prints ONE JSON line naming the last stage each rank reached."""
    import json
    import time
    stub = tmp_path / "stub.py"
    stub.write_text(_STUB)
    monkeypatch.setenv("BENCH_ROOT", ROOT)
    t = time.time()
    got = bench.run_parent([], 2, 5.0, cmd=[sys.executable, str(stub), mode])
    assert got == rc
    assert time.time() - t < 60
    out = capsys.readouterr().out.strip()
    if status is None:
        assert out == ""
        return
    line = json.loads(out.splitlines()[-1])
    assert line["status"] == status and line["n_gpus"] == 2 and line["value"] is None
    assert line["metric"] == bench.METRIC
    st = line["last_stage"]
    if mode == "hang":
        assert st["0"]["stage"] == "timed_loop" and st["1"]["stage"] == "comm_init"
        assert line["ranks_reporting"] == 2
    else:
        assert st["1"]["stage"] == "comm_init"
    for r in st.values():
        assert "pid" not in r


def test_rank_does_not_relaunch(monkeypatch):
    """Inside torch.distributed.run (WORLD_SIZE set) the launcher branch is skipped."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: pytest.fail("relaunched"))
    # stop right after the launcher decision: the first thing a rank does is the gloo group
    import torch.distributed as tdist
    monkeypatch.setattr(tdist, "init_process_group", lambda *a, **k: (_ for _ in ()).throw(
        RuntimeError("rank path reached")))
    with pytest.raises(RuntimeError, match="rank path reached"):
        bench.main()


def test_host_info():
    h = bench.host_info()
    assert h["nproc"] >= 1 and h["allowed_cpus"] >= 1


def test_parent_never_kills_a_reused_pid(tmp_path, capsys, monkeypatch):
    """a rank pid in the markers is killed only while it still names the same
    process (start time from /proc/PID/stat); a process that reuses the pid survives."""
    import subprocess
    assert bench.proc_start(os.getpid()) != ""
    sleeper = subprocess.Popen(["sleep", "60"])
    try:
        stub = tmp_path / "stub.py"
        stub.write_text(_STUB)
        monkeypatch.setenv("BENCH_ROOT", ROOT)
        monkeypatch.setenv("FAKE_PID", str(sleeper.pid))
        assert bench.run_parent([], 2, 5.0, cmd=[sys.executable, str(stub), "fail"]) == 3
        line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
        assert line["status"] == "failed" and "9" in line["last_stage"]
        assert sleeper.poll() is None  # alive: its start time is not the recorded one
    finally:
        sleeper.kill()
        sleeper.wait()


def test_prediction_and_roofline_blocks(tmp_path, monkeypatch):
    """The N > 1 line's `predicted` block and the N = 1 line's predicted curve come from
    the committed rank shares with the stated model (ms_1rank + (3k - 1) L); the roofline
    names the kernel with the larger live time share and carries both SpMVs."""
    rs = {"k": 500, "shares": {"8": {"rank0_rows": 10, "rank0_nnz": 20,
                                     "one_rank_replicated": {"ms_per_solve": 15.0, "steps": 500,
                                                             "pass1_us_per_step": 20.0,
                                                             "pass2_us_per_step": 10.0},
                                     "single_gpu": {"ms_per_solve": 11.0},
                                     "collectives_per_step": {"pass1": 2, "pass2": 1},
                                     "collectives_per_solve": 1499}}}
    f = tmp_path / "rank_share.json"
    f.write_text(json.dumps(rs))
    monkeypatch.setattr(bench, "RANK_SHARE_FILE", str(f))
    p = bench.predicted_block(8, 500, 500, 0.030)
    assert p["source"].startswith(str(f)) or "rank_share.json" in p["source"]
    assert p["ms_at_L_us"]["10"] == round(15.0 + 14.99, 3)
    assert p["implied_L_us"] == round((30.0 - 15.0) * 1000.0 / 1499, 2)
    assert bench.predicted_block(4, 500, 500, 0.03) is None  # no share for N = 4
    assert "error" in bench.predicted_block(8, 400, 400, 0.03)
    c = bench.predicted_curve(500, 66.0)
    assert c["N"]["8"]["L10us"]["speedup"] == round(66.0 / (15.0 + 14.99), 2)
    # every rank's share measured: the solve waits for the slowest
    rs["shares"]["8"]["ms_per_solve_every_rank"] = [15.0, 16.5, 14.0]
    f.write_text(json.dumps(rs))
    p = bench.predicted_block(8, 500, 500, 0.030)
    assert p["ms_1rank"] == 16.5 and p["ms_at_L_us"]["10"] == round(16.5 + 14.99, 3)
    assert bench.predicted_curve(500, 66.0)["N"]["8"]["ms_1rank_share"] == 16.5
    r = bench.roofline_block(34e6, 40e6, 6.3, 6.5, 4.6, 8, 500, 11.1, 8.8e-3, 22e6, "p2",
                             {"k_p1_spmv": 19e6, "k_p1_axpy": 12e6}, "p1", {}, False)
    assert r["kernel"] == "k_p1_spmv" and r["avg_launch_us_events"] == 6.5
    assert r["frac"] == round(34e6 / 6.5e-6 / 1e9 / 8000.0, 4)
    assert r["frac_counter_bytes"] == round(19e6 / 6.5e-6 / 1e9 / 8000.0, 4)
    assert set(r["kernels"]) == {"k_p1_spmv", "k_p2_spmv", "k_p1_axpy"}
    r2 = bench.roofline_block(34e6, 40e6, 6.3, None, None, 0, 500, 11.1, 8.8e-3, None, None,
                              None, None, {}, True)
    assert r2["kernel"].startswith("k_p2_spmv") and "all_spmv_time_weighted_frac" not in r2


def test_multi_line():
    """N > 1: `value` is the partitioned headline (strong scaling of the N = 1 workload);
    configs[4] partitioned and the replicas ride along as sub-blocks, and the parity block
    covers every workload checked."""
    import argparse
    head = {"value": 90000.0, "unit": "Lanczos iterations/s", "ms_per_step": 5.5,
            "ms_per_solve_median": 5.5, "data": "netgen 500000-arc",
            "config": {"workload": "500k partitioned"}, "roofline": {"kernel": "k_p2_spmv"},
            "predicted": {"implied_L_us": 10.0}, "exchange": {"comm_frac": 0.5},
            "parity": {"configs2_replicated_N4": {"ok": True}}}
    args = argparse.Namespace(steps=5, warmup=1, k=500)
    line = bench.multi_line(head, 4, args)
    assert line["value"] == 90000.0 and line["scaling"] == "strong" and line["n_gpus"] == 4
    assert line["metric"] == bench.METRIC and line["status"] == "ok"
    assert line["predicted"]["implied_L_us"] == 10.0
    assert line["parity"]["all_ok"] and line["parity"]["checked"] == 1
    head["parity"]["configs2_replicated_N4"]["ok"] = False
    assert not bench.multi_line(head, 4, args)["parity"]["all_ok"]
    # a later phase that failed keeps the value, names the phase, and fails the parity
    line = bench.sub_phase_failed(bench.multi_line(dict(head, parity={"a": {"ok": True}}), 4,
                                                   args), "partitioned_configs4", "failed", "x")
    assert line["value"] == 90000.0 and line["partitioned_configs4"]["status"] == "failed"
    assert line["status"] == "partitioned_configs4: failed" and not line["parity"]["all_ok"]
    assert bench.failed_line(4, "failed", "x")["value"] is None


_RANK = r"""
import json, os, sys, time
sys.path.insert(0, os.environ["BENCH_ROOT"])
import bench, argparse
mode = sys.argv[1]
args = argparse.Namespace(steps=5, warmup=1, k=500, rank_timeout=1.0)
def fake_main():
    bench.stage_marker("partitioned 500000: timed_loop")
    if mode.endswith("late"):  # the headline was measured; a later phase fails / hangs
        bench._PROGRESS["line"] = bench.multi_line(
            {"value": 90000.0, "ms_per_step": 5.5, "parity": {"configs2_replicated_N2": {"ok": True}}},
            2, args)
        bench._PROGRESS["phase"] = "partitioned_configs4"
        bench.stage_marker("partitioned 5000000: first_solve (graph capture)")
    if mode.startswith("hang"):
        time.sleep(30)  # a hung collective
    raise RuntimeError("rank 1 lost")
bench.main = fake_main
bench.parse = lambda argv=None: args
bench.run()
"""


@pytest.mark.parametrize("mode,rc,value", [("fail", 1, None), ("hang", 124, None),
                                           ("fail_late", 0, 90000.0),
                                           ("hang_late", 0, 90000.0)])
def test_rank_failure_lines(mode, rc, value):
    """N > 1 under the driver's torchrun (bench.run on rank 0): a partitioned headline that
    raises or hangs prints a line with NO value and exits non-zero; a
    later phase that raises or hangs leaves the measured value and names the phase."""
    import subprocess
    t = time.time()
    p = subprocess.run([sys.executable, "-c", _RANK, mode], capture_output=True, text=True,
                       timeout=60, env=dict(os.environ, BENCH_ROOT=ROOT, WORLD_SIZE="2", RANK="0"))
    assert p.returncode == rc, p.stderr[-2000:]
    assert time.time() - t < 25
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] == value and line["metric"] == bench.METRIC
    if value is None:
        assert line["status"] == ("failed" if mode == "fail" else "timeout")
        assert line["last_stage_rank0"] == "partitioned 500000: timed_loop"
    else:
        pc = line["partitioned_configs4"]
        assert pc["status"] == ("failed" if mode == "fail_late" else "timeout")
        assert pc["last_stage_rank0"].startswith("partitioned 5000000")
        assert line["parity"]["all_ok"] is False and line["scaling"] == "strong"


def test_cpu_threads_allowed(monkeypatch):
    """The all-cores CPU baseline's thread count: the affinity mask, capped by the cgroup
    quota and OMP_NUM_THREADS (a GPU box's mask shows the whole machine)."""
    n = bench.cpu_threads_allowed()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.cpu_threads_allowed() == 1
