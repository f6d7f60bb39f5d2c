"""The experiment harness (tpl_amd.harness) — the reference binaries' callers of the
path — on the GPU, against the reference's published CSVs (results/*.csv, copied under
tests/golden/reference_results)."""
import csv
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "two-pass-lanczos_amd"))

from conftest import REF_RESULTS  # noqa: E402

pytestmark = pytest.mark.gpu


def _published(name):
    with open(os.path.join(REF_RESULTS, name)) as f:
        return {int(r["k"]): r for r in csv.DictReader(f)}


def test_accuracy_rows_match_published():
    from tpl_amd import harness
    rows = harness.accuracy("inv", "well-conditioned", k_min=10, k_max=80, k_step=10)
    pub = _published("accuracy_inv_well-conditioned.csv")
    assert [r["k"] for r in rows] == list(range(10, 81, 10))
    for r in rows:
        ref = float(pub[r["k"]]["relative_error_standard"])
        assert abs(r["relative_error_standard"] - ref) <= 1e-9 * max(ref, 1e-300) + 1e-13
        assert abs(r["relative_error_two_pass"] - ref) <= 1e-9 * max(ref, 1e-300) + 1e-13
        assert r["relative_solution_deviation"] < 1e-13


def test_orthogonality_rows_match_published():
    from tpl_amd import harness
    rows = harness.orthogonality("inv", "well-conditioned", k_min=20, k_max=100, k_step=20)
    pub = _published("orthogonality_inv_well-conditioned.csv")
    for r in rows:
        assert r["basis_drift_fro"] == 0.0 and r["solution_deviation_l2"] == 0.0
        ref = float(pub[r["k"]]["ortho_loss_standard"])
        assert ref / 3 <= r["ortho_loss_standard"] <= 3 * ref
        assert r["ortho_loss_regenerated"] == r["ortho_loss_standard"]


def test_tradeoff_schema_and_memory_tradeoff(tmp_path):
    """src/bin/tradeoff.rs: one fresh worker per variant, rows grouped by variant (the
    orchestrator appends each worker's output), k ascending; the device column shows the
    reference's trade-off — the standard variant holds V_k (8 n k bytes), the two-pass
    variant's footprint does not grow with k."""
    from tpl_amd import harness
    out = str(tmp_path / "t.csv")
    harness.main(["tradeoff", "--arcs", "5000", "--k-start", "50", "--k-end", "150",
                  "--k-step", "50", "--output", out])
    with open(out) as f:
        rows = list(csv.DictReader(f))
    assert list(rows[0].keys()) == ["variant", "k", "time_s", "rss_kb", "device_kb"]
    assert [(r["variant"], int(r["k"])) for r in rows] == [
        ("standard", 50), ("standard", 100), ("standard", 150),
        ("two-pass", 50), ("two-pass", 100), ("two-pass", 150)]
    assert all(float(r["time_s"]) > 0 and int(r["rss_kb"]) > 0 for r in rows)
    dev = {(r["variant"], int(r["k"])): int(r["device_kb"]) for r in rows}
    n = 5115
    for k in (50, 100, 150):
        basis_kb = 8 * n * k // 1024
        assert dev[("standard", k)] - dev[("two-pass", k)] >= basis_kb - 64
    # two-pass: only the k-sized solver state grows (a few KB)
    assert dev[("two-pass", 150)] - dev[("two-pass", 50)] < 64


def test_scalability_rows(tmp_path):
    """src/bin/scalability.rs schema, fresh worker per variant, two instances."""
    from tpl_amd import harness
    out = str(tmp_path / "s.csv")
    harness.main(["scalability", "--arcs", "5000", "50000", "--k", "100", "--output", out])
    with open(out) as f:
        rows = list(csv.DictReader(f))
    assert list(rows[0].keys()) == ["variant", "n", "k", "time_s", "rss_kb", "device_kb"]
    assert [(r["variant"], int(r["n"])) for r in rows] == [
        ("standard", 5115), ("standard", 50365), ("two-pass", 5115), ("two-pass", 50365)]
    d = {(r["variant"], int(r["n"])): int(r["device_kb"]) for r in rows}
    assert d[("standard", 50365)] - d[("two-pass", 50365)] >= 8 * 50365 * 100 // 1024 - 64
