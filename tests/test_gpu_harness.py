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


def test_tradeoff_schema(tmp_path):
    from tpl_amd import harness
    out = str(tmp_path / "t.csv")
    harness.main(["tradeoff", "--arcs", "5000", "--k-start", "50", "--k-end", "100",
                  "--k-step", "50", "--output", out])
    with open(out) as f:
        rows = list(csv.DictReader(f))
    assert list(rows[0].keys()) == ["variant", "k", "time_s", "rss_kb"]
    assert [(r["variant"], int(r["k"])) for r in rows] == [
        ("standard", 50), ("two-pass", 50), ("standard", 100), ("two-pass", 100)]
    assert all(float(r["time_s"]) > 0 for r in rows)
