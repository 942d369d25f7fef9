"""The comparison report (fir_1d/sim/vector/gen_compare_report.py) against the REFERENCE's report
functions on every scenario of tests/report_scenarios.py (tests/golden/report_contract.json, made
by tests/golden/make_report_contract.py): the returned dict or the exception's type and text, the
CSV text and the summary JSON must be the reference's.  On the CPU the per-case metrics come from
the oracle (oracle/fir_oracle.compute_metrics, pinned to the reference's _compute_metrics by
tests/test_oracle_golden.py) standing in for the GPU reduction; tests/test_gpu_report_contract.py
runs the same scenarios on the GPU."""
from __future__ import annotations

import contextlib
import io
import json
from pathlib import Path

import pytest

import report_scenarios as S

CONTRACT = json.loads((Path(__file__).resolve().parent / "golden" / "report_contract.json").read_text())
BY_NAME = {r["name"]: r for r in CONTRACT["scenarios"]}


def report_fn(tap):
    from fir_1d.sim.vector.gen_3tap_compare_report import generate_3tap_compare_report
    from fir_1d.sim.vector.gen_5tap_compare_report import generate_5tap_compare_report

    return generate_5tap_compare_report if tap == "5tap" else generate_3tap_compare_report


def check(scn, tmp_path):
    with contextlib.redirect_stdout(io.StringIO()):
        got = S.run(scn, tmp_path, report_fn(scn.get("tap", "3tap")))
    want = BY_NAME[scn["name"]]
    assert got["error"] == want["error"]
    assert got["returned"] == want["returned"]
    assert got["csv"] == want["csv"]
    assert got["json"] == want["json"]


def test_every_scenario_has_a_reference_record():
    assert sorted(BY_NAME) == sorted(s["name"] for s in S.SCENARIOS)


@pytest.mark.parametrize("batch_bytes", [1 << 30, 4096])
@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_report_matches_reference_with_oracle_metrics(scn, batch_bytes, tmp_path, monkeypatch):
    """4096-byte windows: each plain pair read in a window of its own."""
    import fir_hip
    from fir_1d.sim.vector import stage_io
    from oracle import fir_oracle as fo

    monkeypatch.setattr(stage_io, "BATCH_BYTES", batch_bytes)

    def metrics(y_ideal, y_fixed, device=0):
        if y_ideal.shape != y_fixed.shape:
            raise ValueError(f"Shape mismatch: ideal={y_ideal.shape}, fixed={y_fixed.shape}")
        return fo.compute_metrics(y_ideal, y_fixed)

    monkeypatch.setattr(fir_hip, "compare_metrics", metrics)
    check(scn, tmp_path)
