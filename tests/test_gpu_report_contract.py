"""The comparison report with the GPU metrics reduction against the REFERENCE's report functions
on every scenario of tests/report_scenarios.py (tests/golden/report_contract.json): returned dict
or exception, CSV text and summary JSON equal -- every metric bit-identical, since the JSON holds
them at full precision.  Whole-report and per-pair read windows."""
from __future__ import annotations

import pytest

import report_scenarios as S
from test_report_contract import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch_bytes", [1 << 30, 4096])
@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_report_matches_reference(scn, batch_bytes, tmp_path, monkeypatch):
    from fir_1d.sim.vector import stage_io

    monkeypatch.setattr(stage_io, "BATCH_BYTES", batch_bytes)
    check(scn, tmp_path)
