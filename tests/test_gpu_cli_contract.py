"""The vector stages as programs, on the GPU, against the REFERENCE's programs on every scenario of
tests/cli_scenarios.py (tests/golden/cli_contract.json): printed lines, exit status, exceptions and
every file left equal."""
from __future__ import annotations

import pytest

import cli_scenarios as S
from test_cli_contract import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_programs_match_reference(scn, tmp_path):
    check(scn, tmp_path)
