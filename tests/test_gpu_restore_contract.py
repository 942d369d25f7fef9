"""The image restore stage with the GPU u8 conversions against the REFERENCE's restore_images on
every scenario of tests/restore_scenarios.py (tests/golden/restore_contract.json): returned summary
or exception, and every file left in the image tree (PNG bytes and pixels) equal."""
from __future__ import annotations

import pytest

import restore_scenarios as S
from test_restore_contract import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_restore_matches_reference(scn, tmp_path):
    check(scn, tmp_path)
