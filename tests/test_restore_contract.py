"""The image restore stage (fir_1d/sim/vector/restore_images.py) against the REFERENCE's
restore_images on every scenario of tests/restore_scenarios.py (tests/golden/restore_contract.json,
made by tests/golden/make_restore_contract.py): the returned summary or the exception's type and
text, and every file the stage leaves in the image tree -- PNG bytes, decoded mode, size and
pixels -- must be the reference's.  On the CPU the u8 conversions come from the oracle
(oracle/fir_oracle.to_u8_clip / to_u8_normalized, pinned to the reference's conversions by
tests/test_oracle_golden.py) standing in for the GPU kernel; tests/test_gpu_restore_contract.py runs
the same scenarios on the GPU."""
from __future__ import annotations

import json
from pathlib import Path

import pytest

import restore_scenarios as S

CONTRACT = json.loads((Path(__file__).resolve().parent / "golden" / "restore_contract.json").read_text())
BY_NAME = {r["name"]: r for r in CONTRACT["scenarios"]}


def check(scn, tmp_path):
    from fir_1d.sim.vector.restore_images import restore_images

    got = S.run(scn, tmp_path, restore_images)
    want = BY_NAME[scn["name"]]
    assert got["error"] == want["error"]
    assert got["returned"] == want["returned"]
    assert got["images"] == want["images"]


def test_every_scenario_has_a_reference_record():
    assert sorted(BY_NAME) == sorted(s["name"] for s in S.SCENARIOS)


@pytest.mark.parametrize("workers,inflight", [(1, 1 << 30), (3, 1 << 30), (3, 64)])
@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_restore_matches_reference_with_oracle_conversions(scn, workers, inflight, tmp_path, monkeypatch):
    """inflight = 64 pixels: every image waits for the ones before it to be written and committed
    (the memory bound of a long restore)."""
    import numpy as np

    import fir_hip
    from fir_1d.sim.vector import restore_images as ri
    from oracle import fir_oracle as fo

    monkeypatch.setattr(ri, "INFLIGHT_BYTES", inflight)

    def restore_u8(a, policy=fir_hip.RESTORE_CLIP, device=0):
        arr = np.ascontiguousarray(a, dtype=np.float64)
        if policy == fir_hip.RESTORE_NORMALIZE:
            return fo.to_u8_normalized(arr)
        return fo.to_u8_clip(arr)

    monkeypatch.setattr(fir_hip, "restore_u8", restore_u8)
    monkeypatch.setenv("FIR_RESTORE_WRITERS", str(workers))
    check(scn, tmp_path)
