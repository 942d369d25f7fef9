"""CPU side of the stage contract (tests/golden/stage_contract.json, recorded from the
reference's stage functions by tests/golden/make_stage_contract.py): every scenario has a
record, and the scenarios whose outcome needs no device work -- every output already present,
a coefficient set that fails before the first image is computed -- give the reference's exact
outcome here.  The rest run on the GPU (tests/test_gpu_stage_contract.py)."""
from __future__ import annotations

import json
from pathlib import Path

import pytest

import stage_scenarios as S
from fir_1d.sim.vector import gen_fixed_output as gf
from fir_1d.sim.vector import gen_ideal_output as gi

CONTRACT = json.loads((Path(__file__).resolve().parent / "golden" / "stage_contract.json").read_text())
BY_NAME = {r["name"]: r for r in CONTRACT["scenarios"]}


def test_every_scenario_has_a_reference_record():
    assert sorted(BY_NAME) == sorted(s["name"] for s in S.SCENARIOS)


@pytest.mark.parametrize("name", ["fixed_all_exist", "fixed_q_range_error"])
def test_device_free_scenarios_match_reference(name, tmp_path):
    scn = next(s for s in S.SCENARIOS if s["name"] == name)
    got = S.run(scn, tmp_path, gf._generate_fixed_outputs_for_tap_map, gi._generate_ideal_outputs_for_tap_map)
    want = BY_NAME[name]
    assert (got["returned"], got["error"], got["files"]) == (want["returned"], want["error"], want["files"])
