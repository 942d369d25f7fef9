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


def _oracle_batches(monkeypatch):
    """The two image-batch C entries replaced by the oracle (same signatures, planes delivered
    largest first through ``ready``): every scenario then runs on the CPU through the product's
    stage driver -- planning, skip / error order, page-locked staging fallback, windows, ordered
    concurrent writes -- with only the device call stood in for."""
    import numpy as np

    import fir_hip
    from oracle import fir_oracle as fo

    def deliver(xs, outs, nf, ready, timing):
        order = sorted(((i, f) for i in range(len(xs)) for f in range(nf)), key=lambda p: -xs[p[0]].size)
        for i, f in order:
            if ready is not None:
                ready(i, f)
        if timing is not None:
            timing.update({k: 0.0 for k in fir_hip.TIMING_KEYS})
        return outs

    def fixed(xs, hq2, frac_bits=12, acc_bits=32, out_stage=0, channels=1, device=0, outs=None, ready=None,
              timing=None):
        h2 = np.asarray(hq2, dtype=np.int64)
        for x, planes in zip(xs, outs):
            for h, y in zip(h2, planes):
                y[...] = fo.fir1d_rows(x, h, frac_bits, acc_bits, fo.OUT_U8_SAT)
        return deliver(xs, outs, len(h2), ready, timing)

    def ideal(xs, hs, device=0, outs=None, ready=None, timing=None):
        for x, planes in zip(xs, outs):
            for h, y in zip(hs, planes):
                y[...] = fo.fir1d_ideal_rows(x, h)
        return deliver(xs, outs, len(hs), ready, timing)

    monkeypatch.setattr(fir_hip, "fir1d_fixed_images_multi", fixed)
    monkeypatch.setattr(fir_hip, "fir1d_ideal_images_multi", ideal)


@pytest.mark.parametrize("batch_bytes,read_chunk", [(1 << 30, 4 << 20), (4096, 4 << 20), (1 << 30, 1000)])
@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_stage_driver_matches_reference_with_oracle_compute(scn, batch_bytes, read_chunk, tmp_path, monkeypatch):
    """Every scenario through the product's stage driver with the device call replaced by the
    oracle: the reference's return value, exception text and every file's SHA-256.  4096-byte
    windows split each stage into one device call per image or two (stage_io.BATCH_BYTES);
    1000-byte read pieces read every larger input in several parallel pieces (stage_io.READ_CHUNK)."""
    from fir_1d.sim.vector import stage_io

    _oracle_batches(monkeypatch)
    monkeypatch.setattr(stage_io, "BATCH_BYTES", batch_bytes)
    monkeypatch.setattr(stage_io, "READ_CHUNK", read_chunk)
    got = S.run(scn, tmp_path, gf._generate_fixed_outputs_for_tap_map, gi._generate_ideal_outputs_for_tap_map)
    want = BY_NAME[scn["name"]]
    assert (got["returned"], got["error"], got["files"]) == (want["returned"], want["error"], want["files"])
    assert not list((tmp_path / "output").rglob(".*.part"))  # no temporary file left behind


def test_device_error_in_a_later_window_keeps_the_earlier_windows(tmp_path, monkeypatch):
    """A device call that fails in window 3 of a pipelined stage (the next window's reads and the
    previous window's writes run under each call): the outputs of the windows before it are put
    in place -- the reference's files for those images -- the failing window's planes are not, no
    temporary file is left, and the device error is raised."""
    import fir_hip
    from fir_1d.sim.vector import stage_io

    _oracle_batches(monkeypatch)
    good = fir_hip.fir1d_fixed_images_multi
    calls = []

    def failing(xs, *a, **kw):
        calls.append(len(xs))
        if len(calls) == 3:
            raise fir_hip.FirHipError("injected device failure")
        return good(xs, *a, **kw)

    monkeypatch.setattr(fir_hip, "fir1d_fixed_images_multi", failing)
    monkeypatch.setattr(stage_io, "BATCH_BYTES", 4096)  # one image per window
    scn = next(s for s in S.SCENARIOS if s["name"] == "fixed_ten_images")
    got = S.run(scn, tmp_path, gf._generate_fixed_outputs_for_tap_map, gi._generate_ideal_outputs_for_tap_map)
    assert got["error"] == ["FirHipError", "injected device failure"]
    want = BY_NAME["fixed_ten_images"]["files"]
    nsets = len(want) // 10
    first_two = dict(sorted(want.items())[:2 * nsets])  # the images of windows 1 and 2
    assert got["files"] == first_two
    assert not list((tmp_path / "output").rglob(".*.part"))
