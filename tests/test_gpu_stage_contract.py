"""The batched vector stages (one device call per stage, stage_io.run_image_stage) against the
reference's own stage functions: every scenario of tests/stage_scenarios.py -- pre-existing
outputs, overwrite, inputs np.load refuses (3-D, junk, truncated), failing coefficient sets (in
the first image or only later, after an image with no rows), empty images, non-uint8 and
Fortran-order inputs, other bit widths, mixed tap lengths, ten images of widths 1..100000 --
must leave exactly the files the reference left (SHA-256 of each .npy) and return or raise
exactly what it did (tests/golden/stage_contract.json, recorded by make_stage_contract.py from
fir_1d/sim/vector/gen_fixed_output.py:70-107 and gen_ideal_output.py:60-88).  Also the
image-batch C entries directly (fir1d_fixed_images_multi / fir1d_ideal_images_multi) against
the C oracle, with page-locked and pageable planes, and the stage's timing breakdown."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

import fir_hip
import stage_scenarios as S
from fir_1d.sim.vector import gen_fixed_output as gf
from fir_1d.sim.vector import gen_ideal_output as gi
from oracle import c_oracle

pytestmark = pytest.mark.gpu
CONTRACT = json.loads((Path(__file__).resolve().parent / "golden" / "stage_contract.json").read_text())
BY_NAME = {r["name"]: r for r in CONTRACT["scenarios"]}


@pytest.mark.parametrize("batch_bytes", [1 << 30, 4096])
@pytest.mark.parametrize("scn", S.SCENARIOS, ids=[s["name"] for s in S.SCENARIOS])
def test_stage_matches_reference_outcome(scn, batch_bytes, tmp_path, monkeypatch):
    """One device call per stage, and (4096-byte windows) one per image or two."""
    from fir_1d.sim.vector import stage_io

    monkeypatch.setattr(stage_io, "BATCH_BYTES", batch_bytes)
    got = S.run(scn, tmp_path, gf._generate_fixed_outputs_for_tap_map, gi._generate_ideal_outputs_for_tap_map)
    want = BY_NAME[scn["name"]]
    assert got["error"] == want["error"]
    assert got["returned"] == want["returned"]
    assert got["files"] == want["files"]


def test_stage_timings_breakdown(tmp_path):
    scn = next(s for s in S.SCENARIOS if s["name"] == "fixed_ten_images")
    inp, out = S.build(scn, tmp_path)
    t: dict = {}
    n = gf.generate_fixed_3tap_output_vector(input_dir=inp, output_dir=out, timings=t)
    assert n == 40 and t["files"] == 40 and t["device_calls"] == 1
    for k in ("plan_ms", "load_ms", "h2d_ms", "kernel_ms", "d2h_ms", "call_ms", "save_write_ms", "save_tail_ms",
              "wall_ms"):
        assert t[k] >= 0.0, k
    assert t["call_ms"] <= t["wall_ms"]
    t2: dict = {}
    assert gi.generate_ideal_5tap_output_vector(input_dir=inp, output_dir=out, timings=t2) == 40
    assert t2["device_calls"] == 1


def _rand_images(rng, shapes, dtype=np.uint8):
    if dtype == np.uint8:
        return [rng.integers(0, 256, s, dtype=np.uint8) for s in shapes]
    return [rng.integers(-32768, 32768, s, dtype=np.int16) for s in shapes]


SHAPES = [(1, 1), (3, 17), (9, 4499), (16, 16), (5, 640), (0, 7), (2, 0), (64, 64), (2, 4096), (1, 100003),
          (33, 4496)]


@pytest.mark.parametrize("pinned", [True, False])
def test_fixed_images_multi_host_entry_vs_oracle(pinned):
    co = c_oracle()
    rng = np.random.default_rng(5)
    xs = _rand_images(rng, SHAPES)
    bank = np.array([[1365] * 3, [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512], [7, -3, 9]])
    outs = None
    if pinned:
        outs = [[fir_hip.host_empty(max(1, x.size))[:x.size].reshape(x.shape) for _ in bank] for x in xs]
    seen = []
    got = fir_hip.fir1d_fixed_images_multi(xs, bank, 12, 32, fir_hip.OUT_U8_SAT, outs=outs,
                                           ready=lambda i, f: seen.append((i, f)))
    sizes = [xs[i].size for i, _ in seen]
    assert sorted(seen) == [(i, f) for i in range(len(xs)) for f in range(len(bank))]  # each plane once
    assert sizes == sorted(sizes, reverse=True)  # largest planes first
    for x, planes in zip(xs, got):
        for h, y in zip(bank, planes):
            ref = co.fir1d_rows(x, h, 12, 32, co.OUT_U8_SAT) if x.size else np.zeros(x.shape, np.uint8)
            assert np.array_equal(y, ref)


def test_fixed_images_multi_int16_complex_vs_oracle():
    co = c_oracle()
    rng = np.random.default_rng(6)
    xs = _rand_images(rng, [(3, 34), (1, 1 << 16), (7, 2 * 4499)], np.int16)
    bank = np.array([[-256, -1024, 6656, -1024, -256], [32767, -32768, 32767, -32768, 32767]])
    t: dict = {}
    got = fir_hip.fir1d_fixed_images_multi(xs, bank, 12, 32, fir_hip.OUT_I32, channels=2, timing=t)
    assert set(t) == set(fir_hip.TIMING_KEYS)
    for x, planes in zip(xs, got):
        for h, y in zip(bank, planes):
            assert np.array_equal(y, co.fir1d_rows(x, h, 12, 32, co.OUT_I32, channels=2))
    with pytest.raises(fir_hip.FirHipError, match="multiple of channels"):
        fir_hip.fir1d_fixed_images_multi([np.zeros((2, 5), np.int16)], bank, channels=2)


def test_ideal_images_multi_host_entry_vs_oracle():
    co = c_oracle()
    rng = np.random.default_rng(7)
    xs = _rand_images(rng, SHAPES)
    hs = [[1 / 16, 4 / 16, 6 / 16, 4 / 16, 1 / 16], [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16],
          [0.1, -0.2, 0.3, -0.4, 0.5]]
    got = fir_hip.fir1d_ideal_images_multi(xs, hs)
    for x, planes in zip(xs, got):
        for h, y in zip(hs, planes):
            ref = co.fir1d_ideal_rows(x, h) if x.size else np.zeros(x.shape)
            assert np.array_equal(y.view(np.uint64), ref.view(np.uint64))


def test_ready_callback_error_is_raised_after_the_call():
    xs = [np.zeros((2, 16), np.uint8)] * 3

    def boom(i, f):
        if i == 1:
            raise RuntimeError("stop at image 1")

    with pytest.raises(RuntimeError, match="stop at image 1"):
        fir_hip.fir1d_fixed_images_multi(xs, [[1, 2, 1]], ready=boom)
