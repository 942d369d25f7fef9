"""Host-side logic of the fir_1d mirror: validation order and ValueError texts, exactly as
the reference raises them (pinned by the error records of tests/golden/kat_*.json, which
hold the reference's own messages), plus coefficient quantization.  No GPU needed: every
case here raises before the device call or touches no device.

Mirrors the error tests of the reference's fir_1d/sim/tests/test_1d_fixed.py:43-92 and
test_1d_ideal.py:45-69.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import iter_ragged, load_kats
from fir_1d.model.python.fir_1d_fixed_ref import device_bits, fir_1d_fixed_golden, quantize_fixed_taps
from fir_1d.model.python.fir_1d_ref import MAX_ABS_H_COEFF, _prepare_x_u8, fir_1d_ideal
from oracle import fir_oracle as fo


@pytest.mark.parametrize("rec", [r for r in load_kats("fixed") if "error" in r], ids=lambda r: r["message"][:40])
def test_fixed_error_records_match_reference_text(rec):
    with pytest.raises(ValueError) as ei:
        fir_1d_fixed_golden(rec["x"], rec["h"], **rec["kwargs"])
    assert rec["error"] == "ValueError"
    assert str(ei.value) == rec["message"]


@pytest.mark.parametrize("rec", [r for r in load_kats("ideal") if "error" in r], ids=lambda r: r["message"][:40])
def test_ideal_error_records_match_reference_text(rec):
    with pytest.raises(ValueError) as ei:
        fir_1d_ideal(rec["x"], rec["h"])
    assert str(ei.value) == rec["message"]


@pytest.mark.parametrize("bad_x", [float("nan"), float("inf"), float("-inf")])
def test_non_finite_x_raises_value_error(bad_x):
    with pytest.raises(ValueError, match=r"x\[1\].*finite"):
        fir_1d_fixed_golden([10, bad_x, 20], [0.5])
    with pytest.raises(ValueError, match=r"x\[1\].*finite"):
        fir_1d_fixed_golden(np.array([10, bad_x, 20]), [0.5])


@pytest.mark.parametrize("bad_h", [float("nan"), float("inf"), float("-inf")])
def test_non_finite_h_raises_value_error(bad_h):
    with pytest.raises(ValueError, match=r"h\[0\].*finite"):
        fir_1d_fixed_golden([10, 20], [bad_h])


def test_empty_h_and_bad_bits():
    with pytest.raises(ValueError, match="must not be empty"):
        fir_1d_fixed_golden([10, 20], [])
    with pytest.raises(ValueError, match="Invalid coeff_bits=12"):
        fir_1d_fixed_golden([10, 20], [0.5], coeff_bits=12)
    for f, a in ((0, 32), (-1, 32), (12, 0), (12, -1)):
        with pytest.raises(ValueError):
            fir_1d_fixed_golden([10, 20], [0.5], frac_bits=f, acc_bits=a)


def test_q_range_errors():
    with pytest.raises(ValueError, match="out of Q-format real range"):
        fir_1d_fixed_golden([10, 20], [8.0])
    with pytest.raises(ValueError, match="out of Q-format real range"):
        fir_1d_fixed_golden([10, 20], [1.0], frac_bits=7, coeff_bits=8)
    with pytest.raises(ValueError, match=r"\|h\| must be <="):
        fir_1d_ideal([10, 20, 30], [MAX_ABS_H_COEFF + 1e-6])


def test_empty_x_returns_empty_without_device():
    y = fir_1d_fixed_golden([], [0.5, 0.25])
    assert isinstance(y, np.ndarray) and y.dtype == np.uint8 and y.size == 0
    assert fir_1d_ideal([], [1.0, 2.0]) == []


def test_input_prep_matches_oracle():
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-40, 300, 5000), np.arange(-3, 260) + 0.5, [0.49999999, 254.5, 255.5]])
    assert np.array_equal(_prepare_x_u8(x), fo.prep_x(x))
    assert np.array_equal(_prepare_x_u8(x.tolist()), fo.prep_x(x))
    xi = rng.integers(-1000, 1000, 100)
    assert np.array_equal(_prepare_x_u8(xi.tolist()), np.clip(xi, 0, 255).astype(np.uint8))
    # the u8-range int list fast path (bytearray) and everything it must hand to the general path
    xb = rng.integers(0, 256, 4499)
    for lst in (xb.tolist(), tuple(xb.tolist()), list(xb.astype(np.uint8)), [True, False, 0, 255],
                xb.tolist() + [256], [-1] + xb.tolist(), xb.tolist() + [3.5], [255.49, 7], []):
        got = _prepare_x_u8(lst)
        assert got.dtype == np.uint8 and got.flags.writeable
        assert np.array_equal(got, fo.prep_x(np.asarray(lst, dtype=np.float64))), lst[:4]
    with pytest.raises(ValueError, match=r"Invalid x\[2\]=nan: x must be finite"):
        _prepare_x_u8([1, 2, float("nan")])


def test_quantization_matches_oracle_on_random_sweep():
    n = 0
    for _x, h, (f, a, c), _y in iter_ragged("fixed"):
        hq = quantize_fixed_taps(h.tolist(), f, a, c)
        assert hq.dtype == np.int32
        assert np.array_equal(hq, fo.quantize_h(h, f, c))
        n += 1
    assert n == 3000


def test_device_bits_clamp_is_result_preserving():
    acc = np.array([-(1 << 63), -(1 << 62) - 1, -(1 << 51), -5, -1, 0, 7, (1 << 51) - 1, (1 << 63) - 1], dtype=np.int64)
    for f, a in ((12, 70), (12, 64), (70, 32), (63, 40), (62, 100), (64, 64), (65, 64), (200, 200), (63, 64)):
        fd, ad = device_bits(f, a)
        assert np.array_equal(fo.wrap_round(acc, f, a), fo.wrap_round(acc, fd, ad))


def test_wrap_round_equals_unbounded_reference_arithmetic():
    """fir_1d_fixed_ref.py:110-120 on Python ints vs the oracle's overflow-free int64 form, for
    sums up to the full int64 range (long filters) and every frac / acc width class."""
    rng = np.random.default_rng(63)
    acc = np.concatenate([rng.integers(-(1 << 63), (1 << 63) - 1, 400, dtype=np.int64),
                          np.array([-(1 << 63), (1 << 63) - 1, -1, 0, 1], dtype=np.int64)])
    for f in (1, 2, 12, 31, 32, 52, 62, 63, 64, 65, 90):
        for a in (1, 8, 32, 33, 63, 64, 70):
            got = fo.wrap_round(acc, f, a)
            for v, g in zip(acc.tolist(), got.tolist()):
                if a < 64:  # the reference's mask + sign restore
                    v &= (1 << a) - 1
                    if v & (1 << (a - 1)):
                        v -= 1 << a
                assert g == (v + (1 << (f - 1))) >> f, (v, f, a)


def test_parse_devices():
    """``--devices``: a count, a comma list (repeats allowed), a sequence; None = device 0."""
    from fir_hip import parse_devices

    assert parse_devices(None) == [0]
    assert parse_devices(3) == [0, 1, 2]
    assert parse_devices("2") == [0, 1]
    assert parse_devices("0,0,3") == [0, 0, 3]
    assert parse_devices([1, 1]) == [1, 1]
    assert parse_devices("3,") == [3]  # one non-zero device id
    assert parse_devices("1,2,") == [1, 2]
    for bad in (0, "0", [], [-1], ","):
        with pytest.raises(ValueError):
            parse_devices(bad)


def test_rows_over_devices_blocks_cover_every_row_once():
    from fir_hip import _over_devices

    for nrows in (0, 1, 5, 37):
        for devs in ([0], [0, 0, 0], [0, 1], [2, 0, 2, 1]):
            seen = []
            _over_devices(nrows, devs, lambda r0, r1, d: seen.extend(range(r0, r1)))
            assert sorted(seen) == list(range(nrows)), (nrows, devs)


def test_pipeline_default_image_source_is_package_data(image_outputs):
    """The CLI's default inputs (pipeline_fir_1d.default_image_source) are the package's own decoded
    copy of the reference images, not a test fixture; every image has the reference decode's
    SHA-256."""
    import hashlib
    from pathlib import Path

    import pipeline_fir_1d

    src = pipeline_fir_1d.default_image_source()
    pkg = Path(pipeline_fir_1d.__file__).resolve().parent
    assert src.is_relative_to(pkg) and "tests" not in src.relative_to(pkg).parts
    with np.load(src) as d:
        got = {k: hashlib.sha256(np.ascontiguousarray(d[k]).tobytes()).hexdigest() for k in d.files}
    assert got == {k: v["sha256"] for k, v in image_outputs["inputs"].items()}
