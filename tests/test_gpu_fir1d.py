"""GPU parity of the 1-D fixed-point path through the C ABI.

Every result is compared bit-exactly with either the reference's own golden vectors
(tests/golden, produced by running the reference) or the C/NumPy oracle that those
vectors pin.  Mirrors the reference's fir_1d/sim/tests/test_1d_fixed.py (known answers,
saturation, output contract) and test_fixed_output.py (generator files), then goes
past them: random (x, h, frac, acc, coeff) sweeps, every image x filter, int16 /
complex variants, ragged / narrow / unaligned buffers, halo edges, guard bytes and the
full 2^28-sample benchmark size.
"""
from __future__ import annotations

import ctypes
import hashlib
from pathlib import Path

import numpy as np
import pytest
import torch

import fir_hip
from conftest import iter_ragged, load_kats
from fir_1d.model.python.fir_1d_fixed_ref import fir_1d_fixed_golden
from fir_1d.sim.vector.gen_fixed_output import (_run_fixed_rowwise, generate_fixed_3tap_output_vector,
                                                generate_fixed_5tap_output_vector)
from fir_1d.sim.vector.h_coeff import h_coeff_3tap_map, h_coeff_5tap_map
from fir_hip import torch_ops
from oracle import c_oracle, fir_oracle as fo

DEV = torch.device("cuda:0")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_device_present():
    assert fir_hip.device_count() >= 1


# ---- the reference's own unit tests (fir_1d/sim/tests/test_1d_fixed.py) -------------
def test_same_mode_center_aligned_q412_exact_case():
    assert fir_1d_fixed_golden([10, 20, 30, 40], [0.25, 0.5, 0.25]).tolist() == [10, 20, 30, 28]


def test_input_preprocessing_round_half_up_then_clamp():
    assert fir_1d_fixed_golden([-1.2, 0.5, 1.5, 254.6, 300.2], [1.0]).tolist() == [0, 1, 2, 255, 255]


def test_output_saturates_high_and_low():
    assert fir_1d_fixed_golden([255, 255], [7.999755859375]).tolist() == [255, 255]
    assert fir_1d_fixed_golden([255, 255], [-8.0]).tolist() == [0, 0]


def test_output_contract_dtype_length_and_range():
    r = fir_1d_fixed_golden([255, 255, 255, 255], [0.5, 0.25])
    assert isinstance(r, np.ndarray) and r.dtype == np.uint8 and len(r) == 4
    assert fir_1d_fixed_golden([10, 20], [7.999755859375]).shape == (2,)


def test_all_known_answer_records():
    n = 0
    for rec in load_kats("fixed"):
        if "expect" in rec:
            assert fir_1d_fixed_golden(rec["x"], rec["h"], **rec["kwargs"]).tolist() == rec["expect"], rec
            n += 1
    assert n >= 12


def test_random_reference_sweep_3000_cases():
    """(x, h, frac_bits, acc_bits, coeff_bits) drawn at random, outputs from the reference."""
    bad = []
    for i, (x, h, (f, a, c), y) in enumerate(iter_ragged("fixed")):
        got = fir_1d_fixed_golden(x.tolist(), h.tolist(), frac_bits=f, acc_bits=a, coeff_bits=c)
        if not np.array_equal(got, y):
            bad.append((i, f, a, c, len(h), len(x)))
    assert not bad, bad[:10]


# ---- golden images: all 56 fixed outputs of the reference pipeline -------------------
def test_all_56_image_outputs_bit_exact(images, image_outputs):
    for o in image_outputs["outputs"]:
        x = images[o["case_stem"]]
        h = image_outputs["banks"][o["tap"]][o["coeff_name"]]
        y = _run_fixed_rowwise(x, h, frac_bits=12, acc_bits=32, coeff_bits=16)
        assert _sha(y) == o["fixed_u8_sha256"], (o["case_stem"], o["tap"], o["coeff_name"])


def test_small_images_full_arrays(images):
    d = np.load(Path(__file__).parent / "golden" / "small_image_outputs.npz")
    for key in d.files:
        if "_fixed_" not in key:
            continue
        stem, rest = key.split("__")
        coeff, tap = rest.split("_fixed_")
        bank = h_coeff_3tap_map if tap == "3tap" else h_coeff_5tap_map
        y = _run_fixed_rowwise(images[stem], bank[coeff], frac_bits=12, acc_bits=32, coeff_bits=16)
        assert np.array_equal(y, d[key]), key


# ---- generator stage (reference fir_1d/sim/tests/test_fixed_output.py) ---------------
def _small_case(input_dir: Path) -> Path:
    input_dir.mkdir(parents=True, exist_ok=True)
    x = np.array([[10, 20, 30, 40, 50, 60, 70, 80], [80, 70, 60, 50, 40, 30, 20, 10],
                  [0, 10, 0, 10, 0, 10, 0, 10], [255, 200, 150, 100, 50, 0, 25, 75]], dtype=np.uint8)
    p = input_dir / "case_000_small_x_u8.npy"
    np.save(p, x)
    return p


def test_generator_files_shapes_and_spot_rows(tmp_path):
    xin = np.load(_small_case(tmp_path / "input"))
    out = tmp_path / "output"
    assert generate_fixed_3tap_output_vector(input_dir=tmp_path / "input", output_dir=out) == 4
    assert generate_fixed_5tap_output_vector(input_dir=tmp_path / "input", output_dir=out) == 4
    f3 = sorted((out / "fixed_3tap").glob("*.npy"))
    f5 = sorted((out / "fixed_5tap").glob("*.npy"))
    assert len(f3) == 4 and all("__" in p.name and "_fixed_3tap_y_u8.npy" in p.name for p in f3)
    assert len(f5) == 4 and all("_fixed_5tap_y_u8.npy" in p.name for p in f5)
    for p in f3 + f5:
        y = np.load(p)
        assert y.shape == xin.shape and y.dtype == np.uint8
    y = np.load(out / "fixed_3tap" / "case_000_small__simple_lp_fixed_3tap_y_u8.npy")
    for r in (0, 2):
        assert np.array_equal(y[r], fir_1d_fixed_golden(xin[r].tolist(), h_coeff_3tap_map["simple_lp"]))
    # skip-if-exists, then overwrite
    assert generate_fixed_3tap_output_vector(input_dir=tmp_path / "input", output_dir=out) == 0
    assert generate_fixed_3tap_output_vector(input_dir=tmp_path / "input", output_dir=out, overwrite=True) == 4


# ---- int16 -> int32 (a6) and complex int16 (a7) ----------------------------------------
CO = None


def _co():
    global CO
    if CO is None:
        CO = c_oracle()
    return CO


TAPS = {
    "sharpen5": [-256, -1024, 6656, -1024, -256],
    "wrap5": [32767, -32768, 32767, -32768, 32767],  # |acc| up to 5.4e9: exercises the 32-bit wrap
    "lp3": [1024, 2048, 1024],
    "one": [4096],
    "even4": [100, -200, 300, -400],
    "nine": [3, -5, 7, -11, 13, -11, 7, -5, 3],
    "t24": [(1 << 23) - 1, -(1 << 23), 12345],  # largest 24-bit taps (mul24 path)
    "t32": [(1 << 30), -(1 << 31), (1 << 31) - 1],  # > 24 bits: generic kernel
    "long17": list(range(-8, 9)),
}


@pytest.mark.parametrize("name", list(TAPS))
@pytest.mark.parametrize("channels", [1, 2])
@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 511, 512, 513, 4096 * 8 + 3, 1_000_003])
def test_int16_to_int32_vs_oracle(name, channels, n):
    hq = TAPS[name]
    rng = np.random.default_rng(n * 31 + len(hq))
    x = rng.integers(-32768, 32768, n * channels, dtype=np.int16)
    got = fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32, channels=channels)
    assert np.array_equal(got, fo.fir1d_i16_i32(x, hq, channels=channels))


@pytest.mark.parametrize("L", [10, 13, 16, 17, 24, 31, 32, 33, 48, 63, 64, 65])
@pytest.mark.parametrize("dtype,stage", [(np.int16, fir_hip.OUT_I32), (np.uint8, fir_hip.OUT_U8_SAT),
                                         (np.int16, fir_hip.OUT_U8_SAT), (np.uint8, fir_hip.OUT_I32)])
@pytest.mark.parametrize("shape", [(1, 100_003), (1, 2048), (37, 4096), (5, 1000), (3, 1001), (9, 8)])
def test_long_filters_vs_oracle(L, dtype, stage, shape):
    """10..64 taps: the int8 matrix-core kernel (fir1d_mfma.hip) or the LDS-window v_dot2 kernel
    (fir1d_lds.hip, int16 -> int32 below 40 taps, and ragged single rows) for one row or rows of
    a multiple of 8 samples (narrow rows included), the generic kernel otherwise / beyond 64
    taps; 32- and 24-bit accumulators."""
    rng = np.random.default_rng(L * 1000 + shape[1])
    info = np.iinfo(dtype)
    x = rng.integers(info.min, info.max + 1, shape, dtype=dtype)
    hq = rng.integers(-3000, 3000, L).tolist()
    for acc in (32, 24):
        got = fir_hip.fir1d_fixed_rows(x, hq, 12, acc, stage)
        assert np.array_equal(got, _co().fir1d_rows(x, hq, 12, acc, stage)), acc


@pytest.mark.parametrize("L", [17, 31, 64])
@pytest.mark.parametrize("shape", [(7, 3000), (1, 5128), (3, 1032), (2, 2056)])
def test_long_filter_step_geometry(L, shape):
    """The step-form MFMA kernel (fir1d_mfma.hip, two tiles per step) on rows whose tile count is
    odd (the last step's second tile is empty or partial) and on single rows just past a step."""
    rng = np.random.default_rng(L * 7 + shape[1])
    hq = rng.integers(-3000, 3000, L).tolist()
    co = _co()
    for dtype in (np.int16, np.uint8):
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max + 1, shape, dtype=dtype)
        for stage in (fir_hip.OUT_I32, fir_hip.OUT_U8_SAT):
            assert np.array_equal(fir_hip.fir1d_fixed_rows(x, hq, 12, 32, stage), co.fir1d_rows(x, hq, 12, 32, stage)), (
                dtype, stage)


@pytest.mark.parametrize("L", [10, 17, 32, 33, 48, 64])
def test_long_filters_matrix_core_extremes(L):
    """The int8 matrix-core path (fir1d_mfma.hip) at the edges of its signed-byte splits: taps at
    -32768 and 32639 (the largest tap whose high byte stays a signed byte; 32640 goes to the v_dot2
    kernel), full-range int16 samples so the 32-bit sums wrap, 32/24/20-bit accumulators, tiles cut
    by rows of 1000 and 8 samples and by a ragged single row; u8 runs of 0 and 255 (saturation)."""
    rng = np.random.default_rng(7000 + L)
    co = _co()
    for taps in (rng.choice([-32768, 32639, -1, 1, 127, 128, -128, -129, 255, -256], L).tolist(),
                 rng.integers(-600, 600, L).tolist(), [32640] + [3] * (L - 1)):
        for shape in [(1, 70_001), (3, 1000), (2, 4096), (40, 8)]:
            x16 = rng.integers(-32768, 32768, shape, dtype=np.int16)
            xu = rng.integers(0, 256, shape, dtype=np.uint8)
            xu[:, : shape[1] // 3] = 255
            xu[:, shape[1] // 3: shape[1] // 2] = 0
            for acc in (32, 24, 20):
                for stage in (fir_hip.OUT_I32, fir_hip.OUT_U8_SAT):
                    for x in (x16, xu):
                        got = fir_hip.fir1d_fixed_rows(x, taps, 12, acc, stage)
                        assert np.array_equal(got, co.fir1d_rows(x, taps, 12, acc, stage)), (shape, acc, stage, x.dtype)


def test_long_filter_large_vs_oracle():
    """Many workgroups: 31 taps over 2^24 int16 samples, and over u8 images of 4096-sample rows."""
    rng = np.random.default_rng(31)
    hq = rng.integers(-32768, 32768, 31).tolist()  # full int16 taps: the 32-bit sums wrap
    x = rng.integers(-32768, 32768, 1 << 24, dtype=np.int16)
    assert np.array_equal(fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32),
                          _co().fir1d_rows(x, hq, 12, 32, fir_hip.OUT_I32))
    xu = rng.integers(0, 256, (1024, 4096), dtype=np.uint8)
    assert np.array_equal(fir_hip.fir1d_fixed_rows(xu, hq[:20], 12, 32, fir_hip.OUT_U8_SAT),
                          _co().fir1d_rows(xu, hq[:20], 12, 32, fir_hip.OUT_U8_SAT))


@pytest.mark.parametrize("frac,acc", [(1, 32), (12, 16), (12, 24), (15, 31), (20, 32), (12, 40), (12, 64), (31, 32),
                                      (40, 48), (63, 64)])
@pytest.mark.parametrize("stage", [fir_hip.OUT_I32, fir_hip.OUT_U8_SAT])
def test_bit_widths_vs_oracle(frac, acc, stage):
    rng = np.random.default_rng(frac * 100 + acc)
    x = rng.integers(-32768, 32768, 100_003, dtype=np.int16)
    hq = [-30000, 12000, 32767, -5]
    got = fir_hip.fir1d_fixed_rows(x, hq, frac, acc, stage)
    assert np.array_equal(got, fo.fir1d_rows(x.reshape(1, -1), hq, frac, acc, stage).reshape(-1))


def test_u8_inputs_pin_int16_variant():
    """For x in [0,255] the int16 path clipped to [0,255] equals the u8 golden model."""
    for x, h, (f, a, c), y in iter_ragged("fixed"):
        if a != 32 or c != 16 or len(x) < 1:
            continue
        xu = fo.prep_x(x).astype(np.int16)
        y32 = fir_hip.fir1d_fixed_rows(xu, fo.quantize_h(h, f, c), f, a, fir_hip.OUT_I32)
        assert np.array_equal(np.clip(y32, 0, 255).astype(np.uint8), y)


def test_complex_equals_two_real_filters():
    rng = np.random.default_rng(4)
    z = rng.integers(-32768, 32768, (100_001, 2), dtype=np.int16)
    hq = [1024, 2048, 1024]
    yc = fir_hip.fir1d_fixed_rows(z.reshape(-1), hq, 12, 32, fir_hip.OUT_I32, channels=2).reshape(-1, 2)
    re = fir_hip.fir1d_fixed_rows(np.ascontiguousarray(z[:, 0]), hq, 12, 32, fir_hip.OUT_I32)
    im = fir_hip.fir1d_fixed_rows(np.ascontiguousarray(z[:, 1]), hq, 12, 32, fir_hip.OUT_I32)
    assert np.array_equal(yc[:, 0], re) and np.array_equal(yc[:, 1], im)


# ---- row geometry: images of every width, both kernels ---------------------------------
@pytest.mark.parametrize("width", [1, 2, 3, 5, 15, 16, 17, 20, 31, 33, 64, 100, 640, 1279, 1280, 4499])
@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 8, 9, 10, 31])
def test_u8_rows_vs_oracle(width, L):
    rng = np.random.default_rng(width * 17 + L)
    rows = max(1, 50_000 // width) if width > 1 else 300
    x = rng.integers(0, 256, (rows, width), dtype=np.uint8)
    hq = rng.integers(-4096, 4096, L)
    for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
        got = fir_hip.fir1d_fixed_rows(x, hq, 12, 32, stage)
        assert np.array_equal(got, fo.fir1d_rows(x, hq, 12, 32, stage)), (width, L, stage)


@pytest.mark.parametrize("L", [2, 3, 4, 5, 6, 7, 8, 9])
def test_ragged_row_seams_vs_oracle(L):
    """Rows that straddle 16-byte vectors, u8 stage, one channel: computed as one signal with the
    L - 1 outputs around every row seam rewritten from their own row (kRagged, fir1d_reg.h).
    Widths from the narrowest the register kernel takes (vector + L - 1) up, seams at every
    vector offset, saturating pixels on both sides of each seam, banks of 1-4 filters mixing the
    packed-16 and v_dot2 forms, and int16 samples (8-sample vectors)."""
    rng = np.random.default_rng(L)
    for width in (16 + L - 1, 16 + L, 33 + L, 4499):
        rows = 48 if width < 100 else 9
        x = rng.integers(0, 256, (rows, width), dtype=np.uint8)
        x[:, :L] = 255
        x[:, -L:] = 255
        x[::3, :L] = 0
        for F in (1, 2, 4):
            hq = rng.integers(-3000, 3000, (F, L))
            hq[0] = np.abs(hq[0])
            if F > 1:
                hq[1] = rng.integers(0, 4, L) << 10  # packed-16 form
                hq[1, 0] |= 1 << 10
            ys = fir_hip.fir1d_fixed_rows_multi(x, hq, 12, 32, fir_hip.OUT_U8_SAT)
            for f in range(F):
                want = fo.fir1d_rows(x, hq[f], 12, 32, fir_hip.OUT_U8_SAT)
                assert np.array_equal(ys[f], want), (width, F, f)
        x16 = rng.integers(-32768, 32768, (rows, width), dtype=np.int16)
        hq = rng.integers(-3000, 3000, L)
        assert np.array_equal(fir_hip.fir1d_fixed_rows(x16, hq, 12, 32, fir_hip.OUT_U8_SAT),
                              fo.fir1d_rows(x16, hq, 12, 32, fir_hip.OUT_U8_SAT)), width


@pytest.mark.parametrize("width", [8, 17, 1280, 4499])
def test_i16_rows_and_complex_rows(width):
    rng = np.random.default_rng(width)
    x = rng.integers(-32768, 32768, (37, width * 2), dtype=np.int16)
    for hq in ([1, 2, 1], [5, -4, 3, -2, 1], [7] * 9):
        for ch in (1, 2):
            got = fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32, channels=ch)
            assert np.array_equal(got, fo.fir1d_rows(x, hq, 12, 32, fo.OUT_I32, channels=ch))


def test_many_taps_generic():
    rng = np.random.default_rng(9)
    x = rng.integers(0, 256, (13, 777), dtype=np.uint8)
    hq = rng.integers(-100, 100, 300)
    assert np.array_equal(fir_hip.fir1d_fixed_rows(x, hq, 12, 40, fir_hip.OUT_I32),
                          fo.fir1d_rows(x, hq, 12, 40, fo.OUT_I32))


# ---- device-pointer entries: alignment, guard bytes, halo edges, full size ------------
@pytest.mark.parametrize("offset", [0, 1, 3, 8])
def test_dev_path_offsets_and_guard_bytes(offset):
    rng = np.random.default_rng(offset)
    n = 300_001
    x = rng.integers(-32768, 32768, n, dtype=np.int16)
    hq = TAPS["sharpen5"]
    xbuf = torch.zeros(n + 64, dtype=torch.int16, device=DEV)
    xbuf[offset:offset + n] = torch.from_numpy(x).to(DEV)
    guard = 64
    ybuf = torch.full((n + 2 * guard + offset,), 0x5A5A5A5A, dtype=torch.int32, device=DEV)
    yv = ybuf[guard + offset:guard + offset + n]
    torch_ops.fir1d_fixed_rows_dev(xbuf[offset:offset + n], hq, 12, 32, fir_hip.OUT_I32, out=yv)
    torch.cuda.synchronize()
    yb = ybuf.cpu().numpy()
    assert np.array_equal(yb[guard + offset:guard + offset + n], fo.fir1d_i16_i32(x, hq))
    assert (yb[:guard + offset] == 0x5A5A5A5A).all() and (yb[guard + offset + n:] == 0x5A5A5A5A).all()


@pytest.mark.parametrize("hq,channels", [(TAPS["sharpen5"], 1), (TAPS["even4"], 1), (TAPS["lp3"], 2),
                                         (TAPS["nine"], 2), (TAPS["one"], 1)])
def test_edges_dev_rebuild_shards(hq, channels):
    rng = np.random.default_rng(len(hq) + channels)
    n = 200_003
    x = rng.integers(-32768, 32768, n * channels, dtype=np.int16)
    full = fo.fir1d_i16_i32(x, hq, channels=channels)
    hl, hr = fo.halo_sizes(len(hq))
    hl, hr = hl * channels, hr * channels
    cuts = [0, 12_345, 100_000, 100_001, n]
    outs = []
    for lo, hi in zip(cuts, cuts[1:]):
        seg = torch.from_numpy(x[lo * channels:hi * channels].copy()).to(DEV)
        out = torch_ops.fir1d_fixed_rows_dev(seg, hq, 12, 32, fir_hip.OUT_I32, channels)
        left = torch.from_numpy(x[lo * channels - hl:lo * channels].copy()).to(DEV) if lo > 0 and hl else None
        right = torch.from_numpy(x[hi * channels:hi * channels + hr].copy()).to(DEV) if hi < n and hr else None
        torch_ops.fir1d_fixed_edges_dev(seg, hq, out, left, right, 12, 32, fir_hip.OUT_I32, channels)
        outs.append(out.cpu().numpy())
    assert np.array_equal(np.concatenate(outs), full)


def test_full_benchmark_size_2_28_bit_exact():
    """The bench workload itself (BASELINE configs[1]): 2^28 int16 samples, 5-tap sharpen."""
    x = np.random.default_rng(20260227).integers(-32768, 32768, 1 << 28, dtype=np.int16)
    xd = torch.from_numpy(x).to(DEV)
    for hq in (TAPS["sharpen5"], TAPS["wrap5"]):
        y = torch_ops.fir1d_fixed_rows_dev(xd, hq, 12, 32, fir_hip.OUT_I32)
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), _co().fir1d_rows(x, hq, 12, 32, 1))
        del y


def test_full_size_complex_2_27():
    x = np.random.default_rng(20260227).integers(-32768, 32768, 1 << 28, dtype=np.int16)
    y = torch_ops.fir1d_fixed_rows_dev(torch.from_numpy(x).to(DEV), TAPS["lp3"], 12, 32, fir_hip.OUT_I32, 2)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), _co().fir1d_rows(x, TAPS["lp3"], 12, 32, 1, channels=2))


def test_host_entry_large_prefaulted_output():
    """The NumPy entry at 2^26 int16 -> int32 (a fresh 256 MiB output, pre-faulted by the host
    threads of run_host) and the C entry writing u8 output over its own u8 input (aliased:
    no pre-fault writes may touch the input)."""
    x = np.random.default_rng(20260301).integers(-32768, 32768, 1 << 26, dtype=np.int16)
    y = fir_hip.fir1d_fixed_rows(x, TAPS["wrap5"], 12, 32, fir_hip.OUT_I32)
    assert np.array_equal(y, _co().fir1d_rows(x, TAPS["wrap5"], 12, 32, 1))
    xu = np.random.default_rng(20260302).integers(0, 256, 1 << 26, dtype=np.uint8)
    ref = _co().fir1d_rows(xu, TAPS["sharpen5"], 12, 32, 0)
    h = np.asarray(TAPS["sharpen5"], np.int32)
    buf = xu.copy()
    vp = ctypes.c_void_p
    rc = fir_hip.lib().fir1d_fixed_rows(vp(buf.ctypes.data), fir_hip.IN_U8, 1, buf.size, 1, vp(h.ctypes.data),
                                        h.size, 12, 32, fir_hip.OUT_U8_SAT, vp(buf.ctypes.data), 0)
    assert rc == 0
    assert np.array_equal(buf, ref)


def test_repeat_launch_deterministic():
    x = torch.randint(-32768, 32768, (1 << 22,), dtype=torch.int16, device=DEV)
    a = torch_ops.fir1d_fixed_rows_dev(x, TAPS["wrap5"])
    b = torch_ops.fir1d_fixed_rows_dev(x, TAPS["wrap5"])
    torch.cuda.synchronize()
    assert torch.equal(a, b)


# ---- multi-filter fusion ----------------------------------------------
def test_multi_filter_banks_equal_reference_outputs(images, image_outputs):
    """One fused call per (image, bank) reproduces all 56 reference fixed outputs."""
    by_key = {(o["case_stem"], o["tap"], o["coeff_name"]): o["fixed_u8_sha256"] for o in image_outputs["outputs"]}
    for stem, x in images.items():
        for tap, bank in (("3tap", h_coeff_3tap_map), ("5tap", h_coeff_5tap_map)):
            hq = np.stack([fo.quantize_h(h) for h in bank.values()])
            ys = fir_hip.fir1d_fixed_rows_multi(x, hq)
            for name, y in zip(bank, ys):
                assert _sha(y) == by_key[(stem, tap, name)], (stem, tap, name)


@pytest.mark.parametrize("F", [1, 2, 3, 4, 5, 9])
@pytest.mark.parametrize("dtype,L", [(np.uint8, 3), (np.uint8, 5), (np.uint8, 12), (np.int16, 5)])
def test_multi_filter_random_vs_oracle(F, dtype, L):
    rng = np.random.default_rng(F * 100 + L)
    if dtype == np.uint8:
        x = rng.integers(0, 256, (61, 1283), dtype=np.uint8)
    else:
        x = rng.integers(-32768, 32768, (7, 10_001), dtype=np.int16)
    hq = rng.integers(-5000, 5000, (F, L))
    for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
        ys = fir_hip.fir1d_fixed_rows_multi(x, hq, 12, 32, stage)
        assert ys.shape == (F,) + x.shape
        for f in range(F):
            assert np.array_equal(ys[f], fo.fir1d_rows(x, hq[f], 12, 32, stage)), (f, stage)


@pytest.mark.parametrize("width", [1283, 4096, 640])
@pytest.mark.parametrize("frac", [12, 8, 15, 20])
def test_multi_filter_packed16_forms_vs_oracle(width, frac):
    """u8 banks whose filters fit the packed-16 form (taps = small ints x 2^s): unsigned,
    signed, high-byte and v_dot2 filters mixed in one fused launch, bit-exact."""
    rng = np.random.default_rng(width + frac)
    x = rng.integers(0, 256, (37, width), dtype=np.uint8)
    x[0, :] = 255  # extremes of every sum
    x[1, :] = 0
    x[2, ::2] = 255
    for L in (2, 3, 5, 9):
        for trial in range(4):
            F = int(rng.integers(2, 5))
            small = rng.integers(-12, 13, (F, L))
            small[0] = np.abs(small[0])  # an unsigned-sum filter
            shifts = rng.integers(0, frac, (F, 1))
            hq = small << shifts
            hq[-1] = rng.integers(-3000, 3000, L) | 1  # odd taps: the v_dot2 form
            for f in range(F):
                if not hq[f].any():
                    hq[f, 0] = 1 << int(shifts[f, 0])
            for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
                ys = fir_hip.fir1d_fixed_rows_multi(x, hq, frac, 32, stage)
                for f in range(F):
                    assert np.array_equal(ys[f], fo.fir1d_rows(x, hq[f], frac, 32, stage)), (L, trial, f, stage)


def test_generator_over_golden_images_uses_fused_path(tmp_path, images, image_outputs):
    inp = tmp_path / "input"
    inp.mkdir()
    for stem, x in images.items():
        np.save(inp / f"{stem}_x_u8.npy", x)
    out = tmp_path / "output"
    assert generate_fixed_3tap_output_vector(input_dir=inp, output_dir=out) == 28
    assert generate_fixed_5tap_output_vector(input_dir=inp, output_dir=out) == 28
    for o in image_outputs["outputs"]:
        p = out / f"fixed_{o['tap']}" / f"{o['case_stem']}__{o['coeff_name']}_fixed_{o['tap']}_y_u8.npy"
        assert _sha(np.load(p)) == o["fixed_u8_sha256"], p.name


@pytest.mark.gpu
def test_out_argument_reuses_the_buffer():
    """``out=`` returns the caller's array filled with the same bits as a fresh call, for the
    single, multi-filter and 2-D entries, and in place over a u8 input."""
    rng = np.random.default_rng(20261016)
    x = rng.integers(0, 256, (37, 1001), dtype=np.uint8)
    h = TAPS["sharpen5"]
    ref = _co().fir1d_rows(x, h, 12, 32, 0)
    out = np.full_like(x, 7)
    assert fir_hip.fir1d_fixed_rows(x, h, out=out) is out and np.array_equal(out, ref)
    buf = x.copy()
    assert fir_hip.fir1d_fixed_rows(buf, h, out=buf) is buf and np.array_equal(buf, ref)
    o32 = np.zeros(x.shape, np.int32)
    fir_hip.fir1d_fixed_rows(x, h, out_stage=fir_hip.OUT_I32, out=o32)
    assert np.array_equal(o32, fir_hip.fir1d_fixed_rows(x, h, out_stage=fir_hip.OUT_I32))
    hq = np.stack([np.asarray(TAPS["lp3"] + [0, 0]), np.asarray(h)])
    om = np.zeros((2,) + x.shape, np.uint8)
    assert fir_hip.fir1d_fixed_rows_multi(x, hq, out=om) is om
    assert np.array_equal(om, fir_hip.fir1d_fixed_rows_multi(x, hq))
    k = [[1, 2, 1], [2, 4, 2], [1, 2, 1]]
    o2 = np.zeros(x.shape, np.uint8)
    assert fir_hip.fir2d_fixed(x, k, out=o2) is o2 and np.array_equal(o2, fir_hip.fir2d_fixed(x, k))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,dtype,channels,taps", [
    ((1, 2 * ((1 << 25) + 37)), np.int16, 2, 63),    # one long row: 8 halo-reading segments
    ((1, (1 << 26) + 13), np.uint8, 1, 4),            # ragged last segment, even taps
    ((4099, 16411), np.uint8, 1, 5),                  # row blocks
    ((1, 3 * ((1 << 26) + 11)), np.uint8, 3, 5),      # frames of 3 channels: segments start on a frame
    ((1, 3 * ((1 << 25) + 5)), np.int16, 3, 3),       # same, int16 (generic kernel per segment)
    ((1, 5 * ((1 << 24) + 3)), np.int16, 5, 1),       # one tap: any channel count is legal
    ((1, 1000003 * 70), np.uint8, 1000003, 1),        # frames longer than a chunk: unchunked
    ((1031, 3 * 21701), np.int16, 3, 5),              # row blocks of 3-channel rows
])
def test_host_entry_chunked_overlap(shape, dtype, channels, taps):
    """Host calls of >= 64 MiB run in 8 chunks with the H2D and D2H copies overlapped
    (capi.hip run_host_chunked); same bits as the oracle, also in place for u8."""
    rng = np.random.default_rng(20261017)
    info = np.iinfo(dtype)
    x = rng.integers(info.min, info.max + 1, shape, dtype=dtype)
    hq = rng.integers(-3000, 3000, taps).tolist()
    stage = fir_hip.OUT_I32 if dtype == np.int16 else fir_hip.OUT_U8_SAT
    ref = _co().fir1d_rows(x, hq, 12, 32, 1 if stage == fir_hip.OUT_I32 else 0, channels=channels)
    assert np.array_equal(fir_hip.fir1d_fixed_rows(x, hq, out_stage=stage, channels=channels), ref)
    if dtype == np.uint8:
        buf = x.copy()
        fir_hip.fir1d_fixed_rows(buf, hq, channels=channels, out=buf)
        assert np.array_equal(buf, ref)


@pytest.mark.parametrize("c", [1365, 1366, 1370, 1371, 4095])
def test_bank_noclamp_stage_boundary(c):
    """A v_dot2-form filter whose biased sum provably stays in [0, 256 * 2^frac) runs its u8 stage
    as a shift alone (fir1d_reg.h plan_u8_noclamp): moving averages c * [1, 1, 1] on both sides of
    that bound (3 * 255 * c + 2048 < 2^20 holds up to c = 1368), on all-zero, all-255 and random
    u8 rows, beside packed-16 filters in one bank, against the C oracle bit for bit."""
    co = c_oracle()
    rng = np.random.default_rng(c)
    hq = np.array([[c] * 3, [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]])
    for x in (np.zeros((8, 4096), np.uint8), np.full((8, 4096), 255, np.uint8),
              rng.integers(0, 256, (8, 4096), dtype=np.uint8), rng.integers(250, 256, (8, 4096), dtype=np.uint8)):
        ys = fir_hip.fir1d_fixed_rows_multi(x, hq, 12, 32, fir_hip.OUT_U8_SAT)
        for f in range(4):
            assert np.array_equal(ys[f], co.fir1d_rows(x, hq[f], 12, 32, fir_hip.OUT_U8_SAT)), (c, f)
