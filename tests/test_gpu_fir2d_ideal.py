"""GPU parity of the 2-D fixed path and the float64 ideal model (§8(f) 1).

fir_2d has no reference implementation (fir_2d/model/cpp/CMakeLists.txt is empty); its
semantics are pinned two ways: (1) a 5x5 kernel with only the centre row (column)
non-zero must equal the reference's row-wise golden model on the image (its transpose),
using the reference's own golden outputs; (2) general kernels against the C oracle.
The ideal kernel is pinned bit-for-bit (float64 bytes) to the reference's outputs.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

import numpy as np
import pytest
import torch

import fir_hip
from conftest import iter_ragged, load_kats
from fir_1d.model.python.fir_1d_ref import fir_1d_ideal
from fir_1d.sim.vector.gen_ideal_output import _run_ideal_rowwise
from fir_1d.sim.vector.h_coeff import h_coeff_3tap_map, h_coeff_5tap_map
from fir_hip import torch_ops
from oracle import c_oracle, fir_oracle as fo

DEV = torch.device("cuda:0")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---- fir_2d ---------------------------------------------------------------------------
def test_fir2d_centre_row_and_column_pins(images, image_outputs):
    for o in image_outputs["outputs"]:
        if o["tap"] != "5tap":
            continue
        x = images[o["case_stem"]]
        h1 = fo.quantize_h(image_outputs["banks"]["5tap"][o["coeff_name"]])
        k = np.zeros((5, 5), np.int64)
        k[2] = h1
        assert _sha(fir_hip.fir2d_fixed(x, k)) == o["fixed_u8_sha256"], o["case_stem"]
        xt = np.ascontiguousarray(x.T)
        yt = fir_hip.fir2d_fixed(xt, k.T.copy())
        assert _sha(np.ascontiguousarray(yt.T)) == o["fixed_u8_sha256"], o["case_stem"]


@pytest.mark.parametrize("shape", [(1, 16), (3, 32), (37, 64), (64, 64), (100, 1280), (257, 4096), (5, 16 * 300),
                                   (33, 17), (40, 4499), (1, 1), (7, 3)])
@pytest.mark.parametrize("R,C", [(5, 5), (3, 3), (1, 5), (5, 1), (3, 5), (2, 4), (7, 7)])
def test_fir2d_vs_oracle(shape, R, C):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1] + R * 10 + C)
    x = rng.integers(0, 256, shape, dtype=np.uint8)
    hq = rng.integers(-2048, 2048, (R, C))
    co = c_oracle()
    for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
        assert np.array_equal(fir_hip.fir2d_fixed(x, hq, 12, 32, stage), co.fir2d(x, hq, 12, 32, stage)), stage


def test_fir2d_wrap_and_bit_widths():
    rng = np.random.default_rng(12)
    x = rng.integers(0, 256, (96, 512), dtype=np.uint8)
    hq = np.full((5, 5), 8_000_000, dtype=np.int64)  # 25 * 255 * 8e6 = 5.1e10: wraps 32 bits
    co = c_oracle()
    for frac, acc in ((12, 32), (12, 24), (20, 32), (12, 40)):
        assert np.array_equal(fir_hip.fir2d_fixed(x, hq, frac, acc, 1), co.fir2d(x, hq, frac, acc, 1))


SEP_KERNELS = [  # (col, row): rank-1 kernels reaching each separable variant
    ([16, 64, 96, 64, 16], [1, 4, 6, 4, 1]),            # int16 row sums, no wrap (the bench kernel)
    ([-3, 7, 11, 7, -3], [2, -5, 9, -5, 2]),            # signed, int16 row sums
    ([1, 2, 1], [1000, -3000, 1000]),                   # row sums beyond int16: 32-bit column pass
    ([3, -1, 3], [200, 300, -100, 300, 200]),          # 32-bit column pass, 3x5
    ([127] * 5, [255, 255, 255]),                       # near-int16 taps; wraps at acc_bits = 24
    ([40000, -1, 3], [1, 1, 1]),                        # taps beyond int16: generic kernel
    ([-1, 3, -1], [1, -2, 5, -2, 1]),                   # packed 16-bit pairs, signed sum
    ([1, 2, 1], [1, 2, 1]),                             # packed 16-bit pairs, unsigned, shift 12
]
# Kernel 0 reaches the packed 16-bit path with f - s = 8 (high-byte output) at frac 12, with a
# clamped shift of 4 at frac 8, and sep16 at frac 16 (its 16-bit sum would overflow there).


@pytest.mark.parametrize("path", ["auto", "mfma"])
@pytest.mark.parametrize("k", range(len(SEP_KERNELS)))
@pytest.mark.parametrize("shape", [(1, 16), (29, 64), (64, 1280), (300, 4096 + 16)])
def test_fir2d_separable_variants_vs_oracle(k, shape, path, monkeypatch):
    monkeypatch.setenv("FIR2D_PATH", path)  # rank-1 kernels: register form by default, or MFMA
    col, row = SEP_KERNELS[k]
    hq = np.outer(np.array(col, np.int64), np.array(row, np.int64))
    rng = np.random.default_rng(k * 7 + shape[0])
    x = rng.integers(0, 256, shape, dtype=np.uint8)
    co = c_oracle()
    for frac, acc in ((12, 32), (8, 24), (16, 32)):
        for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
            assert np.array_equal(fir_hip.fir2d_fixed(x, hq, frac, acc, stage),
                                  co.fir2d(x, hq, frac, acc, stage)), (frac, acc, stage)


GEN_PK_KERNELS = [  # non-separable kernels reaching the general packed-16 forms at frac 12
    [[16, 32, 16], [32, 48, 32], [16, 32, 16]],                       # unsigned, f - s = 8: high byte
    [[1, 2, 3], [4, 5, 6], [7, 8, 10]],                               # unsigned, shift 12
    [[-1, 3, -1], [3, -8, 3], [-1, 3, -1]],                           # signed sum
    [[0, -512, 0], [-512, 3072, -512], [0, -512, 0]],                 # Laplacian sharpen, s = 9
    [[1, -2, 5, -2, 1]],                                              # 1 x 5 (never rank-1 split)
    [[2], [-1], [7], [-1], [2]],                                      # 5 x 1
    np.random.default_rng(55).integers(-4, 5, (5, 5)).tolist(),       # general 5x5, signed
    np.random.default_rng(56).integers(0, 5, (3, 5)).tolist(),        # 3x5, unsigned
]
# At frac 8 the same kernels take the clamped shift (s <= f - 1); at frac 16 most exceed
# 16-bit shifts (f - s > 15) or the range and fall back to v_dot2; acc 24 keeps the no-wrap proof.


@pytest.mark.parametrize("path", ["auto", "reg"])
@pytest.mark.parametrize("k", range(len(GEN_PK_KERNELS)))
@pytest.mark.parametrize("shape", [(1, 16), (29, 64), (64, 1280), (300, 4096 + 16)])
def test_fir2d_general_packed16_vs_oracle(k, shape, path, monkeypatch):
    monkeypatch.setenv("FIR2D_PATH", path)  # general kernels: MFMA by default, or the register form
    hq = np.array(GEN_PK_KERNELS[k], np.int64)
    rng = np.random.default_rng(k * 11 + shape[0])
    x = rng.integers(0, 256, shape, dtype=np.uint8)
    x[0, : min(16, shape[1])] = 255  # saturating corners
    co = c_oracle()
    for frac, acc in ((12, 32), (8, 24), (16, 32), (10, 32)):
        for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
            assert np.array_equal(fir_hip.fir2d_fixed(x, hq, frac, acc, stage),
                                  co.fir2d(x, hq, frac, acc, stage)), (frac, acc, stage)


@pytest.mark.parametrize("path", ["auto", "reg"])
def test_fir2d_full_frame_8192_general(path, monkeypatch):
    """configs[4] frame with a non-separable 5x5 kernel (MFMA by default, general packed-16 form)."""
    monkeypatch.setenv("FIR2D_PATH", path)
    x = np.random.default_rng(20260228).integers(0, 256, (8192, 8192), dtype=np.uint8)
    hq = np.array(GEN_PK_KERNELS[6], np.int64)
    y = torch_ops.fir2d_fixed_dev(torch.from_numpy(x).to(DEV), hq)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), c_oracle().fir2d(x, hq))


MFMA_KERNELS = [  # fir2d_mfma.hip: one tap byte plane after the power-of-two factor, or two
    np.random.default_rng(55).integers(-4, 5, (5, 5)),                # 1 plane
    np.random.default_rng(7).integers(-3000, 3000, (5, 5)),           # 2 planes (Q4.12-sized)
    np.random.default_rng(8).integers(-32768, 32640, (5, 5)),         # 2 planes, wraps 32 bits
    np.random.default_rng(9).integers(-100, 100, (3, 4)),             # even width: halo 1 + 2
    np.random.default_rng(10).integers(-100, 100, (5, 2)),
    np.array([[2], [-1], [7], [-1], [2]]) * 64,                       # column filter, s = 6
    np.random.default_rng(11).integers(-127, 128, (3, 5)) | 1,        # odd taps: s = 0
    np.zeros((5, 5), np.int64),                                       # all zero
]


@pytest.mark.parametrize("k", range(len(MFMA_KERNELS)))
@pytest.mark.parametrize("shape", [(1, 16), (2, 1024), (7, 48), (33, 1040), (100, 4096 + 16), (37, 3072 + 512)])
def test_fir2d_mfma_vs_oracle(k, shape, monkeypatch):
    """The matrix-core path forced on: ragged widths (partial 1024-pixel tiles), heights that
    are not a whole strip, saturating corners, every bit width class (fast byte-2 form at
    frac <= 16, rounded wrap form above it or when the sum can wrap)."""
    monkeypatch.setenv("FIR2D_PATH", "mfma")
    hq = MFMA_KERNELS[k]
    rng = np.random.default_rng(k * 13 + shape[0])
    x = rng.integers(0, 256, shape, dtype=np.uint8)
    x[0, : min(32, shape[1])] = 255
    x[-1, -min(32, shape[1]):] = 0
    co = c_oracle()
    for frac, acc in ((12, 32), (8, 24), (16, 32), (10, 32), (20, 32), (12, 20)):
        assert np.array_equal(fir_hip.fir2d_fixed(x, hq, frac, acc, fir_hip.OUT_U8_SAT),
                              co.fir2d(x, hq, frac, acc, 0)), (frac, acc)


def test_fir2d_mfma_frames_and_full_frame(monkeypatch):
    """Batched frames and the configs[4] frame size on the matrix-core path, rank-1 bench kernel
    included (forced: by default it stays on the separable register form)."""
    monkeypatch.setenv("FIR2D_PATH", "mfma")
    rng = np.random.default_rng(91)
    co = c_oracle()
    x = rng.integers(0, 256, (3, 70, 2048 + 64), dtype=np.uint8)
    for hq in (MFMA_KERNELS[0], MFMA_KERNELS[1]):
        got = fir_hip.fir2d_fixed(x, hq)
        for f in range(3):
            assert np.array_equal(got[f], co.fir2d(x[f], hq, 12, 32, 0)), f
    xf = rng.integers(0, 256, (8192, 8192), dtype=np.uint8)
    sep = np.outer([256, 1024, 1536, 1024, 256], [256, 1024, 1536, 1024, 256]) // 4096
    y = torch_ops.fir2d_fixed_dev(torch.from_numpy(xf).to(DEV), sep)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), co.fir2d(xf, sep))


PK16_KERNELS = [  # rank-1 kernels on the separable packed-16 strip kernel (fir2d_pk16.h)
    np.outer([16, 64, 96, 64, 16], [1, 4, 6, 4, 1]),                 # high-byte output (bench kernel form)
    np.outer([1, 2, 1], [1, 2, 1]),                                   # unsigned, shift 12, R = 3 (turns of 15)
    np.outer([-1, 3, -1], [1, -2, 5, -2, 1]),                         # signed sum, 3 x 5
]


def test_fir2d_pk16_strip_heights_vs_oracle():
    """Strips walking down (even strips) and up (odd strips), over frames whose height is not a
    whole number of strips (and shorter than one), batched frames included."""
    rng = np.random.default_rng(3)
    co = c_oracle()
    for k in PK16_KERNELS:
        for shape in ((1, 64), (2, 48), (5, 4096), (17, 1040), (64, 8192), (101, 256), (3, 41, 512)):
            x = rng.integers(0, 256, shape, dtype=np.uint8)
            x[..., 0, :16] = 255
            got = fir_hip.fir2d_fixed(x, k)
            xs = x if x.ndim == 3 else x[None]
            for f in range(xs.shape[0]):
                want = co.fir2d(xs[f], k, 12, 32, 0)
                assert np.array_equal(got if x.ndim == 2 else got[f], want), (k.shape, shape, f)


def test_fir2d_pk16_frame_past_2p31_pixels():
    """A 32768 x 65536 frame (2^31 pixels) takes the unrolled 32-row strip kernel; rows at the top,
    bottom and across strip seams are compared with the oracle run on row bands of the frame."""
    H, W = 32768, 65536
    k = PK16_KERNELS[0]
    xd = torch.randint(0, 256, (H, W), dtype=torch.uint8, device=DEV)
    yd = torch_ops.fir2d_fixed_dev(xd, k)
    torch.cuda.synchronize()
    co = c_oracle()
    for a, b in ((0, 40), (16000, 16070), (H - 40, H)):
        lo, hi = max(a - 2, 0), min(b + 2, H)
        band = xd[lo:hi].cpu().numpy()
        want = co.fir2d(band, k, 12, 32, 0)[a - lo:a - lo + (b - a)]
        assert np.array_equal(yd[a:b].cpu().numpy(), want), (a, b)


def test_fir2d_frame_batches_device_and_host():
    """(frames, H, W) batches: one launch, every frame = its own single-frame result, on the
    register (8192-wide, separable packed-16 and general) and generic (odd width) paths."""
    rng = np.random.default_rng(77)
    sep = (np.outer([1, 4, 6, 4, 1], [1, 4, 6, 4, 1]) * 16).tolist()
    gen = rng.integers(-4, 5, (5, 5)).tolist()
    for shape in ((3, 64, 8192), (2, 37, 1001), (4, 130, 640)):
        x = rng.integers(0, 256, shape, dtype=np.uint8)
        for k in (sep, gen):
            got = fir_hip.fir2d_fixed(x, k)
            dev = torch_ops.fir2d_fixed_dev(torch.from_numpy(x).cuda(), k)
            torch.cuda.synchronize()
            assert np.array_equal(dev.cpu().numpy(), got)
            for f in range(shape[0]):
                assert np.array_equal(got[f], c_oracle().fir2d(x[f], np.asarray(k), 12, 32, 0)), (shape, f)


def test_fir2d_full_frame_8192():
    """BASELINE configs[4]: 8192 x 8192 u8 frame, 5x5 unity-gain kernel."""
    x = np.random.default_rng(20260227).integers(0, 256, (8192, 8192), dtype=np.uint8)
    h1 = np.array([256, 1024, 1536, 1024, 256], dtype=np.int64)
    hq = np.outer(h1, h1) // 4096
    y = torch_ops.fir2d_fixed_dev(torch.from_numpy(x).to(DEV), hq)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), c_oracle().fir2d(x, hq))


# ---- ideal float64 ---------------------------------------------------------------------
def test_ideal_reference_unit_cases():
    # fir_1d/sim/tests/test_1d_ideal.py:8-42 vectors, bit-exact here
    assert fir_1d_ideal([10, 20, 30, 40], [0.25, 0.5, 0.25]) == [10.0, 20.0, 30.0, 27.5]
    assert len(fir_1d_ideal([3, 7, 11, 15, 19], [0.1, 0.5, 0.3, 0.1])) == 5
    assert fir_1d_ideal([-1.2, 0.49, 0.5, 1.5, 254.6, 300.2], [1.0]) == [0.0, 0.0, 1.0, 2.0, 255.0, 255.0]
    assert fir_1d_ideal([255, 255], [5.0]) == [1275.0, 1275.0]
    assert len(fir_1d_ideal([10, 20], [-8.0, 8.0])) == 2


def test_ideal_known_answers_and_random_sweep_bits():
    for rec in load_kats("ideal"):
        if "expect" in rec:
            assert fir_1d_ideal(rec["x"], rec["h"]) == rec["expect"]
    for x, h, _, y in iter_ragged("ideal"):
        got = np.asarray(fir_1d_ideal(x.tolist(), h.tolist()), dtype=np.float64)
        assert got.tobytes() == y.tobytes()


def test_ideal_all_56_image_outputs_bit_exact(images, image_outputs):
    for o in image_outputs["outputs"]:
        h = image_outputs["banks"][o["tap"]][o["coeff_name"]]
        y = _run_ideal_rowwise(images[o["case_stem"]], h)
        assert _sha(y) == o["ideal_f64_sha256"], (o["case_stem"], o["tap"], o["coeff_name"])


def test_ideal_small_images_full_arrays(images):
    d = np.load(Path(__file__).parent / "golden" / "small_image_outputs.npz")
    for key in d.files:
        if "_ideal_" not in key:
            continue
        stem, rest = key.split("__")
        coeff, tap = rest.split("_ideal_")
        bank = h_coeff_3tap_map if tap == "3tap" else h_coeff_5tap_map
        assert _run_ideal_rowwise(images[stem], bank[coeff]).tobytes() == d[key].tobytes(), key
