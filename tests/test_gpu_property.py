"""Property-based GPU parity (hypothesis, derandomized): random shapes, tap sets, bit widths,
channel counts, buffer alignments and halos through the C ABI, each compared bit-exactly with
the C oracle (itself pinned to the reference's golden vectors by tests/test_oracle_golden.py).

Complements the fixed parameter grids of test_gpu_fir1d.py / test_gpu_fir2d_ideal.py: the
strategies cover every kernel the launchers can pick (register v_dot2 / byte-pair / packed-16 /
mad24 forms, the generic LDS kernel, the 2-D separable, packed-16 and general forms, the 2-D
int8 matrix-core kernel forced on, the halo segment path) without enumerating them, and hypothesis shrinks any failure to a small case.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from hypothesis import HealthCheck, given, settings, strategies as st

import fir_hip
from fir_hip import torch_ops
from oracle import c_oracle

SETTINGS = dict(deadline=None, database=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
DEV = torch.device("cuda:0")



def _taps(draw, n: int) -> list[int]:
    kind = draw(st.sampled_from(["q412", "q412", "small", "int16", "mad24", "wide"]))
    lim = {"q412": 8192, "small": 8, "int16": 32767, "mad24": (1 << 23) - 1, "wide": (1 << 31) - 1}[kind]
    return draw(st.lists(st.integers(-lim - 1 if kind != "small" else -lim, lim), min_size=n, max_size=n))


def _unaligned(a: np.ndarray, off: int) -> np.ndarray:
    """A C-contiguous copy of `a` starting `off` elements into a larger buffer (misaligned)."""
    buf = np.empty(a.size + off, a.dtype)
    v = buf[off:off + a.size].reshape(a.shape)
    v[...] = a
    return v


@st.composite
def fir1d_case(draw):
    dtype = draw(st.sampled_from([np.uint8, np.int16]))
    ch = draw(st.sampled_from([1, 1, 1, 2, 2, 3]))
    L = draw(st.one_of(st.integers(1, 9), st.integers(10, 24), st.integers(25, 70)))
    rows = draw(st.one_of(st.just(1), st.integers(2, 40)))
    width = draw(st.one_of(st.integers(1, 64), st.integers(65, 3000), st.sampled_from([256, 512, 4096]),
                           st.integers(1, 300).map(lambda k: 8 * k)))
    frac = draw(st.one_of(st.just(12), st.integers(1, 31), st.integers(32, 40)))
    acc = draw(st.one_of(st.just(32), st.integers(max(1, frac - 4), 64)))
    stage = draw(st.sampled_from([fir_hip.OUT_U8_SAT, fir_hip.OUT_I32]))
    off = draw(st.sampled_from([0, 0, 0, 1, 3, 8]))
    seed = draw(st.integers(0, 2**32 - 1))
    return dtype, ch, _taps(draw, L), rows, width, frac, acc, stage, off, seed


@settings(max_examples=1000, **SETTINGS)
@given(fir1d_case())
def test_fir1d_rows_random_vs_oracle(case):
    dtype, ch, hq, rows, width, frac, acc, stage, off, seed = case
    info = np.iinfo(dtype)
    x = np.random.default_rng(seed).integers(info.min, info.max + 1, (rows, width * ch), dtype=dtype)
    xin = _unaligned(x, off)
    got = fir_hip.fir1d_fixed_rows(xin, hq, frac, acc, stage, channels=ch)
    ref = c_oracle().fir1d_rows(x, hq, frac, acc, stage, channels=ch)
    assert np.array_equal(got, ref)


@st.composite
def segment_case(draw):
    dtype = draw(st.sampled_from([np.uint8, np.int16]))
    ch = 1 if dtype == np.uint8 else draw(st.sampled_from([1, 2]))
    L = draw(st.integers(1, 9))
    tile = 4096 if dtype == np.uint8 else 512
    n = draw(st.one_of(st.integers(1, 3000), st.integers(1, 6).map(lambda k: k * tile // ch)))
    sides = draw(st.sampled_from(["both", "left", "right", "none"]))
    stage = draw(st.sampled_from([fir_hip.OUT_U8_SAT, fir_hip.OUT_I32]))
    seed = draw(st.integers(0, 2**32 - 1))
    return dtype, ch, _taps(draw, L), n, sides, stage, seed


@settings(max_examples=500, **SETTINGS)
@given(segment_case())
def test_segment_with_random_halos_vs_oracle(case):
    """fir1d_fixed_segment_dev (one shard of a longer row, the multi-GPU step): the halos stand
    in for the zero padding; = the oracle over the segment with the same halos."""
    dtype, ch, hq, n, sides, stage, seed = case
    info = np.iinfo(dtype)
    rng = np.random.default_rng(seed)
    L = len(hq)
    hl_n, hr_n = (L - 1 - L // 2) * ch, (L // 2) * ch
    x = rng.integers(info.min, info.max + 1, n * ch, dtype=dtype)
    hl = rng.integers(info.min, info.max + 1, hl_n, dtype=dtype) if sides in ("both", "left") and hl_n else None
    hr = rng.integers(info.min, info.max + 1, hr_n, dtype=dtype) if sides in ("both", "right") and hr_n else None
    xd = torch.from_numpy(x).to(DEV)
    got = torch_ops.fir1d_fixed_segment_dev(xd, hq, None if hl is None else torch.from_numpy(hl).to(DEV),
                                            None if hr is None else torch.from_numpy(hr).to(DEV), 12, 32, stage, ch)
    torch.cuda.synchronize()
    ref = c_oracle().fir1d_rows(x, hq, 12, 32, stage, channels=ch, halo_left=hl, halo_right=hr)
    assert np.array_equal(got.cpu().numpy(), ref)


@st.composite
def fir2d_case(draw):
    R = draw(st.integers(1, 7))
    C = draw(st.integers(1, 7))
    kind = draw(st.sampled_from(["outer", "outer", "small", "q412", "wide"]))
    if kind == "outer":  # exactly rank-1: the separable / packed-16 forms
        col = draw(st.lists(st.integers(-64, 64), min_size=R, max_size=R))
        row = draw(st.lists(st.integers(-64, 64), min_size=C, max_size=C))
        hq = (np.outer(col, row) * draw(st.sampled_from([1, 4, 16]))).tolist()
    else:
        lim = {"small": 8, "q412": 4096, "wide": 1 << 20}[kind]
        hq = np.asarray(draw(st.lists(st.integers(-lim, lim), min_size=R * C, max_size=R * C))).reshape(R, C).tolist()
    H = draw(st.one_of(st.integers(1, 40), st.integers(41, 140)))
    W = draw(st.one_of(st.integers(1, 80), st.integers(81, 700), st.sampled_from([1024, 1040])))
    frac = draw(st.one_of(st.just(12), st.integers(1, 22)))
    acc = draw(st.one_of(st.just(32), st.integers(16, 48)))
    stage = draw(st.sampled_from([fir_hip.OUT_U8_SAT, fir_hip.OUT_U8_SAT, fir_hip.OUT_I32]))
    frames = draw(st.sampled_from([0, 0, 1, 2, 3]))  # 0: one 2-D frame; else a (frames, H, W) batch
    seed = draw(st.integers(0, 2**32 - 1))
    return hq, H, W, frac, acc, stage, frames, seed


@settings(max_examples=600, **SETTINGS)
@given(fir2d_case())
def test_fir2d_random_vs_oracle(case):
    """2-D kernels, single frames and batches of frames (each frame zero padded on its own)."""
    hq, H, W, frac, acc, stage, frames, seed = case
    x = np.random.default_rng(seed).integers(0, 256, (frames, H, W) if frames else (H, W), dtype=np.uint8)
    got = fir_hip.fir2d_fixed(x, hq, frac, acc, stage)
    for f in range(max(frames, 1)):
        xf = x[f] if frames else x
        ref = c_oracle().fir2d(xf, np.asarray(hq), frac, acc, stage)
        assert np.array_equal(got[f] if frames else got, ref), f


@st.composite
def fir2d_mfma_case(draw):
    R = draw(st.sampled_from([3, 5]))
    C = draw(st.integers(1, 5))
    kind = draw(st.sampled_from(["byte", "byte", "pow2", "pair", "pair_wide"]))
    lim = {"byte": 127, "pow2": 127, "pair": 8192, "pair_wide": 32639}[kind]
    hq = np.asarray(draw(st.lists(st.integers(-lim - 1, lim), min_size=R * C, max_size=R * C))).reshape(R, C)
    if kind == "pow2":  # a common power of two moves into the shift
        hq = hq * (1 << draw(st.integers(1, 10)))
    H = draw(st.one_of(st.integers(1, 40), st.integers(41, 300)))
    W = 16 * draw(st.one_of(st.integers(1, 70), st.integers(63, 66), st.integers(120, 200)))
    frac = draw(st.one_of(st.just(12), st.integers(1, 24)))
    acc = draw(st.one_of(st.just(32), st.integers(12, 32)))
    frames = draw(st.sampled_from([0, 0, 1, 2, 3]))
    seed = draw(st.integers(0, 2**32 - 1))
    return hq.tolist(), H, W, frac, acc, frames, seed


@settings(max_examples=400, **SETTINGS)
@given(fir2d_mfma_case())
def test_fir2d_mfma_random_vs_oracle(case):
    """The 2-D matrix-core kernel forced on (FIR2D_PATH=mfma): one or two tap byte planes, a power
    of two factored into the shift, 16-byte rows around the 1024-pixel tile edges, any height
    (strips sized at launch), batches of frames, the fast byte-2 stage and the rounded wrap form."""
    hq, H, W, frac, acc, frames, seed = case
    x = np.random.default_rng(seed).integers(0, 256, (frames, H, W) if frames else (H, W), dtype=np.uint8)
    old = os.environ.get("FIR2D_PATH")
    os.environ["FIR2D_PATH"] = "mfma"
    try:
        got = fir_hip.fir2d_fixed(x, hq, frac, acc, fir_hip.OUT_U8_SAT)
    finally:
        if old is None:
            os.environ.pop("FIR2D_PATH")
        else:
            os.environ["FIR2D_PATH"] = old
    for f in range(max(frames, 1)):
        xf = x[f] if frames else x
        ref = c_oracle().fir2d(xf, np.asarray(hq), frac, acc, fir_hip.OUT_U8_SAT)
        assert np.array_equal(got[f] if frames else got, ref), f


@st.composite
def bank_case(draw):
    F = draw(st.integers(1, 6))
    L = draw(st.integers(1, 9))
    hq = [_taps(draw, L) for _ in range(F)]
    rows = draw(st.integers(1, 30))
    width = draw(st.one_of(st.integers(1, 100), st.sampled_from([640, 1280, 4096, 4499])))
    stage = draw(st.sampled_from([fir_hip.OUT_U8_SAT, fir_hip.OUT_I32]))
    seed = draw(st.integers(0, 2**32 - 1))
    return hq, rows, width, stage, seed


@settings(max_examples=300, **SETTINGS)
@given(bank_case())
def test_filter_bank_random_vs_oracle(case):
    """fir1d_fixed_rows_multi (F filters per read of x: byte-pair / packed-16 mixes) = the
    oracle filter by filter."""
    hq, rows, width, stage, seed = case
    x = np.random.default_rng(seed).integers(0, 256, (rows, width), dtype=np.uint8)
    got = fir_hip.fir1d_fixed_rows_multi(x, hq, 12, 32, stage)
    for f, h in enumerate(hq):
        assert np.array_equal(got[f], c_oracle().fir1d_rows(x, h, 12, 32, stage)), f


@st.composite
def ideal_case(draw):
    L = draw(st.integers(1, 11))
    h = draw(st.lists(st.one_of(st.floats(-8.0, 8.0, allow_nan=False, allow_infinity=False),
                                st.sampled_from([0.25, 0.5, -1.0, 1 / 3, 0.0, -0.0])), min_size=L, max_size=L))
    rows = draw(st.integers(1, 20))
    width = draw(st.one_of(st.integers(1, 64), st.integers(65, 2000)))
    seed = draw(st.integers(0, 2**32 - 1))
    return h, rows, width, seed


@settings(max_examples=400, **SETTINGS)
@given(ideal_case())
def test_ideal_random_vs_oracle(case):
    """float64 ideal model: products and sums rounded separately in k order, so equal to the
    oracle bit for bit (NaN-free inputs)."""
    h, rows, width, seed = case
    x = np.random.default_rng(seed).integers(0, 256, (rows, width), dtype=np.uint8)
    got = fir_hip.fir1d_ideal_rows(x, h)
    ref = c_oracle().fir1d_ideal_rows(x, h)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
