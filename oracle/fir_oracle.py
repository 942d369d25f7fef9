"""CPU oracle for the fixed-point FIR hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``fir_hip`` + the ``fir_1d`` host mirror) never calls it and
fails loudly when the HIP library is missing.

It is a vectorised NumPy restatement of the reference algorithm, written from
the reference's behaviour, and pinned by ``tests/golden/*`` (vectors produced by
running the reference itself; see ``tests/golden/make_golden.py``).

Reference lines restated (paths relative to the reference root):
  quantize_h      fir_1d/model/python/fir_1d_fixed_ref.py:54-81  (Q range, rint ties-to-even, clip)
  prep_x          fir_1d/model/python/fir_1d_ref.py:35-41        (floor(x+0.5), clamp [0,255])
                  fir_1d/model/python/fir_1d_fixed_ref.py:75     (cast to uint8)
  wrap_round      fir_1d/model/python/fir_1d_fixed_ref.py:94,110-120 (mask to acc_bits,
                  sign-extend, + 2^(f-1), arithmetic >> f)
  fir1d_loop      fir_1d/model/python/fir_1d_fixed_ref.py:94-128 as its per-sample Python loop
                  (the reference's CPU cost, timed by bench.py on a small sample)
  fir1d_rows      fir_1d/model/python/fir_1d_fixed_ref.py:95-128 (same-mode, centre-aligned,
                  zero-padded MAC, saturate :123-126) applied per row as in
                  fir_1d/sim/vector/gen_fixed_output.py:34-60
  fir1d_ideal_rows fir_1d/model/python/fir_1d_ref.py:43-65 (float64, k-order sum, no clamp)
                  per row as in fir_1d/sim/vector/gen_ideal_output.py:37-50
  compute_metrics fir_1d/sim/vector/gen_3tap_compare_report.py:67-112
  to_u8_clip      fir_1d/sim/vector/restore_images.py:51-54 (rint, clip, cast)
  to_u8_normalized fir_1d/sim/vector/restore_images.py:57-64 (min/max rescale)

Variants the reference does not have are defined here by
the same arithmetic:
  a6 int16 -> int32: input clamp (fir_1d_fixed_ref.py:36) bypassed and
     saturation (:123-126) dropped: out = (wrap(acc) + 2^(f-1)) >> f as int32.
  a7 complex int16 (lib/mycomplex.h: complex x real scalar only): real taps
     applied to the re and im channels of interleaved (re, im) samples.
  a8 fir_2d: y[i,j] = stage(wrap(sum_m sum_n hq[m,n] x[i-m+R//2, j-n+C//2])),
     zero padded, the 2-D extension of the centre-aligned rule
     (fir_1d/docs/fir_1d_golden_spec_v1.md:65-74).

Index convention (all paths): y[n] = sum_k hq[k] * x[n - k + c], c = L // 2, so
an output needs HL = L-1-c samples on its left and HR = c on its right.
"""
from __future__ import annotations

import numpy as np

OUT_U8_SAT = 0
OUT_I32 = 1


def halo_sizes(L: int) -> tuple[int, int]:
    """(left, right) halo sample counts for an L-tap centre-aligned filter."""
    c = L // 2
    return L - 1 - c, c


def quantize_h(h, frac_bits: int = 12, coeff_bits: int = 16) -> np.ndarray:
    """fir_1d_fixed_ref.py:54-81: hq = clip(rint(h * 2^f), MIN, MAX) (ties-to-even)."""
    lo = -(1 << (coeff_bits - 1))
    hi = (1 << (coeff_bits - 1)) - 1
    hf = np.rint(np.asarray(h, dtype=np.float64) * (1 << frac_bits))
    return np.clip(hf, lo, hi).astype(np.int64)


def prep_x(x) -> np.ndarray:
    """fir_1d_ref.py:35-41 + fir_1d_fixed_ref.py:75 for finite input: floor(x+0.5), clamp, u8."""
    a = np.asarray(x)
    if a.dtype == np.uint8:
        return a.copy()
    a = a.astype(np.float64)
    return np.clip(np.floor(a + 0.5), 0, 255).astype(np.uint8)


def wrap_round(acc: np.ndarray, frac_bits: int, acc_bits: int) -> np.ndarray:
    """fir_1d_fixed_ref.py:94,110-120 on int64 sums: exact mod 2^64 (all the wrap to
    acc_bits < 64 needs) or, for acc_bits >= 64, the exact sum (|acc| < 2^63).  The reference's
    (v + 2^(f-1)) >> f on unbounded ints equals (v >> f) + bit (f-1) of v, which cannot
    overflow; for f >= 64 it is 0 for every |v| < 2^63."""
    acc = np.asarray(acc, dtype=np.int64)
    if acc_bits < 64:
        s = np.uint64(64 - acc_bits)
        acc = ((acc.astype(np.uint64) << s).view(np.int64)) >> np.int64(64 - acc_bits)
    if frac_bits >= 64:
        return np.zeros_like(acc)
    return (acc >> np.int64(frac_bits)) + ((acc >> np.int64(frac_bits - 1)) & np.int64(1))


def _stage(q: np.ndarray, out_stage: int) -> np.ndarray:
    if out_stage == OUT_U8_SAT:
        return np.clip(q, 0, 255).astype(np.uint8)  # fir_1d_fixed_ref.py:123-126
    if out_stage == OUT_I32:
        return q.astype(np.int32)
    raise ValueError(f"unknown out_stage {out_stage}")


def _mac_rows(x2: np.ndarray, hq: np.ndarray, left: np.ndarray | None = None,
              right: np.ndarray | None = None) -> np.ndarray:
    """Exact int64 sum_k hq[k] * x[n - k + c] over each row (last axis), zero padded
    unless halo rows are given (left: [..., HL], right: [..., HR])."""
    L = len(hq)
    HL, HR = halo_sizes(L)
    rows, n = x2.shape
    lpad = np.zeros((rows, HL), np.int64) if left is None else np.asarray(left, np.int64).reshape(rows, HL)
    rpad = np.zeros((rows, HR), np.int64) if right is None else np.asarray(right, np.int64).reshape(rows, HR)
    xp = np.concatenate([lpad, x2.astype(np.int64), rpad], axis=1)
    acc = np.zeros((rows, n), np.int64)
    with np.errstate(over="ignore"):  # int64 arithmetic wraps mod 2^64, which is what wrap_round needs
        for k in range(L):
            # x[n - k + c] sits at xp[n - k + c + HL] = xp[n + (L - 1) - k]
            off = L - 1 - k
            acc += np.int64(hq[k]) * xp[:, off:off + n]
    return acc


def fir1d_rows(x, hq, frac_bits: int = 12, acc_bits: int = 32, out_stage: int = OUT_U8_SAT,
               channels: int = 1, halo_left=None, halo_right=None) -> np.ndarray:
    """Row-wise same-mode fixed FIR.  ``x``: (..., W*channels) integer samples; rows are
    independent (zero padding resets at every row edge).  ``channels`` > 1 means
    interleaved channels (complex = 2) filtered independently with the same taps."""
    x = np.asarray(x)
    shape = x.shape
    hq = np.asarray(hq, dtype=np.int64)
    if x.size == 0:
        return np.zeros(shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32)
    x2 = x.reshape(-1, shape[-1]) if x.ndim else x.reshape(1, 1)
    rows, wc = x2.shape
    if wc % channels:
        raise ValueError("row length not a multiple of channels")
    w = wc // channels
    # de-interleave channels into independent rows
    xc = x2.reshape(rows, w, channels).transpose(0, 2, 1).reshape(rows * channels, w)
    L = len(hq)
    HL, HR = halo_sizes(L)
    lh = rh = None
    if halo_left is not None:
        lh = np.asarray(halo_left).reshape(rows, HL, channels).transpose(0, 2, 1).reshape(rows * channels, HL)
    if halo_right is not None:
        rh = np.asarray(halo_right).reshape(rows, HR, channels).transpose(0, 2, 1).reshape(rows * channels, HR)
    acc = _mac_rows(xc, hq, lh, rh)
    q = wrap_round(acc, frac_bits, acc_bits)
    y = _stage(q, out_stage)
    y = y.reshape(rows, channels, w).transpose(0, 2, 1).reshape(shape)
    return np.ascontiguousarray(y)


def fir1d_loop(x, hq, frac_bits: int = 12, acc_bits: int = 32, out_stage: int = OUT_U8_SAT) -> list:
    """The reference's own per-sample x per-tap Python loop (fir_1d_fixed_ref.py:94-128) over
    one row, as plain Python ints: bounds-checked zero padding, mask to acc_bits, sign
    restore, + 2^(f-1), >> f, then saturation (OUT_U8_SAT) or none (OUT_I32, variant a6).
    Only for small inputs: bench.py times it to show what the reference's CPU path costs."""
    xs = [int(v) for v in x]
    hs = [int(v) for v in hq]
    n_x, n_h, c = len(xs), len(hs), len(hs) // 2
    mask, sign, bias = (1 << acc_bits) - 1, 1 << (acc_bits - 1), 1 << (frac_bits - 1)
    out = []
    for n in range(n_x):
        acc = 0
        for k in range(n_h):
            i = n - k + c
            acc += (xs[i] if 0 <= i < n_x else 0) * hs[k]
        acc &= mask
        if acc & sign:
            acc -= 1 << acc_bits
        v = (acc + bias) >> frac_bits
        if out_stage == OUT_U8_SAT:
            v = 0 if v < 0 else (255 if v > 255 else v)
        out.append(v)
    return out


def fir_1d_fixed_golden(x, h, frac_bits: int = 12, acc_bits: int = 32, coeff_bits: int = 16) -> np.ndarray:
    """Whole reference pipeline for valid inputs (validation is the host's job)."""
    xu = prep_x(x).reshape(-1)
    hq = quantize_h(h, frac_bits, coeff_bits)
    if xu.size == 0:
        return np.zeros(0, np.uint8)
    return fir1d_rows(xu, hq, frac_bits, acc_bits, OUT_U8_SAT)


def fir1d_i16_i32(x, hq, frac_bits: int = 12, acc_bits: int = 32, halo_left=None, halo_right=None,
                  channels: int = 1) -> np.ndarray:
    """a6 / a7: int16 (or interleaved complex-int16) -> int32, no saturation."""
    return fir1d_rows(np.asarray(x, np.int16).reshape(1, -1), hq, frac_bits, acc_bits, OUT_I32,
                      channels=channels, halo_left=halo_left, halo_right=halo_right).reshape(-1)


def fir2d_fixed(x, hq2, frac_bits: int = 12, acc_bits: int = 32, out_stage: int = OUT_U8_SAT) -> np.ndarray:
    """a8: y[i,j] = stage(wrap(sum_m sum_n hq[m,n] * x[i - m + R//2, j - n + C//2]))."""
    x = np.asarray(x)
    hq2 = np.asarray(hq2, dtype=np.int64)
    R, C = hq2.shape
    H, W = x.shape
    tL, tR = halo_sizes(R)  # rows above / below
    lL, lR = halo_sizes(C)
    xp = np.zeros((H + R - 1, W + C - 1), np.int64)
    xp[tL:tL + H, lL:lL + W] = x
    acc = np.zeros((H, W), np.int64)
    for m in range(R):
        for n in range(C):
            acc += hq2[m, n] * xp[R - 1 - m:R - 1 - m + H, C - 1 - n:C - 1 - n + W]
    return _stage(wrap_round(acc, frac_bits, acc_bits), out_stage)


def fir1d_ideal_rows(x, h) -> np.ndarray:
    """fir_1d_ref.py:43-65 per row: float64 acc, k-order, no FMA, no clamp.  Adding the
    zero-padded terms instead of skipping them is bit-identical (acc never becomes -0.0)."""
    x = prep_x(x) if np.asarray(x).dtype != np.uint8 else np.asarray(x)
    shape = x.shape
    if x.size == 0:
        return np.zeros(shape, np.float64)
    x2 = x.reshape(-1, shape[-1]) if x.ndim else x.reshape(1, 1)
    rows, n = x2.shape
    h = [float(v) for v in h]
    L = len(h)
    HL, HR = halo_sizes(L)
    xp = np.zeros((rows, n + L - 1), np.float64)
    xp[:, HL:HL + n] = x2
    acc = np.zeros((rows, n), np.float64)
    for k in range(L):
        off = L - 1 - k
        acc = acc + h[k] * xp[:, off:off + n]
    return acc.reshape(shape)


def compute_metrics(y_ideal, y_fixed) -> dict:
    """gen_3tap_compare_report.py:67-112 (same numpy reductions, same order)."""
    ideal = np.asarray(y_ideal).astype(np.float64, copy=False)
    fixed_u8 = np.asarray(y_fixed)
    fixed = fixed_u8.astype(np.float64, copy=False)
    d = fixed - ideal
    ad = np.abs(d)
    n = ideal.size
    lo = float(np.mean(fixed_u8.reshape(-1) == 0)) if n else 0.0
    hi = float(np.mean(fixed_u8.reshape(-1) == 255)) if n else 0.0
    return {
        "num_samples": int(n),
        "max_abs_err": float(ad.max()) if n else 0.0,
        "mae": float(ad.mean()) if n else 0.0,
        "rmse": float(np.sqrt(np.mean(np.square(d)))) if n else 0.0,
        "mean_err": float(d.mean()) if n else 0.0,
        "sat_low_ratio": lo,
        "sat_high_ratio": hi,
        "sat_ratio": lo + hi,
        "clip_needed_ratio": float(np.mean((ideal < 0.0) | (ideal > 255.0))) if n else 0.0,
    }


def to_u8_clip(a) -> np.ndarray:
    """restore_images.py:51-54."""
    return np.clip(np.rint(np.asarray(a, np.float64)), 0, 255).astype(np.uint8)


def to_u8_normalized(a) -> np.ndarray:
    """restore_images.py:57-64."""
    a = np.asarray(a, np.float64)
    lo, hi = float(a.min()), float(a.max())
    if hi <= lo:
        return np.zeros(a.shape, dtype=np.uint8)
    return np.rint(np.clip((a - lo) * (255.0 / (hi - lo)), 0, 255)).astype(np.uint8)
