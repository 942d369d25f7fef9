"""Ideal (float64) FIR model and the shared input/coefficient validators.

Host-side mirror of the reference module ``fir_1d/model/python/fir_1d_ref.py``:
same public names, argument meaning and ``ValueError`` texts; the per-sample loop
(reference :55-63) runs as the HIP kernel ``fir1d_ideal_rows`` in libfir_hip.so.

Reference lines mirrored (paths relative to the reference root):
  MAX_ABS_H_COEFF            fir_1d_ref.py:6
  _validate_h_coefficients   fir_1d_ref.py:9-24   (empty / finite / |h| <= 8, first bad index wins)
  _validate_x                fir_1d_ref.py:27-33  (finite, first bad index wins)
  _round_half_up_x           fir_1d_ref.py:35-38  (floor(x + 0.5))
  _clamp_x                   fir_1d_ref.py:40-41  ([0, 255])
  fir_1d_ideal               fir_1d_ref.py:43-65  (same-mode, centre-aligned, float64, no clamp)
"""
from __future__ import annotations

import math
from collections.abc import Sequence

import numpy as np

import fir_hip

MAX_ABS_H_COEFF = 8.0


def _validate_h_coefficients(h: Sequence[float]) -> None:
    """fir_1d_ref.py:9-24 — raises on the first offending coefficient, in index order."""
    if len(h) == 0:
        raise ValueError("Invalid h: h coefficients must not be empty.")
    for index, coeff in enumerate(h):
        if not math.isfinite(coeff):
            raise ValueError(f"Invalid h[{index}]={coeff}: h coefficients must be finite.")
        if abs(coeff) > MAX_ABS_H_COEFF:
            raise ValueError(f"Invalid h[{index}]={coeff}: |h| must be <= {MAX_ABS_H_COEFF}.")


def _validate_x(x) -> np.ndarray:
    """fir_1d_ref.py:27-33, vectorised.  Returns the samples as an ndarray (uint8 input is
    passed through untouched; everything else as float64)."""
    a = np.asarray(x)
    if a.dtype == np.uint8 or a.dtype.kind in "iub":
        return a.reshape(-1)
    af = a.astype(np.float64).reshape(-1)
    bad = ~np.isfinite(af)
    if bad.any():
        index = int(np.flatnonzero(bad)[0])
        sample = x[index] if not isinstance(x, np.ndarray) else a.reshape(-1)[index]
        raise ValueError(f"Invalid x[{index}]={sample}: x must be finite.")
    return af


def _round_half_up_x(x: np.ndarray) -> np.ndarray:
    """fir_1d_ref.py:35-38: floor(x + 0.5) (integer input is unchanged)."""
    a = np.asarray(x)
    if a.dtype.kind in "iub":
        return a
    return np.floor(a + 0.5)


def _clamp_x(x: np.ndarray) -> np.ndarray:
    """fir_1d_ref.py:40-41: clamp to [0, 255]."""
    a = np.asarray(x)
    if a.dtype == np.uint8:
        return a
    return np.clip(a, 0, 255)


def _prepare_x_u8(x) -> np.ndarray:
    """Validation + round-half-up + clamp + uint8 cast (fir_1d_fixed_ref.py:34-36,75).

    A list / tuple whose samples are all ints in [0, 255] (the reference's row driver passes
    ``row.tolist()`` of a uint8 image, gen_fixed_output.py:44-52) has nothing to validate,
    round or clamp: it converts in one C loop (bytearray), ~15x faster than np.asarray of the
    list; any other list (floats, values outside [0, 255]) takes the general path below."""
    if isinstance(x, (list, tuple)):
        try:
            return np.frombuffer(bytearray(x), dtype=np.uint8)
        except (TypeError, ValueError):
            pass
    x1 = _validate_x(x)
    return np.ascontiguousarray(_clamp_x(_round_half_up_x(x1)), dtype=np.uint8)


def fir_1d_ideal(x: Sequence[int | float], h: Sequence[float]) -> list[float]:
    """fir_1d_ref.py:43-65 on the GPU: y[n] = sum_k h[k] * x_sat[n - k + L//2] in float64."""
    _validate_h_coefficients(h)
    x_sat = _prepare_x_u8(x)
    if x_sat.size == 0:
        return []
    y = fir_hip.fir1d_ideal_rows(x_sat, [float(v) for v in h])
    return y.tolist()
