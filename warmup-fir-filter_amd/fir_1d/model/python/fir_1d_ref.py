"""Ideal (float64) FIR model and the shared input/coefficient validators.

Host-side mirror of the reference module ``fir_1d/model/python/fir_1d_ref.py``:
same public names, argument meaning, exception types and texts; the per-sample loop
(reference :55-63) runs as the HIP kernel ``fir1d_ideal_rows`` in libfir_hip.so.

Reference lines mirrored (paths relative to the reference root):
  MAX_ABS_H_COEFF            fir_1d_ref.py:6
  _validate_h_coefficients   fir_1d_ref.py:9-24   (empty / finite / |h| <= 8, first bad index wins)
  _validate_x                fir_1d_ref.py:27-33  (math.isfinite per element, first bad index wins)
  _round_half_up_x           fir_1d_ref.py:35-38  (math.floor(sample + 0.5))
  _clamp_x                   fir_1d_ref.py:40-41  ([0, 255])
  fir_1d_ideal               fir_1d_ref.py:43-65  (same-mode, centre-aligned, float64, no clamp)

Input contract.  The reference prepares ``x`` by iterating it: every element goes through
``math.isfinite``, then ``math.floor(s + 0.5)``, then the clamp.  Whatever that raises for an
input (TypeError for str / complex / None elements, for a scalar, a 0-d array or a 2-D array
with rows longer than 1; OverflowError for an int beyond the float range) is what the caller
gets here too, and whatever it accepts (bytes, ranges, generators, dicts, object arrays) gives
the same samples.  ``_prepare_x_u8`` reaches that result three ways:

  * a list / tuple / bytes / bytearray of ints in [0, 255]: one C-level ``bytearray`` copy
    (the reference row driver's ``row.tolist()`` of a uint8 image; nothing to round or clamp);
  * a 1-D ``numpy.ndarray`` of bool / integer / float16 / float32 / float64, and a list or
    tuple of Python ints / floats: vectorised, in the arithmetic the element-wise loop would
    use (a float32 sample plus the Python float 0.5 is a float32 sum under NumPy 2's
    promotion rules, so ``float32(0.49999997)`` rounds to 1, not 0);
  * anything else: the element-wise restatement below, which performs the reference's own
    operations on the same objects (so its exceptions and accepted inputs are the same).

Pinned by ``tests/golden/input_contract.json`` (outputs and exception texts recorded from the
reference itself, ``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import math
from collections.abc import Sequence

import numpy as np

import fir_hip

MAX_ABS_H_COEFF = 8.0

# ndarray dtypes whose element-wise preparation has a vectorised equivalent
_VEC_FLOAT = (np.dtype(np.float16), np.dtype(np.float32), np.dtype(np.float64))
_PY_NUMBER_TYPES = frozenset((int, float, bool, np.float64))
_BYTE_SEQUENCES = (list, tuple, bytes, bytearray)


def _validate_h_coefficients(h: Sequence[float]) -> None:
    """fir_1d_ref.py:9-24 — raises on the first offending coefficient, in index order."""
    if len(h) == 0:
        raise ValueError("Invalid h: h coefficients must not be empty.")
    for index, coeff in enumerate(h):
        if not math.isfinite(coeff):
            raise ValueError(f"Invalid h[{index}]={coeff}: h coefficients must be finite.")
        if abs(coeff) > MAX_ABS_H_COEFF:
            raise ValueError(f"Invalid h[{index}]={coeff}: |h| must be <= {MAX_ABS_H_COEFF}.")


def _validate_x(x) -> list:
    """fir_1d_ref.py:27-33: every element through math.isfinite (TypeError for non-real
    elements), ValueError at the first non-finite one; returns ``list(x)``."""
    for index, sample in enumerate(x):
        if not math.isfinite(sample):
            raise ValueError(f"Invalid x[{index}]={sample}: x must be finite.")
    return list(x)


def _round_half_up_x(x) -> list:
    """fir_1d_ref.py:35-38: math.floor(sample + 0.5), element by element."""
    return [math.floor(sample + 0.5) for sample in x]


def _clamp_x(x) -> list:
    """fir_1d_ref.py:40-41: clamp to [0, 255]."""
    return [max(0, min(255, sample)) for sample in x]


def _nonfinite_error(index: int, sample) -> ValueError:
    return ValueError(f"Invalid x[{index}]={sample}: x must be finite.")


def _prep_numeric_array(a: np.ndarray) -> np.ndarray:
    """Vectorised prep of a 1-D bool / integer / float16-64 ndarray, equal to the element-wise
    loop on its NumPy scalars: integers are finite and floor(i + 0.5) == i within [0, 255]
    (beyond it both sides clamp), floats round in their own precision."""
    if a.dtype == np.uint8:
        return np.ascontiguousarray(a)
    if a.dtype.kind == "b":
        return a.astype(np.uint8)
    if a.dtype.kind in "iu":
        return np.clip(a, 0, 255).astype(np.uint8)
    bad = ~np.isfinite(a)
    if bad.any():
        index = int(np.flatnonzero(bad)[0])
        raise _nonfinite_error(index, a[index])
    return np.clip(np.floor(a + a.dtype.type(0.5)), 0, 255).astype(np.uint8)


def _prep_float64(a: np.ndarray, samples) -> np.ndarray:
    """Vectorised prep of Python numbers already converted to float64 (the conversion the
    element-wise loop's ``sample + 0.5`` performs); ``samples`` supplies the reported element."""
    bad = ~np.isfinite(a)
    if bad.any():
        index = int(np.flatnonzero(bad)[0])
        raise _nonfinite_error(index, samples[index])
    return np.clip(np.floor(a + 0.5), 0, 255).astype(np.uint8)


def _prepare_generic(x) -> np.ndarray:
    """The reference chain as written (fir_1d_ref.py:27-41, then fir_1d_fixed_ref.py:75)."""
    return np.array(_clamp_x(_round_half_up_x(_validate_x(x))), dtype=np.uint8)


def _prepare_x_u8(x) -> np.ndarray:
    """Validation + round-half-up + clamp + uint8 cast (fir_1d_fixed_ref.py:34-36,75) with the
    reference's exceptions; see the module docstring for the three routes."""
    t = type(x)
    if t in _BYTE_SEQUENCES:
        try:
            return np.frombuffer(bytearray(x), dtype=np.uint8)
        except (TypeError, ValueError):
            pass
        if t in (list, tuple) and set(map(type, x)) <= _PY_NUMBER_TYPES:
            try:
                a = np.array(x, dtype=np.float64)
            except OverflowError:  # an int beyond float range: let the loop raise it in order
                return _prepare_generic(x)
            return _prep_float64(a, x)
    elif t is np.ndarray and x.ndim == 1 and (x.dtype.kind in "biu" or x.dtype in _VEC_FLOAT):
        return _prep_numeric_array(x)
    return _prepare_generic(x)


def _prepare_rows_u8(x: np.ndarray, after_row0=None) -> np.ndarray:
    """Per-row preparation of an H x W image, as the reference row drivers do it: each row
    goes through the model as ``row.tolist()`` (gen_fixed_output.py:44-52,
    gen_ideal_output.py:40-42), so float rows are prepared in float64 (``tolist`` widens
    float16 / float32 exactly) and a non-finite sample is reported with its index in its row.
    ``after_row0`` runs once row 0 is prepared and before any later row: the checks the model
    performs after its x preparation (bits / Q-range), which therefore win over a bad sample
    in rows 1..H-1 but not over one in row 0.  Returns a C-contiguous uint8 image."""
    height = x.shape[0]
    exact = type(x) is np.ndarray  # a subclass (masked array ...) takes the row-by-row path
    if exact and x.dtype == np.uint8:
        if after_row0 is not None:
            after_row0()
        return np.ascontiguousarray(x)
    if exact and x.dtype.kind in "biu":
        if after_row0 is not None:
            after_row0()
        return np.ascontiguousarray(np.clip(x, 0, 255).astype(np.uint8))
    out = np.empty(x.shape, dtype=np.uint8)
    if exact and x.dtype in _VEC_FLOAT:
        a = x.astype(np.float64)
        bad = ~np.isfinite(a)
        bad_rows = np.flatnonzero(bad.any(axis=1)) if bad.any() else np.zeros(0, np.int64)
        first_bad = int(bad_rows[0]) if bad_rows.size else height
        if first_bad == 0 < height:
            col = int(np.flatnonzero(bad[0])[0])
            raise _nonfinite_error(col, float(a[0, col]))
        if after_row0 is not None:
            after_row0()
        if first_bad < height:
            col = int(np.flatnonzero(bad[first_bad])[0])
            raise _nonfinite_error(col, float(a[first_bad, col]))
        out[...] = np.clip(np.floor(a + 0.5), 0, 255)
        return out
    for r in range(height):
        out[r] = _prepare_generic(x[r, :].tolist())
        if r == 0 and after_row0 is not None:
            after_row0()
    return out


def fir_1d_ideal(x: Sequence[int | float], h: Sequence[float]) -> list[float]:
    """fir_1d_ref.py:43-65 on the GPU: y[n] = sum_k h[k] * x_sat[n - k + L//2] in float64."""
    _validate_h_coefficients(h)
    x_sat = _prepare_x_u8(x)
    if x_sat.size == 0:
        return []
    y = fir_hip.fir1d_ideal_rows(x_sat, [float(v) for v in h])
    return y.tolist()
