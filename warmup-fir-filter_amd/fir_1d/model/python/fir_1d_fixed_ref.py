"""Fixed-point (Q-format) FIR golden model — host side of the MI355X path.

Mirror of the reference module ``fir_1d/model/python/fir_1d_fixed_ref.py``: the
public function keeps its signature, return contract (1-D ``uint8`` ndarray, same
length as ``x``) and ``ValueError`` texts; validation and coefficient quantization
stay on the host exactly as in the reference, and the per-sample x per-tap MAC loop
(reference :95-128) runs as the gfx950 kernel behind ``fir1d_fixed_rows`` in
libfir_hip.so.  There is no CPU fallback: without the library or a gfx950 device the
call raises ``fir_hip.FirHipError``.

Reference lines mirrored (paths relative to the reference root):
  validation order          fir_1d_fixed_ref.py:33-47 (h, then x, then frac/acc/coeff bits;
                            x's own contract is fir_1d_ref._prepare_x_u8)
  Q-format range check      fir_1d_fixed_ref.py:52-72
  quantization              fir_1d_fixed_ref.py:78-81 (np.rint ties-to-even, clip, cast)
  MAC / wrap / round / sat  fir_1d_fixed_ref.py:95-126 (device kernel)
"""
from __future__ import annotations

import numpy as np
import numpy.typing as npt

import fir_hip

from .fir_1d_ref import _prepare_x_u8, _validate_h_coefficients

MAX_ABS_H_COEFF = 8.0

_VALID_COEFF_BITS = (8, 16, 32)
_DTYPE_H = {8: np.int8, 16: np.int16, 32: np.int32}


def _check_bits(frac_bits: int, acc_bits: int, coeff_bits: int) -> None:
    """fir_1d_fixed_ref.py:39-47."""
    if frac_bits <= 0:
        raise ValueError(f"Invalid frac_bits={frac_bits}. frac_bits must be > 0.")
    if acc_bits <= 0:
        raise ValueError(f"Invalid acc_bits={acc_bits}. acc_bits must be > 0.")
    if coeff_bits not in _VALID_COEFF_BITS:
        raise ValueError(
            f"Invalid coeff_bits={coeff_bits}. coeff_bits must be one of {_VALID_COEFF_BITS}."
        )


def _quantize_checked(h, frac_bits: int, coeff_bits: int) -> np.ndarray:
    """fir_1d_fixed_ref.py:52-81: Q-range check, then rint / clip / cast.  Returns int32 taps."""
    min_coeff = -(1 << (coeff_bits - 1))
    max_coeff = (1 << (coeff_bits - 1)) - 1
    scale = 1 << frac_bits
    min_real = min_coeff / scale
    max_real = max_coeff / scale
    for index, coeff in enumerate(h):
        if coeff < min_real or coeff > max_real:
            raise ValueError(
                f"Invalid h[{index}]={coeff}: out of Q-format real range "
                f"[{min_real}, {max_real}]."
            )
    hf = np.rint(np.array(h, dtype=np.float64) * scale)
    hf = np.clip(hf, min_coeff, max_coeff)
    return hf.astype(_DTYPE_H[coeff_bits]).astype(np.int32)


def _coeff_stage(h, frac_bits, acc_bits, coeff_bits) -> np.ndarray:
    """What fir_1d_fixed_golden does between its x preparation and its MAC loop
    (fir_1d_fixed_ref.py:39-94): bit-width checks, Q-range check, quantization, and the
    accumulator mask ``1 << acc_bits`` (:94), which raises TypeError for a non-integer
    acc_bits even when x is empty.  Returns int32 taps."""
    _check_bits(frac_bits, acc_bits, coeff_bits)
    hq = _quantize_checked(h, frac_bits, coeff_bits)
    if not isinstance(acc_bits, (int, np.integer)):
        1 << acc_bits  # noqa: B018 -- the reference's own TypeError for float / Fraction widths
    return hq


def quantize_fixed_taps(h, frac_bits: int = 12, acc_bits: int = 32, coeff_bits: int = 16) -> np.ndarray:
    """All coefficient-side checks of fir_1d_fixed_golden, in the reference's order, for a
    caller whose samples are already uint8 (so the x checks cannot fail): returns int32 taps."""
    _validate_h_coefficients(h)
    return _coeff_stage(h, frac_bits, acc_bits, coeff_bits)


def device_bits(frac_bits: int, acc_bits: int) -> tuple[int, int]:
    """Clamp the bit widths to what changes the result (the exact sum |acc| < 2^127 for any tap
    count up to FIR_MAX_TAPS): acc_bits >= 128 never wraps, frac_bits >= 128 always rounds to 0;
    the library sums in 64 bits while that is exact and in 128 bits otherwise."""
    return min(int(frac_bits), 128), min(int(acc_bits), 128)


def fir_1d_fixed_golden(
    x,
    h,
    frac_bits: int = 12,
    acc_bits: int = 32,
    coeff_bits: int = 16,
) -> npt.NDArray[np.uint8]:
    """Hardware-behaviour model of the 1-D fixed-point FIR (fir_1d_fixed_ref.py:12-130).

    Args:
        x: input pixels (int | float), rounded half-up and clamped to [0, 255].
        h: real-valued taps, quantized to Q(coeff_bits - frac_bits).frac_bits.
        frac_bits: fraction bits of the coefficients (default 12).
        acc_bits: accumulator width; the exact sum wraps to this many bits (default 32).
        coeff_bits: coefficient width, one of 8 / 16 / 32 (default 16).

    Returns:
        uint8 ndarray of len(x): saturate(((wrap(acc) + 2^(f-1)) >> f)).
    """
    _validate_h_coefficients(h)
    x_u8 = _prepare_x_u8(x)
    hq = _coeff_stage(h, frac_bits, acc_bits, coeff_bits)
    if x_u8.size == 0:
        return np.zeros(0, dtype=np.uint8)
    f, a = device_bits(frac_bits, acc_bits)
    return fir_hip.fir1d_fixed_rows(x_u8, hq, f, a, fir_hip.OUT_U8_SAT)
