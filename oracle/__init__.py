"""CPU oracle package — TEST INFRASTRUCTURE ONLY.

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, as the checker.  The product path never imports it.

* ``oracle.fir_oracle``  — vectorised NumPy restatement (reference file:line cited there)
* ``oracle.c_oracle()``  — ctypes handle on ``oracle/_build/liboracle_fir.so`` (the C
  restatement in ``oracle/fir_oracle.c``, OpenMP), used for large sizes and as the
  CPU baseline; build it with ``make -C oracle``.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

from . import fir_oracle  # noqa: F401

_HERE = Path(__file__).resolve().parent
_LIB = None


class COracle:
    IN_U8, IN_I16 = 0, 1
    OUT_U8_SAT, OUT_I32 = 0, 1

    def __init__(self, path: Path):
        lib = ctypes.CDLL(str(path))
        i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        lib.oracle_fir1d_rows.argtypes = [vp, i32, i64, i64, i32, vp, i32, i32, i32, i32, vp, vp, vp, i32]
        lib.oracle_fir1d_rows.restype = i32
        lib.oracle_fir2d.argtypes = [vp, i64, i64, vp, i32, i32, i32, i32, i32, vp, i32]
        lib.oracle_fir2d.restype = i32
        lib.oracle_fir1d_ideal_rows.argtypes = [vp, i64, i64, vp, i32, vp, i32]
        lib.oracle_fir1d_ideal_rows.restype = i32
        self.lib = lib

    @staticmethod
    def _p(a):
        return None if a is None else a.ctypes.data_as(ctypes.c_void_p)

    def fir1d_rows(self, x, hq, frac_bits=12, acc_bits=32, out_stage=0, channels=1,
                   halo_left=None, halo_right=None, nthreads=0):
        x = np.ascontiguousarray(x)
        if x.dtype == np.uint8:
            in_dtype = self.IN_U8
        elif x.dtype == np.int16:
            in_dtype = self.IN_I16
        else:
            raise TypeError(x.dtype)
        x2 = x.reshape(-1, x.shape[-1]) if x.ndim > 1 else x.reshape(1, -1)
        rows, wc = x2.shape
        hq32 = np.ascontiguousarray(hq, dtype=np.int32)
        y = np.empty(x.shape, np.uint8 if out_stage == self.OUT_U8_SAT else np.int32)
        hl = None if halo_left is None else np.ascontiguousarray(halo_left, dtype=x.dtype)
        hr = None if halo_right is None else np.ascontiguousarray(halo_right, dtype=x.dtype)
        rc = self.lib.oracle_fir1d_rows(self._p(x2), in_dtype, rows, wc // channels, channels,
                                        self._p(hq32), len(hq32), frac_bits, acc_bits, out_stage,
                                        self._p(hl), self._p(hr), self._p(y), nthreads)
        if rc:
            raise ValueError("oracle_fir1d_rows rejected its arguments")
        return y

    def fir2d(self, x, hq2, frac_bits=12, acc_bits=32, out_stage=0, nthreads=0):
        x = np.ascontiguousarray(x, dtype=np.uint8)
        hq2 = np.ascontiguousarray(hq2, dtype=np.int32)
        R, C = hq2.shape
        H, W = x.shape
        y = np.empty(x.shape, np.uint8 if out_stage == self.OUT_U8_SAT else np.int32)
        rc = self.lib.oracle_fir2d(self._p(x), H, W, self._p(hq2), R, C, frac_bits, acc_bits,
                                   out_stage, self._p(y), nthreads)
        if rc:
            raise ValueError("oracle_fir2d rejected its arguments")
        return y

    def fir1d_ideal_rows(self, x_u8, h, nthreads=0):
        x = np.ascontiguousarray(x_u8, dtype=np.uint8)
        x2 = x.reshape(-1, x.shape[-1]) if x.ndim > 1 else x.reshape(1, -1)
        hh = np.ascontiguousarray(h, dtype=np.float64)
        y = np.empty(x.shape, np.float64)
        rc = self.lib.oracle_fir1d_ideal_rows(self._p(x2), x2.shape[0], x2.shape[1], self._p(hh),
                                              len(hh), self._p(y), nthreads)
        if rc:
            raise ValueError("oracle_fir1d_ideal_rows rejected its arguments")
        return y


def c_oracle() -> COracle:
    """Load (building on first use if a compiler is present) the C oracle."""
    global _LIB
    if _LIB is None:
        path = _HERE / "_build" / "liboracle_fir.so"
        if not path.exists():
            import subprocess
            subprocess.run(["make", "-C", str(_HERE)], check=True, capture_output=True)
        _LIB = COracle(path)
    return _LIB
