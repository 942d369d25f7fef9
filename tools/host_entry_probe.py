#!/usr/bin/env python3
"""Where a host-pointer call's time goes (2^28 int16 -> int32): the whole NumPy entry, a
fresh 1 GiB output's first-touch cost alone, the C entry into an already-touched output, and
the NumPy entry given that output as ``out=``."""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "warmup-fir-filter_amd"))

import numpy as np  # noqa: E402

import fir_hip  # noqa: E402


def best(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 2)


def main():
    x = np.random.default_rng(20260227).integers(-32768, 32768, 1 << 28, dtype=np.int16)
    hq = [-256, -1024, 6656, -1024, -256]
    h = np.asarray(hq, np.int32)
    y = np.zeros(x.size, np.int32)
    vp = ctypes.c_void_p
    L = fir_hip.lib()

    def direct():
        rc = L.fir1d_fixed_rows(vp(x.ctypes.data), fir_hip.IN_I16, 1, x.size, 1, vp(h.ctypes.data), 5, 12, 32,
                                fir_hip.OUT_I32, vp(y.ctypes.data), 0)
        assert rc == 0
    out = {
        "numpy_entry_ms": best(lambda: fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32)),
        "fresh_1GiB_output_first_touch_ms": best(lambda: np.empty(x.size, np.int32).fill(0)),
        "c_entry_touched_output_ms": best(direct),
        "numpy_entry_reused_out_ms": best(lambda: fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32, out=y)),
    }
    out["pcie_bytes"] = 6 * x.size
    print(json.dumps(out))


if __name__ == "__main__":
    main()
