#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer C-ABI entries (DESIGN.md §5 note).

The bench `value` is measured with inputs resident in HBM; the reference-facing host API
(fir1d_fixed_rows & co.) copies NumPy arrays in and out over PCIe on every call.  This
times those calls: H2D + kernel + D2H, synchronous, best of 5.
"""
from __future__ import annotations

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
    return min(ts)


def main():
    rng = np.random.default_rng(20260227)
    out = {}
    x = rng.integers(-32768, 32768, 1 << 28, dtype=np.int16)
    t = best(lambda: fir_hip.fir1d_fixed_rows(x, [-256, -1024, 6656, -1024, -256], 12, 32, fir_hip.OUT_I32))
    out["fir1d_fixed_rows int16->int32 2^28 (512 MiB in, 1 GiB out)"] = {
        "seconds": round(t, 4), "gsamples_per_s": round(x.size / t / 1e9, 3), "pcie_gb_per_s": round(6 * x.size / t / 1e9, 2)}
    imgs = np.load(ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz")
    ims = [imgs[k] for k in sorted(imgs.files)]
    n = sum(a.size for a in ims)
    hq = [-256, -1024, 6656, -1024, -256]
    t = best(lambda: [fir_hip.fir1d_fixed_rows(a, hq) for a in ims])
    out["fir1d_fixed_rows u8 7 golden images, one call each"] = {
        "seconds": round(t, 5), "msamples_per_s": round(n / t / 1e6, 1)}
    bank = np.array([[1365] * 3, [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]])
    t = best(lambda: [fir_hip.fir1d_fixed_rows_multi(a, bank) for a in ims])
    out["fir1d_fixed_rows_multi u8 7 images x 4 filters (3-tap bank)"] = {
        "seconds": round(t, 5), "msamples_per_s": round(4 * n / t / 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
