"""Dev probe: device-resident 1-D FIR time per launch vs tap count, 2^28 samples in 4096-sample
rows (int16 -> int32 as one row), for the four sample/stage pairs; HIP events around
back-to-back launches.  Shows where the register kernel (<= 9 taps) hands over to the long-filter
kernels (fir1d_mfma.hip / fir1d_lds.hip).  FIR_HIP_LIB picks another build for an A/B.
Usage: python tools/long_taps_rate.py [taps,taps,...]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import fir_hip  # noqa: E402
from fir_hip import torch_ops  # noqa: E402


def main():
    taps = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [3, 5, 9, 10, 13, 17, 24, 31, 48, 64]
    n = 1 << 28
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(3)
    x16 = torch.from_numpy(rng.integers(-32768, 32768, n, dtype=np.int16)).to(dev)
    x8 = torch.from_numpy(rng.integers(0, 256, (n // 4096, 4096), dtype=np.uint8)).to(dev)
    y32 = torch.empty(n, dtype=torch.int32, device=dev)
    y8 = torch.empty(n, dtype=torch.uint8, device=dev)
    cases = (("i16->i32", x16, y32, fir_hip.OUT_I32, 6), ("u8->u8", x8, y8.view(x8.shape), fir_hip.OUT_U8_SAT, 2),
             ("i16->u8", x16.view(n // 4096, 4096), y8.view(n // 4096, 4096), fir_hip.OUT_U8_SAT, 3),
             ("u8->i32", x8, y32.view(x8.shape), fir_hip.OUT_I32, 5))
    warm = torch_ops.Taps([1, 2, 3, 4, 5])  # clocks take ~40 launches to ramp: warm before the first row
    for _ in range(60):
        torch_ops.fir1d_fixed_rows_dev(x16, warm, 12, 32, fir_hip.OUT_I32, out=y32)
    print(f"{'taps':>5s}" + "".join(f" {c[0] + ' us':>13s} {'%8TB/s':>7s}" for c in cases))
    for L in taps:
        hq = torch_ops.Taps(rng.integers(-2000, 2000, L).tolist())
        res = []
        for _, x, y, st, bps in cases:
            for _ in range(5):
                torch_ops.fir1d_fixed_rows_dev(x, hq, 12, 32, st, out=y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                torch_ops.fir1d_fixed_rows_dev(x, hq, 12, 32, st, out=y)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            res += [us, n * bps / us / 1e3 / 80]
        print(f"{L:5d}" + "".join(f" {res[2 * i]:13.1f} {res[2 * i + 1]:7.1f}" for i in range(len(cases))), flush=True)


if __name__ == "__main__":
    main()
