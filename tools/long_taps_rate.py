"""Dev probe: device-resident 1-D FIR time per launch vs tap count (2^28 int16 -> int32 and
u8 -> sat-u8 in 4096-sample rows), HIP events around back-to-back launches.  Shows where the
register kernel (<= 9 taps) hands over to the LDS sliding-window kernel (10..64 taps).
Usage: python tools/long_taps_rate.py [log2n]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import fir_hip  # noqa: E402
from fir_hip import torch_ops  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    n = 1 << log2n
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(3)
    x16 = torch.from_numpy(rng.integers(-32768, 32768, n, dtype=np.int16)).to(dev)
    y32 = torch.empty(n, dtype=torch.int32, device=dev)
    x8 = torch.from_numpy(rng.integers(0, 256, (n // 4096, 4096), dtype=np.uint8)).to(dev)
    y8 = torch.empty(x8.shape, dtype=torch.uint8, device=dev)
    print(f"{'taps':>5s} {'i16->i32 us':>12s} {'%8TB/s':>7s} {'u8 us':>9s} {'%8TB/s':>7s}")
    for L in (3, 5, 9, 10, 13, 17, 24, 31, 48, 64):
        hq = torch_ops.Taps(rng.integers(-2000, 2000, L).tolist())
        res = []
        for x, y, st, bps in ((x16, y32, fir_hip.OUT_I32, 6), (x8, y8, fir_hip.OUT_U8_SAT, 2)):
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
        print(f"{L:5d} {res[0]:12.1f} {res[1]:7.1f} {res[2]:9.1f} {res[3]:7.1f}", flush=True)


if __name__ == "__main__":
    main()
