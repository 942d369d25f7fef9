"""Dev probe: per-launch time (HIP events around each launch) over a long back-to-back series,
and the same series with an idle gap after each launch, for one 1-D configuration of 2^28
samples.  Shows whether a kernel slows down as the series runs (clock/power management).
Usage: python tools/launch_drift.py <taps> <i16|i16u8|u8> [launches] [gap_ms]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import fir_hip  # noqa: E402
from fir_hip import torch_ops  # noqa: E402


def series(x, y, hq, st, n, gap_ms):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in ev:
        e0.record()
        torch_ops.fir1d_fixed_rows_dev(x, hq, 12, 32, st, out=y)
        e1.record()
        if gap_ms:
            e1.synchronize()
            time.sleep(gap_ms / 1e3)
    torch.cuda.synchronize()
    return [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]


def main():
    L, kind = int(sys.argv[1]), sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    gap = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
    N = 1 << 28
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    rng = np.random.default_rng(3)
    if kind == "i16":
        x = torch.from_numpy(rng.integers(-32768, 32768, N, dtype=np.int16)).to(dev)
        y, st = torch.empty(N, dtype=torch.int32, device=dev), fir_hip.OUT_I32
    elif kind == "i16u8":
        x = torch.from_numpy(rng.integers(-32768, 32768, (N // 4096, 4096), dtype=np.int16)).to(dev)
        y, st = torch.empty(x.shape, dtype=torch.uint8, device=dev), fir_hip.OUT_U8_SAT
    else:
        x = torch.from_numpy(rng.integers(0, 256, (N // 4096, 4096), dtype=np.uint8)).to(dev)
        y, st = torch.empty(x.shape, dtype=torch.uint8, device=dev), fir_hip.OUT_U8_SAT
    hq = torch_ops.Taps(rng.integers(-2000, 2000, L).tolist())
    for label, g in (("back-to-back", 0.0), (f"{gap} ms gap", gap), ("back-to-back again", 0.0)):
        t = series(x, y, hq, st, n, g)
        q = [round(float(np.median(t[i:i + n // 10])), 1) for i in range(0, n, n // 10)]
        print(f"{kind} {L} taps, {label}: median per tenth of the series {q} us; min {min(t):.1f}", flush=True)


if __name__ == "__main__":
    main()
