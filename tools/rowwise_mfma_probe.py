"""Row-wise 1-D u8 filters on the 2-D matrix-core kernel (a 1 x L kernel, R = 1) against the 1-D
register kernel: the fir1d_u8 bench shape (2^28 u8 samples in 4096-sample rows), bit-exact
check between the two and against the C oracle on a slice, then interleaved event timing.
Usage: python tools/rowwise_mfma_probe.py
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]

import fir_hip  # noqa: E402
from fir_hip import torch_ops  # noqa: E402
from oracle import c_oracle  # noqa: E402

TAPS = {"sharpen5": [-256, -1024, 6656, -1024, -256], "lp5": [256, 1024, 1536, 1024, 256],
        "ma3": [1365, 1365, 1365], "edge3": [-4096, 0, 4096]}


def main() -> None:
    os.environ["FIR2D_PATH"] = "mfma"
    dev = torch.device("cuda:0")
    rows, w = 1 << 16, 4096
    x_host = np.random.default_rng(20260227).integers(0, 256, (rows, w), dtype=np.uint8)
    x = torch.from_numpy(x_host).to(dev)
    y1 = torch.empty_like(x)
    y2 = torch.empty_like(x)
    st = torch.cuda.current_stream()
    co = c_oracle()
    for name, h in TAPS.items():
        k2 = np.array([h], np.int64)
        t1 = torch_ops.Taps(h)
        torch_ops.fir1d_fixed_rows_dev(x, t1, 12, 32, fir_hip.OUT_U8_SAT, out=y1)
        torch_ops.fir2d_fixed_dev(x, k2, out=y2)
        torch.cuda.synchronize()
        same = torch.equal(y1, y2)
        ref = co.fir2d(x_host[:64], k2, 12, 32, 0)
        ok = np.array_equal(y2[:64].cpu().numpy(), ref)
        res = {}
        for rnd in range(3):
            for path in ("reg1d", "mfma2d"):
                for _ in range(20):
                    if path == "reg1d":
                        torch_ops.fir1d_fixed_rows_dev(x, t1, 12, 32, fir_hip.OUT_U8_SAT, out=y1)
                    else:
                        torch_ops.fir2d_fixed_dev(x, k2, out=y2)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(200):
                    if path == "reg1d":
                        torch_ops.fir1d_fixed_rows_dev(x, t1, 12, 32, fir_hip.OUT_U8_SAT, out=y1)
                    else:
                        torch_ops.fir2d_fixed_dev(x, k2, out=y2)
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault(path, []).append(e0.elapsed_time(e1) * 1000 / 200)
        print(f"{name:9s} equal={same} oracle_slice={ok}  " +
              "  ".join(f"{p} {min(v):6.1f} us ({2 * rows * w / min(v) / 8e6 * 100:4.1f} %)" for p, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
