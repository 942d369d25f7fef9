"""2-D FIR on the matrix cores (csrc/fir2d_mfma.hip): parity sweep vs the C oracle with the MFMA
path forced, then a same-process timing A/B against the register kernels on batches of 4
HBM-resident 8192x8192 frames.  Usage: python tools/mfma2d_probe.py [parity] [time]
"""
from __future__ import annotations

import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]

import fir_hip  # noqa: E402
from oracle import c_oracle  # noqa: E402

LP5 = np.array([256, 1024, 1536, 1024, 256], np.int64)
KERNELS = {
    "sep_lp5": np.outer(LP5, LP5) // 4096,                                  # bench, NP=1 after 2^4
    "gen5x5": np.random.default_rng(55).integers(-4, 5, (5, 5)),            # bench gen5x5
    "q412_5x5": np.random.default_rng(7).integers(-3000, 3000, (5, 5)),     # NP=2
    "big_5x5": np.random.default_rng(8).integers(-32768, 32640, (5, 5)),    # NP=2, wraps at acc 32
    "lap3": np.array([[0, -512, 0], [-512, 3072, -512], [0, -512, 0]]),
    "3x5": np.random.default_rng(56).integers(0, 5, (3, 5)),
    "5x1": np.array([[2], [-1], [7], [-1], [2]]),
    "3x4": np.random.default_rng(9).integers(-100, 100, (3, 4)),
    "5x2": np.random.default_rng(10).integers(-100, 100, (5, 2)),
    "odd127": np.random.default_rng(11).integers(-127, 128, (5, 5)) | 1,
}


def parity() -> None:
    os.environ["FIR2D_PATH"] = "mfma"
    co = c_oracle()
    rng = np.random.default_rng(1)
    shapes = [(1, 16), (2, 1024), (7, 48), (33, 1040), (64, 2048), (100, 4096 + 16), (37, 3072 + 512)]
    bad = 0
    n = 0
    for name, hq in KERNELS.items():
        for shape in shapes:
            x = rng.integers(0, 256, shape, dtype=np.uint8)
            x[0, : min(32, shape[1])] = 255
            x[-1, -min(32, shape[1]):] = 0
            for frac, acc in ((12, 32), (8, 24), (16, 32), (10, 32), (20, 32), (12, 20)):
                got = fir_hip.fir2d_fixed(x, hq, frac, acc, fir_hip.OUT_U8_SAT)
                ref = co.fir2d(x, hq, frac, acc, 0)
                n += 1
                if not np.array_equal(got, ref):
                    bad += 1
                    idx = np.argwhere(got != ref)
                    print(f"MISMATCH {name} {shape} f={frac} acc={acc}: {len(idx)} px, first {idx[:4].tolist()} "
                          f"got {got[tuple(idx[0])]} ref {ref[tuple(idx[0])]}", flush=True)
        print(f"parity {name}: done", flush=True)
    # batches of frames
    x = rng.integers(0, 256, (3, 70, 2048 + 64), dtype=np.uint8)
    for name in ("gen5x5", "q412_5x5"):
        got = fir_hip.fir2d_fixed(x, KERNELS[name])
        for f in range(3):
            n += 1
            if not np.array_equal(got[f], co.fir2d(x[f], KERNELS[name], 12, 32, 0)):
                bad += 1
                print(f"MISMATCH frames {name} frame {f}", flush=True)
    print(f"parity: {n - bad}/{n} cases bit-exact", flush=True)
    if bad:
        raise SystemExit(1)


def timing(reps: int = 200) -> None:
    import torch

    from fir_hip import torch_ops

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(20260227)
    frames = torch.from_numpy(rng.integers(0, 256, (4, 8192, 8192), dtype=np.uint8)).to(dev)
    out = torch.empty_like(frames)
    st = torch.cuda.current_stream()
    res = {}
    for rnd in range(2):
        for name in ("sep_lp5", "gen5x5", "q412_5x5", "lap3"):
            for path in ("reg", "mfma"):
                os.environ["FIR2D_PATH"] = path
                hq = KERNELS[name]
                for _ in range(20):
                    torch_ops.fir2d_fixed_dev(frames, hq, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    torch_ops.fir2d_fixed_dev(frames, hq, out=out)
                e1.record(st)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1000 / reps
                res.setdefault((name, path), []).append(us)
                print(f"round {rnd} {name:9s} {path:5s} {us:8.1f} us / 4 frames = {us / 4:6.2f} us/frame "
                      f"({2 * 4 * 8192 * 8192 / us / 8e6 * 100:5.1f} % of 8 TB/s)", flush=True)
    print("best of rounds:")
    for (name, path), v in res.items():
        print(f"  {name:9s} {path:5s} {min(v):8.1f} us ({min(v) / 4:6.2f} us/frame)")


if __name__ == "__main__":
    what = sys.argv[1:] or ["parity", "time"]
    t0 = time.time()
    if "parity" in what:
        parity()
    if "time" in what:
        timing()
    print(f"done in {time.time() - t0:.1f} s")
