"""Dev driver for profiling one long-filter configuration: 2^28 samples, `reps` back-to-back
device launches.  Usage: python tools/long_taps_one.py <taps> <i16|i16u8|u8> [reps] [rand|smooth|sinc]
(the tap kinds of tools/long_taps_ab.py; default rand)"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import fir_hip  # noqa: E402
from fir_hip import torch_ops  # noqa: E402


def main():
    L, kind = int(sys.argv[1]), sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    n = 1 << 28
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    if kind == "i16":
        x = torch.from_numpy(rng.integers(-32768, 32768, n, dtype=np.int16)).to(dev)
        y = torch.empty(n, dtype=torch.int32, device=dev)
        st = fir_hip.OUT_I32
    elif kind == "i16u8":
        x = torch.from_numpy(rng.integers(-32768, 32768, (n // 4096, 4096), dtype=np.int16)).to(dev)
        y = torch.empty(x.shape, dtype=torch.uint8, device=dev)
        st = fir_hip.OUT_U8_SAT
    else:
        x = torch.from_numpy(rng.integers(0, 256, (n // 4096, 4096), dtype=np.uint8)).to(dev)
        y = torch.empty(x.shape, dtype=torch.uint8, device=dev)
        st = fir_hip.OUT_U8_SAT
    tap_kind = sys.argv[4] if len(sys.argv) > 4 else "rand"
    sys.path.insert(0, str(ROOT / "tools"))
    from long_taps_ab import taps_of

    hq = torch_ops.Taps(taps_of(tap_kind, L, rng).tolist())
    for _ in range(reps):
        torch_ops.fir1d_fixed_rows_dev(x, hq, 12, 32, st, out=y)
    torch.cuda.synchronize()
    print("done", L, kind, reps)


if __name__ == "__main__":
    main()
