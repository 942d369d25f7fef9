"""Dev probe: per-batch kernel time of the bench kernel over ~3 s of back-to-back launches,
to see clock/power ramp and drift (batches of 20 launches bracketed by HIP events)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import numpy as np, torch
import fir_hip
from fir_hip import torch_ops

torch.cuda.set_device(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
x = torch.from_numpy(np.random.default_rng(20260227).integers(-32768, 32768, 1 << 28, dtype=np.int16)).cuda()
y = torch.empty(x.shape, dtype=torch.int32, device="cuda")
taps = torch_ops.Taps([-256, -1024, 6656, -1024, -256])
out = []
t_end = time.time() + float(sys.argv[1] if len(sys.argv) > 1 else 3.0)
while time.time() < t_end:
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        torch_ops.fir1d_fixed_rows_dev(x, taps, 12, 32, fir_hip.OUT_I32, out=y)
    b.record(); b.synchronize()
    out.append(a.elapsed_time(b) / 20 * 1e3)
print("batches", len(out))
print("first 10 (us):", [round(v, 1) for v in out[:10]])
print("every 25th:", [round(v, 1) for v in out[::25]])
print("median %.1f  min %.1f  max %.1f" % (np.median(out), min(out), max(out)))
