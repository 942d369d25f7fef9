"""Dev A/B of the report-metrics pass (compare_metrics_dev, u8 fixed, 2^28 samples) across
several builds of libfir_hip.so in ONE process: interleaved batches of back-to-back launches,
timed by HIP events on the launch stream; every build's 9 sums must be bit-identical.
Usage: python tools/metrics_ab.py <lib> [<lib> ...] [--rounds R] [--log2n N]"""
import argparse
import ctypes

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--no-check", action="store_true", help="experiment builds with knowingly wrong sums: time only")
    a = ap.parse_args()
    libs = [ctypes.CDLL(p) for p in a.libs]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    n = 1 << a.log2n
    rng = np.random.default_rng(5)
    xi = rng.uniform(-64.0, 320.0, n)
    xf = np.clip(np.rint(xi) + rng.integers(-3, 4, n), 0, 255).astype(np.uint8)
    ideal = torch.from_numpy(xi).to(dev)
    fixed = torch.from_numpy(xf).to(dev)
    work = torch.empty(int(libs[0].fir_metrics_work_bytes(ctypes.c_int64(n))) + 4096, dtype=torch.uint8, device=dev)
    outs = [torch.empty(9, dtype=torch.float64, device=dev) for _ in libs]
    vp = ctypes.c_void_p

    def run(i, k):
        for _ in range(k):
            rc = libs[i].fir_compare_metrics_dev(vp(ideal.data_ptr()), vp(fixed.data_ptr()), ctypes.c_int(0),
                                                 ctypes.c_int64(n), vp(outs[i].data_ptr()), vp(work.data_ptr()),
                                                 vp(s.cuda_stream))
            assert rc == 0, rc

    for i in range(len(libs)):
        run(i, 30)
    torch.cuda.synchronize()
    ref = outs[0].cpu().numpy()
    for i in range(1, len(libs) if not a.no_check else 1):
        got = outs[i].cpu().numpy()
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (a.libs[i], got, ref)
    times = [[] for _ in libs]
    for _ in range(a.rounds):
        for i in range(len(libs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(i, 5)
            e0.record()
            run(i, a.batch)
            e1.record()
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) * 1e3 / a.batch)
    for p, t in zip(a.libs, times):
        t = sorted(t)
        gbs = n * 9 / (np.median(t) * 1e-6) / 1e9
        print(f"{p}: median {np.median(t):.1f} us  min {t[0]:.1f}  max {t[-1]:.1f}  ({gbs:.0f} GB/s, "
              f"{gbs / 8000:.1%} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
