"""Dev A/B: the read-dominant stream kernels (restore clip, report metrics) of several
libfir_hip.so builds in one process, over 2^28 doubles (2 GiB) resident in HBM; interleaved
batches of back-to-back launches timed by HIP events; outputs compared across builds (restore
bytes exactly; metrics bit for bit).
Usage: python tools/lib_ab_stream.py <lib> [<lib> ...] [--rounds R] [--log2n N]"""
import argparse
import ctypes
from pathlib import Path

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--log2n", type=int, default=28)
    args = ap.parse_args()
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    libs = []
    for p in args.libs:
        lib = ctypes.CDLL(p)
        lib.fir_restore_u8_dev.argtypes = [vp, i64, i32, vp, vp, vp]
        lib.fir_compare_metrics_dev.argtypes = [vp, vp, ctypes.c_int, i64, vp, vp, vp]  # ABI 4: fixed dtype
        lib.fir_metrics_work_bytes.restype = i64
        lib.fir_metrics_work_bytes.argtypes = [i64]
        libs.append(lib)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    n = 1 << args.log2n
    rng = np.random.default_rng(5)
    a_host = rng.uniform(-64.0, 320.0, n)
    a = torch.from_numpy(a_host).to(dev)
    fx = torch.from_numpy(np.clip(np.rint(a_host) + rng.integers(-3, 4, n), 0, 255).astype(np.uint8)).to(dev)
    del a_host
    outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in libs]
    mets = [torch.zeros(9, dtype=torch.float64, device=dev) for _ in libs]
    work = torch.empty(max(int(lib.fir_metrics_work_bytes(n)) for lib in libs) + 4096, dtype=torch.uint8, device=dev)
    S = vp(s.cuda_stream)

    def restore(i):
        assert libs[i].fir_restore_u8_dev(vp(a.data_ptr()), n, 0, vp(outs[i].data_ptr()), None, S) == 0

    def metrics(i):
        assert libs[i].fir_compare_metrics_dev(vp(a.data_ptr()), vp(fx.data_ptr()), 0, n, vp(mets[i].data_ptr()),  # FIR_DT_U8
                                               vp(work.data_ptr()), S) == 0

    ops = {"restore_clip": (restore, 9.0), "metrics": (metrics, 9.0)}
    for name, (fn, _) in ops.items():
        for i in range(len(libs)):
            for _ in range(20):
                fn(i)
        torch.cuda.synchronize()
    for i in range(1, len(libs)):
        assert torch.equal(outs[0], outs[i]), f"restore output of {args.libs[i]} differs"
        m0, m1 = mets[0].cpu().numpy(), mets[i].cpu().numpy()
        assert all(m0[k] == m1[k] for k in (0, 4, 5, 6, 7)), (m0, m1)
        assert np.array_equal(m0[1:4], m1[1:4]), (m0, m1)  # sums in NumPy's order: bit-exact
    batch = 20
    res = {(name, i): [] for name in ops for i in range(len(libs))}
    for _ in range(args.rounds):
        for name, (fn, _) in ops.items():
            for i in range(len(libs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(batch):
                    fn(i)
                e1.record()
                e1.synchronize()
                res[(name, i)].append(e0.elapsed_time(e1) * 1e3 / batch)
    print(f"{'op':14s} {'lib':24s} {'median_us':>10s} {'min_us':>9s} {'%8TB/s':>7s}")
    for name, (_, bps) in ops.items():
        for i in range(len(libs)):
            t = sorted(res[(name, i)])
            med = t[len(t) // 2]
            print(f"{name:14s} {Path(args.libs[i]).name:24s} {med:10.1f} {t[0]:9.1f} {n * bps / med / 1e3 / 80:7.1f}")


if __name__ == "__main__":
    main()
