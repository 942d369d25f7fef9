"""Dev A/B: one register-kernel workload from two builds of libfir_hip.so in one process,
interleaved batches of back-to-back launches timed by HIP events (outputs must be equal).
Workloads: i16 = the headline (2^28 int16 -> int32, 5-tap sharpen), u8 = 2^28 u8 -> sat-u8 in
4096-sample rows (5-tap sharpen), bank = the 4-filter 3-tap u8 bank (h_coeff_3tap_map),
bankw<W> = the same bank over rows of W samples (bankw4499: the reference's widest image's rows,
not a whole number of 16-byte vectors).
Usage: python tools/lib_ab.py <lib A> <lib B> [rounds] [i16|u8|bank|bankw<W>]"""
import ctypes
import os
import sys

import numpy as np
import torch

SHARPEN5 = (-256, -1024, 6656, -1024, -256)
BANK3 = (1365, 1365, 1365, 1024, 2048, 1024, -4096, 0, 4096, -512, 5120, -512)


def main():
    libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    wl = sys.argv[4] if len(sys.argv) > 4 else "i16"
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(1)
    n = 1 << 28
    if wl == "i16":
        x = torch.from_numpy(rng.integers(-32768, 32768, n, dtype=np.int16)).to(dev)
        ys = [torch.empty(n, dtype=torch.int32, device=dev) for _ in libs]
        in_dt, rows, width, stage, h, L, F = 1, 1, n, 1, SHARPEN5, 5, 1
    else:
        width = int(wl[5:]) if wl.startswith("bankw") else 4096
        n = n // width * width
        x = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).to(dev)
        F = 4 if wl.startswith("bank") else 1
        ys = [torch.empty(F * n, dtype=torch.uint8, device=dev) for _ in libs]
        in_dt, rows, stage = 0, n // width, 0
        h, L = (BANK3, 3) if wl.startswith("bank") else (SHARPEN5, 5)
    hc = (ctypes.c_int32 * len(h))(*h)
    vp, ci = ctypes.c_void_p, ctypes.c_int

    def run(i, k):
        for _ in range(k):
            rc = libs[i].fir1d_fixed_rows_multi_dev(vp(x.data_ptr()), ci(in_dt), ctypes.c_int64(rows),
                                                    ctypes.c_int64(width), ci(1), hc, ci(L), ci(F), ci(12), ci(32),
                                                    ci(stage), vp(ys[i].data_ptr()), vp(s.cuda_stream))
            assert rc == 0, rc
    for i in range(len(libs)):
        run(i, 50)
    torch.cuda.synchronize()
    if not os.environ.get("LIB_AB_NOCHECK"):  # timing-only variants (wrong results by design) set it
        assert torch.equal(ys[0], ys[1])
    t = [[] for _ in libs]
    for _ in range(rounds):
        for i in range(len(libs)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(i, 50)
            b.record()
            b.synchronize()
            t[i].append(a.elapsed_time(b) / 50 * 1e3)
    for i, p in enumerate(sys.argv[1:3]):
        v = sorted(t[i])
        print(f"{wl} {p}: median {v[len(v) // 2]:.1f} us  min {v[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
