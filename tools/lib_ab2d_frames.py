"""Dev A/B for the 2-D kernels on batches of 4 HBM-resident 8192x8192 frames (the bench shape):
fir2d_fixed_frames_dev from several builds of libfir_hip.so in one process, interleaved
batches of back-to-back launches timed by HIP events, outputs compared across builds.
Usage: FIR2D_PATH=mfma python tools/lib_ab2d_frames.py <lib A> <lib B> ...   (AB_ROUNDS=6)
"""
import ctypes
import os
import sys

import numpy as np
import torch

KERNELS = {
    "sep5x5_lp": np.outer([256, 1024, 1536, 1024, 256], [256, 1024, 1536, 1024, 256]) // 4096,
    "gen5x5": np.random.default_rng(55).integers(-4, 5, (5, 5)),
    "q412_5x5": np.random.default_rng(7).integers(-3000, 3000, (5, 5)),
    "sharpen3x3": np.array([[0, -512, 0], [-512, 3072, -512], [0, -512, 0]]),
}


def main():
    paths = sys.argv[1:]
    libs = [ctypes.CDLL(p) for p in paths]
    rounds = int(os.environ.get("AB_ROUNDS", "6"))
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    F, H, W = 4, 8192, 8192
    x = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (F, H, W), dtype=np.uint8)).to(dev)
    vp = ctypes.c_void_p
    for lib in libs:
        lib.fir2d_fixed_frames_dev.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
    for kname, k in KERNELS.items():
        R, C = k.shape
        h = (ctypes.c_int32 * (R * C))(*[int(v) for v in k.reshape(-1)])
        ys = [torch.empty_like(x) for _ in libs]

        def run(i, n):
            for _ in range(n):
                rc = libs[i].fir2d_fixed_frames_dev(vp(x.data_ptr()), F, H, W, h, R, C, 12, 32, 0,
                                                    vp(ys[i].data_ptr()), vp(s.cuda_stream))
                assert rc == 0
        for i in range(len(libs)):
            run(i, 30)
        torch.cuda.synchronize()
        if not os.environ.get("AB_NOCHECK"):
            assert all(torch.equal(ys[0], y) for y in ys[1:]), kname
        t = [[] for _ in libs]
        for _ in range(rounds):
            for i in range(len(libs)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(i, 100)
                b.record()
                b.synchronize()
                t[i].append(a.elapsed_time(b) / 100 * 1e3)
        for i, p in enumerate(paths):
            v = sorted(t[i])
            print(f"{kname:11s} {os.path.basename(p):28s} median {v[len(v) // 2]:6.1f} us  min {v[0]:6.1f} us "
                  f"({v[0] / F:5.2f} us/frame, {2 * F * H * W / v[0] / 8e6 * 100:4.1f} % of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
