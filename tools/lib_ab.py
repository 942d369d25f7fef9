"""Dev A/B: the headline kernel (2^28 int16 -> int32, 5-tap sharpen) from two builds of
libfir_hip.so in one process, interleaved batches of back-to-back launches timed by HIP
events.  Usage: python tools/lib_ab.py <lib A> <lib B> [rounds]"""
import ctypes
import sys

import numpy as np
import torch


def main():
    libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    x = torch.from_numpy(np.random.default_rng(1).integers(-32768, 32768, 1 << 28, dtype=np.int16)).to(dev)
    ys = [torch.empty(x.shape, dtype=torch.int32, device=dev) for _ in libs]
    h = (ctypes.c_int32 * 5)(-256, -1024, 6656, -1024, -256)
    vp = ctypes.c_void_p
    for lib in libs:
        lib.fir1d_fixed_rows_dev.argtypes = [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, vp,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]

    def run(i, n):
        for _ in range(n):
            rc = libs[i].fir1d_fixed_rows_dev(vp(x.data_ptr()), 1, 1, x.numel(), 1, h, 5, 12, 32, 1,
                                              vp(ys[i].data_ptr()), vp(s.cuda_stream))
            assert rc == 0
    for i in range(len(libs)):
        run(i, 50)
    torch.cuda.synchronize()
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
        print(f"{p}: median {v[len(v) // 2]:.1f} us  min {v[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
