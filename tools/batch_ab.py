"""Dev A/B: fir1d_fixed_images_multi_dev (the pipeline stage's batch launch) from two builds of
libfir_hip.so in one process, interleaved batches of back-to-back calls timed by HIP events;
every output plane its own allocation.  Outputs must be equal unless LIB_AB_NOCHECK is set
(timing-only variants).  Cases: the 7 golden image shapes, the 4499 x 2999 image alone, the
same with 4496-wide rows.
Usage: python tools/batch_ab.py <lib A> <lib B> [rounds]"""
import ctypes
import os
import sys

import numpy as np
import torch

BANK3 = (1365, 1365, 1365, 1024, 2048, 1024, -4096, 0, 4096, -512, 5120, -512)
CASES = {"golden7": ((853, 1280), (762, 640), (854, 1280), (64, 64), (64, 64), (2999, 4499), (641, 1280)),
         "golden7_big_first": ((2999, 4499), (853, 1280), (854, 1280), (641, 1280), (762, 640), (64, 64), (64, 64)),
         "golden7_big_last": ((64, 64), (64, 64), (762, 640), (641, 1280), (853, 1280), (854, 1280), (2999, 4499)),
         "w4499": ((2999, 4499),), "w4496": ((2999, 4496),)}


def main():
    libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(1)
    hc = (ctypes.c_int32 * len(BANK3))(*BANK3)
    vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    for name, shapes in CASES.items():
        xs = [torch.from_numpy(rng.integers(0, 256, sh, dtype=np.uint8)).to(dev) for sh in shapes]
        outs = [[[torch.empty(sh, dtype=torch.uint8, device=dev) for _ in range(4)] for sh in shapes] for _ in libs]
        n = len(shapes)
        rows = (cl * n)(*[sh[0] for sh in shapes])
        widths = (cl * n)(*[sh[1] for sh in shapes])
        xp = (vp * n)(*[x.data_ptr() for x in xs])
        yps = [(vp * (4 * n))(*[p.data_ptr() for ps in o for p in ps]) for o in outs]

        def run(i, k):
            for _ in range(k):
                rc = libs[i].fir1d_fixed_images_multi_dev(ci(n), xp, rows, widths, ci(0), ci(1), hc, ci(3), ci(4),
                                                          ci(12), ci(32), ci(0), yps[i], vp(s.cuda_stream))
                assert rc == 0, rc
        for i in range(len(libs)):
            run(i, 50)
        torch.cuda.synchronize()
        if not os.environ.get("LIB_AB_NOCHECK"):
            for a, b in zip(outs[0], outs[1]):
                assert all(torch.equal(p, q) for p, q in zip(a, b)), name
        t = [[] for _ in libs]
        for _ in range(rounds):
            for i in range(len(libs)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(i, 100)
                b.record()
                b.synchronize()
                t[i].append(a.elapsed_time(b) / 100 * 1e3)
        for i, p in enumerate(sys.argv[1:3]):
            v = sorted(t[i])
            print(f"{name} {p}: median {v[len(v) // 2]:.2f} us  min {v[0]:.2f} us", flush=True)


if __name__ == "__main__":
    main()
