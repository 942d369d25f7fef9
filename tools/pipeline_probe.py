"""Dev probe: where the pipeline stage (configs[0]: the 4-filter 3-tap u8 bank over the 7 golden
images) spends its time.  Times, with HIP events around back-to-back launches of one library:
each image's bank launch alone, and the big image's shape split into its two irregularities
(rows that straddle 16-byte vectors; output planes that start off a 16-byte boundary).
Usage: python tools/pipeline_probe.py [lib]"""
import ctypes
import sys

import numpy as np
import torch

BANK3 = (1365, 1365, 1365, 1024, 2048, 1024, -4096, 0, 4096, -512, 5120, -512)


def main():
    lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "warmup-fir-filter_amd/fir_hip/libfir_hip.so")
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(1)
    hc = (ctypes.c_int32 * len(BANK3))(*BANK3)
    vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64

    def timed(rows, width, reps=200):
        n = rows * width
        x = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).to(dev)
        y = torch.empty(4 * n, dtype=torch.uint8, device=dev)

        def run(k):
            for _ in range(k):
                rc = lib.fir1d_fixed_rows_multi_dev(vp(x.data_ptr()), ci(0), cl(rows), cl(width), ci(1), hc, ci(3),
                                                    ci(4), ci(12), ci(32), ci(0), vp(y.data_ptr()), vp(s.cuda_stream))
                assert rc == 0, rc
        run(50)
        best = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(reps)
            b.record()
            b.synchronize()
            best.append(a.elapsed_time(b) / reps * 1e3)
        us = min(best)
        gbs = 5 * n / us / 1e3
        print(f"{rows:6d} x {width:9d} ({n / 1e6:7.3f} Mpx, rows%16={width % 16:2d}, plane%16={n % 16:2d}): "
              f"{us:7.2f} us  {gbs:7.1f} GB/s", flush=True)
        return us

    print("== the 7 golden images (one bank launch each)")
    tot = 0.0
    for h, w in ((853, 1280), (762, 640), (854, 1280), (64, 64), (64, 64), (2999, 4499), (641, 1280)):
        tot += timed(h, w)
    print(f"sum of the 7 launches: {tot:.1f} us")
    shapes = ((853, 1280), (762, 640), (854, 1280), (64, 64), (64, 64), (2999, 4499), (641, 1280))

    def batch_time(shapes, layout, reps=200):
        """One fir1d_fixed_images_multi_dev call over the images; layout 'stacked': plane f of image
        i at y_i + f * h * w (the rows_multi layout), 'own': every plane its own allocation,
        'own+16': every plane 16 bytes past a 512-byte boundary."""
        xs = [torch.from_numpy(rng.integers(0, 256, sh, dtype=np.uint8)).to(dev) for sh in shapes]
        keep, planes = [], []
        for sh in shapes:
            px = sh[0] * sh[1]
            if layout == "stacked":
                y = torch.empty(4 * px, dtype=torch.uint8, device=dev)
                keep.append(y)
                planes += [y.data_ptr() + f * px for f in range(4)]
            else:
                off = 16 if layout == "own+16" else 0
                for _ in range(4):
                    y = torch.empty(px + off, dtype=torch.uint8, device=dev)
                    keep.append(y)
                    planes.append(y.data_ptr() + off)
        n = len(xs)
        rows = (cl * n)(*[sh[0] for sh in shapes])
        widths = (cl * n)(*[sh[1] for sh in shapes])
        xp = (vp * n)(*[x.data_ptr() for x in xs])
        yp = (vp * len(planes))(*planes)

        def batch(k):
            for _ in range(k):
                rc = lib.fir1d_fixed_images_multi_dev(ci(n), xp, rows, widths, ci(0), ci(1), hc, ci(3), ci(4),
                                                      ci(12), ci(32), ci(0), yp, vp(s.cuda_stream))
                assert rc == 0, rc
        batch(50)
        best = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch(reps)
            b.record()
            b.synchronize()
            best.append(a.elapsed_time(b) / reps * 1e3)
        px = sum(h * w for h, w in shapes)
        print(f"batch of {n} ({px / 1e6:.2f} Mpx), planes {layout:8s}: {min(best):7.2f} us  "
              f"{5 * px / min(best) / 1e3:7.1f} GB/s", flush=True)

    print("== the 7 golden images in one batch launch")
    for layout in ("stacked", "own", "own+16"):
        batch_time(shapes, layout)
    print("== one image: the single-image kernel vs the batch kernel (stacked planes: the same layout)")
    for sh in ((2999, 4499), (2999, 4496), (65536, 4096), (59666, 4499)):
        timed(*sh, reps=200 if sh[0] < 10000 else 20)
        batch_time((sh,), "stacked", reps=200 if sh[0] < 10000 else 20)
        batch_time((sh,), "own", reps=200 if sh[0] < 10000 else 20)
    print("== 2^28 samples, aligned row widths (the single-image kernel)")
    for w in (2048, 4096, 4112, 4480, 4496, 8192, 1 << 28):
        timed((1 << 28) // w, w, reps=20)
    print("== the big image's shape, irregularities apart")
    timed(2999, 4496)     # rows a whole number of vectors, planes aligned
    timed(3008, 4499)     # rows straddle vectors, planes aligned (3008 * 4499 % 16 == 0)
    timed(1, 13492501)    # one row, planes off 16 bytes
    timed(1, 13492496)    # one row, planes aligned
    timed(2999, 4499)     # both (the real image)
    print("== size ramp, aligned rows")
    for h in (64, 256, 1024, 4096, 16384):
        timed(h, 4096)


if __name__ == "__main__":
    main()
