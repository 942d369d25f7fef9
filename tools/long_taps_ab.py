"""Dev A/B of the long-filter kernels across builds of libfir_hip.so in ONE process: u8 -> u8
(and u8 -> int32) FIR over 2^28 samples in 4096-sample rows for each tap count, interleaved
batches of back-to-back launches timed by HIP events; every build's output must be identical.
Usage: python tools/long_taps_ab.py <taps,taps,...> <lib> [<lib> ...] [--no-check] [--kind rand|smooth|sinc]
(--no-check: experiment builds whose outputs are knowingly wrong, timed only; --kind: the taps --
rand: uniform in [-2000, 2000) (every k-step needs both byte planes), smooth: a Hann window of unit
gain in Q4.12 (every tap in [-128, 127] past ~64 taps), sinc: a Hann-windowed low-pass sinc,
cutoff 0.1, unit gain (only the centre taps need the high byte))"""
import ctypes
import sys

import numpy as np
import torch


def taps_of(kind: str, L: int, rng) -> np.ndarray:
    if kind == "rand":
        return rng.integers(-2000, 2000, L).astype(np.int32)
    w = np.hanning(L + 2)[1:-1]
    if kind == "smooth":
        h = w / w.sum()
    else:
        n = np.arange(L) - (L - 1) / 2
        h = 0.2 * np.sinc(0.2 * n) * w
        h /= h.sum()
    return np.rint(h * 4096).astype(np.int32)


def main():
    taps = [int(t) for t in sys.argv[1].split(",")]
    check = "--no-check" not in sys.argv
    kind = sys.argv[sys.argv.index("--kind") + 1] if "--kind" in sys.argv else "rand"
    skip = {"--no-check", "--kind", kind}
    paths = [p for p in sys.argv[2:] if p not in skip]
    libs = [ctypes.CDLL(p) for p in paths]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    n = 1 << 28
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).to(dev)
    ys = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in libs]
    vp, ci, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    print(f"kind {kind}", flush=True)
    print(f"{'taps':>5s}" + "".join(f" {p.split('/')[-1][:24]:>24s}" for p in paths), flush=True)
    for L in taps:
        hq = taps_of(kind, L, rng)
        hc = hq.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))

        def run(i, k):
            for _ in range(k):
                rc = libs[i].fir1d_fixed_rows_dev(vp(x.data_ptr()), ci(0), i64(n // 4096), i64(4096), ci(1), hc, ci(L),
                                                  ci(12), ci(32), ci(0), vp(ys[i].data_ptr()), vp(s.cuda_stream))
                assert rc == 0, rc

        for i in range(len(libs)):
            run(i, 3)
        torch.cuda.synchronize()
        for i in range(1, len(libs) if check else 1):
            assert torch.equal(ys[0], ys[i]), (L, paths[i])
        t = [[] for _ in libs]
        reps = max(3, min(20, int(20 * 200 / L)))
        for _ in range(4):
            for i in range(len(libs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(i, reps)
                e1.record()
                e1.synchronize()
                t[i].append(e0.elapsed_time(e1) * 1e3 / reps)
        print(f"{L:5d}" + "".join(f" {np.median(v):21.1f} us" for v in t), flush=True)


if __name__ == "__main__":
    main()
