#!/usr/bin/env python3
"""Interleaved A/B of register-kernel builds in ONE process, reported pair by pair.

Each round times a batch of back-to-back launches of every library in turn (HIP events on one
stream; the order reverses every round so clock drift cancels), and every library's output must
equal the first's.  Printed per workload: every round's times, then per library the median and
the median of its per-round difference to library 0 with the count of rounds it was faster.
Workloads: i16 = BASELINE configs[1] (2^28 int16 -> int32, 5-tap sharpen); u8 = the reference's
own u8 -> sat-u8 path (a1: 2^28 u8 in 4096-sample rows, 5-tap sharpen); bank = the 4-filter 3-tap
u8 bank (h_coeff_3tap_map) over the same rows.

Usage: python tools/ab_pairs.py <rounds> <workloads, comma list> <lib0> <lib1> [lib2 ...]
"""
import ctypes
import json
import statistics
import sys

import numpy as np
import torch

SHARPEN5 = (-256, -1024, 6656, -1024, -256)
BANK3 = (1365, 1365, 1365, 1024, 2048, 1024, -4096, 0, 4096, -512, 5120, -512)
BATCH = 50


def main():
    rounds, wls, paths = int(sys.argv[1]), sys.argv[2].split(","), sys.argv[3:]
    libs = [ctypes.CDLL(p) for p in paths]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    rng = np.random.default_rng(1)
    report = {}
    for wl in wls:
        n = 1 << 28
        if wl == "i16":
            x = torch.from_numpy(rng.integers(-32768, 32768, n, dtype=np.int16)).to(dev)
            ys = [torch.empty(n, dtype=torch.int32, device=dev) for _ in libs]
            in_dt, rows, width, stage, h, L, F = 1, 1, n, 1, SHARPEN5, 5, 1
        else:
            width = 4096
            x = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).to(dev)
            F = 4 if wl == "bank" else 1
            ys = [torch.empty(F * n, dtype=torch.uint8, device=dev) for _ in libs]
            in_dt, rows, stage = 0, n // width, 0
            h, L = (BANK3, 3) if wl == "bank" else (SHARPEN5, 5)
        hc = (ctypes.c_int32 * len(h))(*h)
        vp, ci = ctypes.c_void_p, ctypes.c_int

        def run(i, k):
            for _ in range(k):
                rc = libs[i].fir1d_fixed_rows_multi_dev(vp(x.data_ptr()), ci(in_dt), ctypes.c_int64(rows),
                                                        ctypes.c_int64(width), ci(1), hc, ci(L), ci(F), ci(12),
                                                        ci(32), ci(stage), vp(ys[i].data_ptr()), vp(s.cuda_stream))
                assert rc == 0, rc

        for i in range(len(libs)):  # warm every build (clocks, code objects)
            run(i, 100)
        torch.cuda.synchronize()
        for i in range(1, len(libs)):
            assert torch.equal(ys[0], ys[i]), (wl, paths[i])
        t = [[] for _ in libs]
        for r in range(rounds):
            order = list(range(len(libs)))
            if r % 2:
                order.reverse()
            for i in order:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(i, BATCH)
                b.record()
                b.synchronize()
                t[i].append(a.elapsed_time(b) / BATCH * 1e3)
            print(wl, r, " ".join(f"{t[i][-1]:.2f}" for i in range(len(libs))), flush=True)
        summ = {}
        for i, p in enumerate(paths):
            d = [t[i][r] - t[0][r] for r in range(rounds)]
            summ[p] = {"median_us": round(statistics.median(t[i]), 2), "min_us": round(min(t[i]), 2),
                       "median_diff_vs_lib0_us": round(statistics.median(d), 2),
                       "rounds_faster_than_lib0": sum(v < 0 for v in d), "rounds": rounds,
                       "per_round_us": [round(v, 2) for v in t[i]]}
            print(wl, p, json.dumps({k: v for k, v in summ[p].items() if k != "per_round_us"}), flush=True)
        report[wl] = summ
        del x, ys
        torch.cuda.empty_cache()
    print(json.dumps(report))


if __name__ == "__main__":
    main()
