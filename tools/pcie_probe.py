#!/usr/bin/env python3
"""What the host-pointer entries' copies can reach on this box: pageable vs pinned H2D / D2H
(torch copies, 512 MiB / 1 GiB) and the host memcpy rate with 1..16 threads (the staging
copy a pinned-buffer pipeline adds).  Prints one JSON object."""
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def best(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for nbytes in (512 << 20, 1 << 30):
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        hp = torch.from_numpy(np.ones(nbytes, np.uint8))
        hpin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        g = nbytes / 1e9
        out[f"{nbytes >> 20}MiB"] = {
            "h2d_pageable_GBs": round(g / best(lambda: d.copy_(hp)), 1),
            "h2d_pinned_GBs": round(g / best(lambda: d.copy_(hpin, non_blocking=True)), 1),
            "d2h_pageable_GBs": round(g / best(lambda: hp.copy_(d)), 1),
            "d2h_pinned_GBs": round(g / best(lambda: hpin.copy_(d, non_blocking=True)), 1),
        }
        del d, hp, hpin
    src = np.ones(1 << 30, np.uint8)
    dst = np.empty_like(src)
    for nt in (1, 2, 4, 8, 16):
        sl = np.array_split(np.arange(src.size), nt)
        bounds = [(int(s[0]), int(s[-1]) + 1) for s in sl]
        with ThreadPoolExecutor(nt) as ex:
            def run():
                list(ex.map(lambda b: np.copyto(dst[b[0]:b[1]], src[b[0]:b[1]]), bounds))
            t = best(run, 3)
        out[f"host_memcpy_{nt}t_GBs"] = round(src.size / t / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
