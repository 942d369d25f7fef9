#!/usr/bin/env python3
"""A stage larger than one device call's staging window: N copies of the 4499 x 2999 golden image
(13.5 MB each) through generate_fixed_3tap_output_vector (4 output planes per image), fresh output
tree, best of 3, with the stage's breakdown; beside it the host I/O alone on the same files: the
inputs read by the stage's reader pool, the outputs written by 8 np.save threads.  Prints one JSON
object.  Usage: tools/big_stage_probe.py [N=40]"""
import json
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "warmup-fir-filter_amd"))

from fir_1d.sim.vector import stage_io  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import generate_fixed_3tap_output_vector  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    with np.load(ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz") as d:
        big = max((d[k] for k in d.files), key=lambda a: a.size)
    res = {"images": n, "shape": list(big.shape), "batch_bytes": stage_io.BATCH_BYTES}
    with tempfile.TemporaryDirectory(prefix="big_stage_") as tmp:
        t = Path(tmp)
        (t / "in").mkdir()
        for i in range(n):
            np.save(t / "in" / f"case_{i:03d}_big_x_u8.npy", big)
        runs = []
        for r in range(4):
            shutil.rmtree(t / "out", ignore_errors=True)
            tm = {}
            t0 = time.perf_counter()
            got = generate_fixed_3tap_output_vector(t / "in", t / "out", overwrite=True, timings=tm)
            tm["wall_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
            assert got == 4 * n
            runs.append(tm)
        res["stage_runs"] = runs[1:]
        best = min(runs[1:], key=lambda x: x["wall_ms"])
        out_bytes = 4 * n * big.size
        res["stage_best_ms"] = best["wall_ms"]
        res["stage_out_GBps"] = round(out_bytes / best["wall_ms"] / 1e6, 2)
        # host I/O alone
        files = sorted((t / "in").glob("*.npy"))
        buf = np.empty(n * big.size, np.uint8)
        t0 = time.perf_counter()
        futs = []
        for i, p in enumerate(files):
            futs += stage_io.read_into_async(p, 128, buf[i * big.size:(i + 1) * big.size])
        assert all(f.result() for f in futs)
        res["read_all_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        planes = [big] * (4 * n)
        (t / "w").mkdir()
        t0 = time.perf_counter()
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda ip: np.save(t / "w" / f"{ip[0]}.npy", ip[1]), enumerate(planes)))
        res["write_all_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
