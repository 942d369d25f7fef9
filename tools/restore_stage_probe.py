#!/usr/bin/env python3
"""Where the restore stage's wall time goes (the pipeline's last stage, 112 PNGs from the 7 golden
images: ideal + fixed, 3 + 5 taps, 4 filters).  The vector outputs are made by the shipped stages
into a scratch tree; then, best of 3 each:
  shipped       restore_images(kind=all, tap=all) as the CLI runs it
  load          np.load of the 112 .npy inputs alone
  convert       the GPU u8 conversions alone (fir_hip.restore_u8 on the loaded arrays)
  png_T         Pillow PNG encoding of the 112 u8 images alone on T threads (T = 1, 8, 16)
Prints one JSON object."""
import json
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "warmup-fir-filter_amd"))

import fir_hip  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import (generate_fixed_3tap_output_vector,  # noqa: E402
                                                generate_fixed_5tap_output_vector)
from fir_1d.sim.vector.gen_ideal_output import (generate_ideal_3tap_output_vector,  # noqa: E402
                                                generate_ideal_5tap_output_vector)
from fir_1d.sim.vector.restore_images import restore_images  # noqa: E402


def best(fn, n=3):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 1), [round(t * 1e3, 1) for t in ts]


def main():
    from PIL import Image
    res = {}
    with tempfile.TemporaryDirectory(prefix="restore_probe_") as tmp:
        t = Path(tmp)
        (t / "in").mkdir()
        with np.load(ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz") as d:
            for k in d.files:
                np.save(t / "in" / f"{k}_x_u8.npy", d[k])
        for g in (generate_ideal_3tap_output_vector, generate_ideal_5tap_output_vector,
                  generate_fixed_3tap_output_vector, generate_fixed_5tap_output_vector):
            g(t / "in", t / "out", overwrite=True)
        files = sorted((t / "out").glob("*/*.npy"))
        res["inputs"] = len(files)
        res["input_bytes"] = sum(p.stat().st_size for p in files)
        res["shipped_ms"], res["shipped_runs_ms"] = best(lambda: restore_images(
            vector_output_dir=t / "out", output_img_dir=t / "img", kind="all", tap="all", ideal_policy="clip",
            overwrite=True, strict=True))
        arrays = []
        res["load_ms"], _ = best(lambda: arrays.__setitem__(slice(None), [np.load(p) for p in files]))
        u8 = []

        def convert():
            u8[:] = [a if a.dtype == np.uint8 else fir_hip.restore_u8(a, fir_hip.RESTORE_CLIP) for a in arrays]
        res["convert_ms"], _ = best(convert)
        res["pixels"] = int(sum(a.size for a in u8))
        (t / "png").mkdir()

        def encode(threads):
            outs = [t / "png" / f"{i}.png" for i in range(len(u8))]
            if threads == 1:
                for a, o in zip(u8, outs):
                    Image.fromarray(a, mode="L").save(o)
                return
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(lambda ao: Image.fromarray(ao[0], mode="L").save(ao[1]), zip(u8, outs)))
        for th in (1, 8, 16):
            res[f"png_{th}_ms"], _ = best(lambda: encode(th), n=2 if th == 1 else 3)
        big = max(u8, key=lambda a: a.size)
        res["png_largest_image_ms"], _ = best(lambda: Image.fromarray(big, mode="L").save(t / "png" / "big.png"))
        res["largest_image_px"] = int(big.size)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
