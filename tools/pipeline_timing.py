#!/usr/bin/env python3
"""Stage timing of the end-to-end pipeline on the 7 golden images (BASELINE configs[0]).

Runs the reference-shaped stages of warmup-fir-filter_amd/pipeline_fir_1d.py one by one
into a temp dir (overwrite on, both tap counts) and prints one JSON object with the wall
time of each stage and the samples it processed.  The reference's own CPU times for the
same stages are in BASELINE.md (measured in the survey container, one core): fixed 3-tap
92.6 s, fixed 5-tap 134.2 s, ideal 3-tap 44.6 s, ideal 5-tap 63.1 s.  Stage times here
include .npy file I/O and PCIe copies (the stages exchange files, as in the reference).
"""
from __future__ import annotations

import json
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "warmup-fir-filter_amd"))

from fir_1d.sim.vector.gen_3tap_compare_report import generate_3tap_compare_report  # noqa: E402
from fir_1d.sim.vector.gen_5tap_compare_report import generate_5tap_compare_report  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import (generate_fixed_3tap_output_vector,  # noqa: E402
                                                generate_fixed_5tap_output_vector)
from fir_1d.sim.vector.gen_ideal_output import (generate_ideal_3tap_output_vector,  # noqa: E402
                                                generate_ideal_5tap_output_vector)
from fir_1d.sim.vector.gen_input_vectors import generate_input_vector_jsons  # noqa: E402
from fir_1d.sim.vector.restore_images import restore_images  # noqa: E402

SAMPLES = 16_993_813  # the 7 golden images


def timed(fn, *a, **kw):
    t0 = time.perf_counter()
    r = fn(*a, **kw)
    return r, time.perf_counter() - t0


def main():
    cold = "--cold" in sys.argv  # no warm-up call: the first device stage pays the device's start
    t_proc = time.perf_counter()
    import fir_hip

    if not cold:
        fir_hip.fir1d_fixed_rows(__import__("numpy").zeros((2, 64), "uint8"), [1, 2, 1])  # load + init the device
    with tempfile.TemporaryDirectory() as tmp:
        vec = Path(tmp) / "vector"
        inp, out = vec / "input", vec / "output"
        res = {}
        _, res["input_vectors_s"] = timed(generate_input_vector_jsons, ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz", inp,
                                          overwrite=True)
        for tap, ideal, fixed, report in (("3tap", generate_ideal_3tap_output_vector, generate_fixed_3tap_output_vector,
                                           generate_3tap_compare_report),
                                          ("5tap", generate_ideal_5tap_output_vector, generate_fixed_5tap_output_vector,
                                           generate_5tap_compare_report)):
            n, res[f"ideal_{tap}_s"] = timed(ideal, inp, out, overwrite=True)
            m, res[f"fixed_{tap}_s"] = timed(fixed, inp, out, overwrite=True)
            assert n == m == 28
            _, res[f"report_{tap}_s"] = timed(report, ideal_dir=out / f"ideal_{tap}", fixed_dir=out / f"fixed_{tap}",
                                              report_dir=out / f"report_{tap}", top_k=5, strict=True)
        summ, res["restore_all_s"] = timed(restore_images, vector_output_dir=out, output_img_dir=Path(tmp) / "img",
                                           kind="all", tap="all", ideal_policy="clip", overwrite=True, strict=True)
        res["restored_images"] = summ["num_converted"]
    res["total_s"] = time.perf_counter() - t_proc
    res["cold"] = cold
    res = {k: round(v, 4) if isinstance(v, float) else v for k, v in res.items()}
    res["samples_per_stage"] = 4 * SAMPLES
    res["reference_cpu_s (BASELINE.md)"] = {"fixed_3tap": 92.6, "fixed_5tap": 134.2, "ideal_3tap": 44.6,
                                            "ideal_5tap": 63.1}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
