#!/usr/bin/env python3
"""The report stage on the 7 golden images (28 pairs, 544 MB of float64 ideal outputs): the
fixed and ideal 3-tap stages write their outputs into a scratch tree, then the report is timed
(best of 3) as shipped (plain pairs read into page-locked staging by a reader pool) and as the
reference's loop over pairs runs it (np.load of each pair, then the same GPU metrics call), with
the shipped form's timings.  Prints one JSON object."""
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "warmup-fir-filter_amd"))

import fir_hip  # noqa: E402
from fir_1d.sim.vector.gen_compare_report import _collect, generate_compare_report, name_patterns  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import generate_fixed_3tap_output_vector  # noqa: E402
from fir_1d.sim.vector.gen_ideal_output import generate_ideal_3tap_output_vector  # noqa: E402


def loop_form(idir, fdir):
    ire, fre = name_patterns("3tap")
    im, _, _ = _collect(idir, ire)
    fm, _, _ = _collect(fdir, fre)
    out = []
    for k in sorted(set(im) & set(fm)):
        yi, yf = np.load(im[k]), np.load(fm[k])
        out.append(fir_hip.compare_metrics(yi, yf))
    return out


def main():
    res = {}
    with tempfile.TemporaryDirectory(prefix="report_probe_") as tmp:
        t = Path(tmp)
        (t / "in").mkdir()
        with np.load(ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz") as d:
            for k in d.files:
                np.save(t / "in" / f"{k}_x_u8.npy", d[k])
        generate_ideal_3tap_output_vector(t / "in", t / "out", overwrite=True)
        generate_fixed_3tap_output_vector(t / "in", t / "out", overwrite=True)
        idir, fdir = t / "out" / "ideal_3tap", t / "out" / "fixed_3tap"
        shipped, loop = [], []
        for _ in range(3):
            tm = {}
            t0 = time.perf_counter()
            generate_compare_report("3tap", ideal_dir=idir, fixed_dir=fdir, report_dir=t / "rep", verbose=False,
                                    timings=tm)
            shipped.append(dict(tm, total_ms=round((time.perf_counter() - t0) * 1e3, 2)))
            t0 = time.perf_counter()
            loop_form(idir, fdir)
            loop.append(round((time.perf_counter() - t0) * 1e3, 2))
        res["shipped_runs"] = shipped
        res["shipped_best_ms"] = min(r["total_ms"] for r in shipped)
        res["reference_loop_form_ms"] = loop
        res["reference_loop_form_best_ms"] = min(loop)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
