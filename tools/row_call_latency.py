"""Single-row call latency of the drop-in API.

The reference's callers run the golden model once per image row (gen_fixed_output.py:44-52:
``fir_1d_fixed_golden(row.tolist(), h)`` for every row; img_006 = 2999 rows of 4499 samples).
This times, on the box's GPU:
  * the C entry fir1d_fixed_rows on one 4499-sample u8 row (ctypes, no Python validation);
  * fir_1d_fixed_golden(row_ndarray, h) and fir_1d_fixed_golden(row.tolist(), h) per call;
  * the reference-shaped per-row driver over img_006 (2999 calls, list rows, as the reference
    calls it) against the one-launch image driver (_run_fixed_rowwise).
Prints one JSON object.  Usage: python tools/row_call_latency.py [out.json]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
import fir_hip  # noqa: E402
from fir_1d.model.python.fir_1d_fixed_ref import fir_1d_fixed_golden  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import _run_fixed_rowwise  # noqa: E402

SHARPEN5 = [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16]


def per_call_us(fn, reps):
    fn()
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    img = np.load(ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz")["case_005_img_006_4499x2999_gray"]
    row = np.ascontiguousarray(img[1500])
    row_list = row.tolist()
    hq = np.array([-256, -1024, 6656, -1024, -256], np.int32)
    y = np.empty_like(row)
    lib = fir_hip.lib()
    res = {"row_samples": int(row.size), "image": "case_005_img_006 (2999 x 4499)"}
    res["c_entry_us"] = round(per_call_us(lambda: fir_hip.fir1d_fixed_rows(row, hq, 12, 32, fir_hip.OUT_U8_SAT, out=y),
                                          2000), 2)
    res["fir_1d_fixed_golden_ndarray_us"] = round(per_call_us(lambda: fir_1d_fixed_golden(row, SHARPEN5), 2000), 2)
    res["fir_1d_fixed_golden_list_us"] = round(per_call_us(lambda: fir_1d_fixed_golden(row_list, SHARPEN5), 1000), 2)
    rows = [r.tolist() for r in img]
    t0 = time.perf_counter()
    per_row = np.stack([fir_1d_fixed_golden(r, SHARPEN5) for r in rows])
    res["per_row_driver_img006_s"] = round(time.perf_counter() - t0, 4)
    res["per_row_driver_calls"] = len(rows)
    t0 = time.perf_counter()
    whole = _run_fixed_rowwise(img, SHARPEN5, frac_bits=12, acc_bits=32, coeff_bits=16)
    res["image_driver_img006_s"] = round(time.perf_counter() - t0, 5)
    res["per_row_equals_image_driver"] = bool(np.array_equal(per_row, whole))
    del lib
    text = json.dumps(res)
    print(text)
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(text + "\n")


if __name__ == "__main__":
    main()
