"""Ideal (float64) output vectors (.npy) for every input image x every coefficient set.

Mirror of the reference stage ``fir_1d/sim/vector/gen_ideal_output.py`` (entry points,
naming ``{case}__{coeff}_ideal_{3,5}tap_y_f64.npy`` under ``output_dir/ideal_{3,5}tap``,
skip-if-exists, return count, error order, CLI flags).  The reference's loops over images,
coefficient sets (:75-86) and rows (:37-50) become ONE device call per stage
(``fir_hip.fir1d_ideal_images_multi`` through ``stage_io.run_image_stage``: each image uploaded
once for all four sets, every plane bit-exact in float64, downloaded and written while the later
planes are in flight); ``devices`` / ``--devices N`` instead spreads each image's rows over several
GPUs (no exchange).  ``timings`` (a dict) receives the stage's breakdown in milliseconds.
"""
from __future__ import annotations

import argparse
from pathlib import Path
from time import perf_counter

import numpy as np

import fir_hip
from fir_1d.model.python.fir_1d_ref import _prepare_rows_u8, _validate_h_coefficients
from fir_1d.sim.vector import stage_io
from fir_1d.sim.vector.gen_fixed_output import _case_stem_from_input, _iter_input_npy_files, _load_input_image_u8
from fir_1d.sim.vector.h_coeff import h_coeff_3tap_map, h_coeff_5tap_map

THIS_FILE = Path(__file__).resolve()
DEFAULT_INPUT_DIR = THIS_FILE.parent / "input"
DEFAULT_OUTPUT_DIR = THIS_FILE.parent / "output"


def _run_ideal_rowwise(x_u8: np.ndarray, h: list[float], devices=None) -> np.ndarray:
    """Every row of an H x W image through the ideal model in one launch.  A non-uint8 image
    is prepared row by row as the reference's per-row ``fir_1d_ideal(row.tolist(), h)`` calls
    would (gen_ideal_output.py:40-42): h is checked first, then rows in order, each non-finite
    sample reported with its index in its row (fir_1d_ref._prepare_rows_u8)."""
    height, width = x_u8.shape
    if height == 0:
        return np.zeros((0, width), dtype=np.float64)
    _validate_h_coefficients(h)
    xc = _prepare_rows_u8(x_u8)
    if width == 0:
        return np.zeros((height, 0), dtype=np.float64)
    devs = fir_hip.parse_devices(devices)
    return fir_hip.fir1d_ideal_rows(xc, [float(v) for v in h],
                                    device=devs[0], devices=devs if len(devs) > 1 else None)


def _generate_ideal_outputs_for_tap_map(*, input_dir: Path, out_dir: Path, coeff_map: dict[str, list[float]],
                                        tap_label: str, overwrite: bool = False, devices=None,
                                        timings: dict | None = None) -> int:
    inputs = _iter_input_npy_files(input_dir)
    if not inputs:
        raise FileNotFoundError(f"No input .npy files found in {input_dir}")
    out_dir.mkdir(parents=True, exist_ok=True)
    devs = fir_hip.parse_devices(devices)
    if len(devs) > 1:  # each image's rows over several devices, one (image, set) at a time
        generated = 0
        for in_path in inputs:
            x_u8 = _load_input_image_u8(in_path)
            stem = _case_stem_from_input(in_path)
            for coeff_name, h in coeff_map.items():
                out_path = out_dir / f"{stem}__{coeff_name}_ideal_{tap_label}_y_f64.npy"
                if out_path.exists() and not overwrite:
                    continue
                np.save(out_path, _run_ideal_rowwise(x_u8, h, devs))
                generated += 1
        return generated

    def plan_items(stem, shape):
        """The reference's inner loop (gen_ideal_output.py:79-86) without the compute: skipped
        files, then each pending set's check (fir_1d_ref.py:9-24; none for an image with no rows,
        whose row loop never calls the model).  A failing set ends the stage there."""
        items = []
        for name, h in coeff_map.items():
            out_path = out_dir / f"{stem}__{name}_ideal_{tap_label}_y_f64.npy"
            if out_path.exists() and not overwrite:
                continue
            if shape[0] > 0:
                try:
                    _validate_h_coefficients(h)
                except ValueError as exc:
                    return items, exc
            items.append((out_path, name))
        return items, None

    def compute(xs, keys, outs, ready, timing):
        """Every image under the sets ``keys``: one device call per tap length."""
        calls, i = 0, 0
        while i < len(keys):
            j = i
            while j < len(keys) and len(coeff_map[keys[j]]) == len(coeff_map[keys[i]]):
                j += 1
            t: dict = {}
            fir_hip.fir1d_ideal_images_multi(xs, [[float(v) for v in coeff_map[k]] for k in keys[i:j]],
                                             device=devs[0], outs=[o[i:j] for o in outs],
                                             ready=lambda im, g, i=i: ready(im, i + g), timing=t)
            for k, v in t.items():
                timing[k] = timing.get(k, 0.0) + v
            calls += 1
            i = j
        timing["calls"] = calls

    return stage_io.run_image_stage(inputs, _case_stem_from_input, plan_items, compute, np.float64, timings)


def generate_ideal_3tap_output_vector(input_dir: Path = DEFAULT_INPUT_DIR, output_dir: Path = DEFAULT_OUTPUT_DIR,
                                      *, overwrite: bool = False, devices=None, timings: dict | None = None) -> int:
    return _generate_ideal_outputs_for_tap_map(
        input_dir=Path(input_dir).resolve(), out_dir=Path(output_dir).resolve() / "ideal_3tap",
        coeff_map=h_coeff_3tap_map, tap_label="3tap", overwrite=overwrite, devices=devices,
        timings=timings)


def generate_ideal_5tap_output_vector(input_dir: Path = DEFAULT_INPUT_DIR, output_dir: Path = DEFAULT_OUTPUT_DIR,
                                      *, overwrite: bool = False, devices=None, timings: dict | None = None) -> int:
    return _generate_ideal_outputs_for_tap_map(
        input_dir=Path(input_dir).resolve(), out_dir=Path(output_dir).resolve() / "ideal_5tap",
        coeff_map=h_coeff_5tap_map, tap_label="5tap", overwrite=overwrite, devices=devices,
        timings=timings)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Generate FIR 1D ideal output vectors for 3tap/5tap filters (GPU).")
    ap.add_argument("--input-dir", type=Path, default=DEFAULT_INPUT_DIR)
    ap.add_argument("--output-dir", type=Path, default=DEFAULT_OUTPUT_DIR)
    ap.add_argument("--tap", choices=("all", "3", "5"), default="all")
    ap.add_argument("--overwrite", action="store_true")
    ap.add_argument("--devices", default=None,
                    help="GPUs for the rows of each image: N (devices 0..N-1) or a comma list of ids")
    args = ap.parse_args(argv)
    t0 = perf_counter()
    in_dir, out_dir = args.input_dir.resolve(), args.output_dir.resolve()
    counts, expected = {"ideal_3tap": 0, "ideal_5tap": 0}, 0
    try:
        if args.tap in ("all", "3"):
            expected += len(_iter_input_npy_files(in_dir)) * len(h_coeff_3tap_map)
            counts["ideal_3tap"] = generate_ideal_3tap_output_vector(in_dir, out_dir, overwrite=args.overwrite,
                                                                         devices=args.devices)
        if args.tap in ("all", "5"):
            expected += len(_iter_input_npy_files(in_dir)) * len(h_coeff_5tap_map)
            counts["ideal_5tap"] = generate_ideal_5tap_output_vector(in_dir, out_dir, overwrite=args.overwrite,
                                                                         devices=args.devices)
    except Exception as exc:
        # the default folder, as the reference prints (:191-198)
        print(f"[FAIL] gen_ideal_output file=gen_ideal_output.py generated=0 skipped=0 failed=1 "
              f"elapsed={perf_counter() - t0:.2f}s out={DEFAULT_OUTPUT_DIR.resolve()} error=\"{exc}\"")
        raise
    total = sum(counts.values())
    print(f"[OK] gen_ideal_output file=gen_ideal_output.py generated={total} "
          f"skipped={max(expected - total, 0)} failed=0 elapsed={perf_counter() - t0:.2f}s out={out_dir} "
          f"ideal_3tap={counts['ideal_3tap']} ideal_5tap={counts['ideal_5tap']}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
