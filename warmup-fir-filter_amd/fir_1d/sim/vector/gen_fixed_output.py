"""Fixed-point output vectors (.npy) for every input image x every coefficient set.

Mirror of the reference stage ``fir_1d/sim/vector/gen_fixed_output.py``: same public
entry points, keyword arguments, file naming (``{case}__{coeff}_fixed_{3,5}tap_y_u8.npy``
under ``output_dir/fixed_{3,5}tap``), skip-if-exists / ``overwrite`` behaviour, return
value (number of files generated), error order and CLI flags.  The difference is the driver:
the reference calls the golden model once per image row (:34-60) inside its loop over images
and coefficient sets (:88-107); here the whole stage is ONE device call
(``fir_hip.fir1d_fixed_images_multi``, ``stage_io.run_image_stage``): the inputs read straight
into page-locked staging, one upload, one batch launch over every image and coefficient set,
each output plane downloaded on its own and written (np.save) while the later planes are still
in flight.  ``devices`` / ``--devices N`` (Config row) instead spreads each image's
rows over several GPUs (rows are independent: no exchange).  ``timings`` (a dict) receives the
stage's breakdown: plan / load / H2D / kernel / D2H / save / wall, in milliseconds.
"""
from __future__ import annotations

import argparse
from pathlib import Path
from time import perf_counter

import numpy as np

import fir_hip
from fir_1d.model.python.fir_1d_fixed_ref import _coeff_stage, device_bits, quantize_fixed_taps
from fir_1d.model.python.fir_1d_ref import _prepare_rows_u8, _validate_h_coefficients
from fir_1d.sim.vector import stage_io
from fir_1d.sim.vector.h_coeff import h_coeff_3tap_map, h_coeff_5tap_map

THIS_FILE = Path(__file__).resolve()
DEFAULT_INPUT_DIR = THIS_FILE.parent / "input"
DEFAULT_OUTPUT_DIR = THIS_FILE.parent / "output"
_IN_SUFFIX = "_x_u8.npy"


def _iter_input_npy_files(input_dir: Path) -> list[Path]:
    return sorted((p for p in input_dir.glob("*.npy") if p.name.endswith(_IN_SUFFIX)),
                  key=lambda p: p.name.lower())


def _load_input_image_u8(path: Path) -> np.ndarray:
    x = np.load(path)
    if x.ndim != 2:
        raise ValueError(f"{path.name}: expected 2D array, got shape={x.shape}")
    return x if x.dtype == np.uint8 else x.astype(np.uint8)


def _case_stem_from_input(path: Path) -> str:
    return path.name[: -len(_IN_SUFFIX)] if path.name.endswith(_IN_SUFFIX) else path.stem


def _run_fixed_rowwise(x_u8: np.ndarray, h: list[float], *, frac_bits: int, acc_bits: int,
                       coeff_bits: int, devices=None) -> np.ndarray:
    """Every row of an H x W image through the fixed model: one GPU launch (one per device
    when ``devices`` lists several).  A non-uint8 image is prepared row by row with the
    model's own rules and exception order (fir_1d_ref._prepare_rows_u8): the reference calls
    the model per row on ``row.tolist()`` (gen_fixed_output.py:44-52), so h is checked first,
    then row 0's samples, then the bit widths and Q-range, then rows 1..H-1.  An image with
    no rows returns without any check, as the reference's loop never runs."""
    height, width = x_u8.shape
    if height == 0:
        return np.zeros((0, width), dtype=np.uint8)
    _validate_h_coefficients(h)
    taps = []
    xc = _prepare_rows_u8(x_u8, lambda: taps.append(_coeff_stage(h, frac_bits, acc_bits, coeff_bits)))
    hq = taps[0]
    f, a = device_bits(frac_bits, acc_bits)
    devs = fir_hip.parse_devices(devices)
    if len(devs) > 1:
        y = fir_hip.fir1d_fixed_rows_sharded(xc, hq, f, a, fir_hip.OUT_U8_SAT, devices=devs)
    else:
        y = fir_hip.fir1d_fixed_rows(xc, hq, f, a, fir_hip.OUT_U8_SAT, device=devs[0])
    if y.shape != (height, width):
        raise ValueError(f"Output shape mismatch: expected {(height, width)}, got {y.shape}.")
    return y


def _generate_fixed_outputs_for_tap_map(*, input_dir: Path, out_dir: Path, coeff_map: dict[str, list[float]],
                                        tap_label: str, frac_bits: int, acc_bits: int, coeff_bits: int,
                                        overwrite: bool = False, devices=None, timings: dict | None = None) -> int:
    inputs = _iter_input_npy_files(input_dir)
    if not inputs:
        raise FileNotFoundError(f"No input .npy files found in {input_dir}")
    out_dir.mkdir(parents=True, exist_ok=True)
    devs = fir_hip.parse_devices(devices)
    if len(devs) > 1:  # each image's rows over several devices, image by image
        generated = 0
        for in_path in inputs:
            x_u8 = _load_input_image_u8(in_path)
            stem = _case_stem_from_input(in_path)
            pending = []
            for coeff_name, h in coeff_map.items():
                out_path = out_dir / f"{stem}__{coeff_name}_fixed_{tap_label}_y_u8.npy"
                if not out_path.exists() or overwrite:
                    pending.append((out_path, h))
            generated += _run_bank(x_u8, pending, frac_bits=frac_bits, acc_bits=acc_bits, coeff_bits=coeff_bits,
                                   devices=devs)
        return generated
    taps: dict = {}  # coefficient set -> quantized taps, or the exception its validation raised

    def quantized(name):
        if name not in taps:
            try:
                taps[name] = quantize_fixed_taps(coeff_map[name], frac_bits, acc_bits, coeff_bits)
            except ValueError as exc:
                taps[name] = exc
        return taps[name]

    def plan_items(stem, shape):
        """The reference's inner loop (gen_fixed_output.py:92-105) without the compute: skipped
        files, then each pending set's checks in bank order (none for an image with no rows: its
        row loop never calls the model).  A failing set ends the stage there."""
        items = []
        for name in coeff_map:
            out_path = out_dir / f"{stem}__{name}_fixed_{tap_label}_y_u8.npy"
            if out_path.exists() and not overwrite:
                continue
            if shape[0] > 0:
                q = quantized(name)
                if isinstance(q, Exception):
                    return items, q
            items.append((out_path, name))
        return items, None

    f, a = device_bits(frac_bits, acc_bits)

    def compute(xs, keys, outs, ready, timing):
        """Every image under the sets ``keys``: one device call per tap length (the reference's
        banks have one), each a single batch launch."""
        calls, i = 0, 0
        while i < len(keys):
            j = i
            while j < len(keys) and len(taps[keys[j]]) == len(taps[keys[i]]):
                j += 1
            t: dict = {}
            fir_hip.fir1d_fixed_images_multi(xs, np.stack([taps[k] for k in keys[i:j]]), f, a, fir_hip.OUT_U8_SAT,
                                             device=devs[0], outs=[o[i:j] for o in outs],
                                             ready=lambda im, g, i=i: ready(im, i + g), timing=t)
            for k, v in t.items():
                timing[k] = timing.get(k, 0.0) + v
            calls += 1
            i = j
        timing["calls"] = calls

    return stage_io.run_image_stage(inputs, _case_stem_from_input, plan_items, compute, np.uint8, timings)


def _run_bank(x_u8: np.ndarray, pending: list, *, frac_bits: int, acc_bits: int, coeff_bits: int,
              devices=None) -> int:
    """All pending filters of a bank over one image: one fused launch per group of equal tap
    counts (the image is read once per 4 filters).  Taps are validated in bank order, and if
    one fails the filters before it are still written before the error propagates, as the
    reference's one-file-at-a-time loop (gen_fixed_output.py:92-105) would."""
    if not pending:
        return 0
    height, width = x_u8.shape
    if height == 0:  # the reference's row loop never calls the model: no checks, empty outputs
        for out_path, _ in pending:
            np.save(out_path, np.zeros((0, width), dtype=np.uint8))
        return len(pending)
    taps, error = [], None
    for out_path, h in pending:
        try:
            taps.append((out_path, quantize_fixed_taps(h, frac_bits, acc_bits, coeff_bits)))
        except ValueError as exc:
            error = exc
            break
    written, i = 0, 0
    while i < len(taps):
        j = i
        while j < len(taps) and len(taps[j][1]) == len(taps[i][1]):
            j += 1
        group = taps[i:j]
        if width == 0:
            ys = np.zeros((len(group), height, width), dtype=np.uint8)
        else:
            f, a = device_bits(frac_bits, acc_bits)
            devs = fir_hip.parse_devices(devices)
            ys = fir_hip.fir1d_fixed_rows_multi(np.ascontiguousarray(x_u8, dtype=np.uint8),
                                                np.stack([t for _, t in group]), f, a, fir_hip.OUT_U8_SAT,
                                                device=devs[0], devices=devs if len(devs) > 1 else None)
        written += _save_all([(out_path, y) for (out_path, _), y in zip(group, ys)])
        i = j
    if error is not None:
        raise error
    return written


def _save_all(items) -> int:
    """np.save of a group's outputs (stage_io.OrderedSaver): written concurrently, put in place in
    group order; the first failure is raised after the files before it, and none after it exists,
    as the reference's one-file-at-a-time loop (gen_fixed_output.py:92-105) leaves them."""
    saver = stage_io.OrderedSaver(workers=max(1, min(len(items), stage_io.save_workers())))
    try:
        for i, (path, y) in enumerate(items):
            saver.submit(i, path, y)
        return saver.commit()
    finally:
        saver.close()


def generate_fixed_3tap_output_vector(input_dir: Path = DEFAULT_INPUT_DIR, output_dir: Path = DEFAULT_OUTPUT_DIR,
                                      *, frac_bits: int = 12, acc_bits: int = 32, coeff_bits: int = 16,
                                      overwrite: bool = False, devices=None, timings: dict | None = None) -> int:
    return _generate_fixed_outputs_for_tap_map(
        input_dir=Path(input_dir).resolve(), out_dir=Path(output_dir).resolve() / "fixed_3tap",
        coeff_map=h_coeff_3tap_map, tap_label="3tap", frac_bits=frac_bits, acc_bits=acc_bits,
        coeff_bits=coeff_bits, overwrite=overwrite, devices=devices, timings=timings)


def generate_fixed_5tap_output_vector(input_dir: Path = DEFAULT_INPUT_DIR, output_dir: Path = DEFAULT_OUTPUT_DIR,
                                      *, frac_bits: int = 12, acc_bits: int = 32, coeff_bits: int = 16,
                                      overwrite: bool = False, devices=None, timings: dict | None = None) -> int:
    return _generate_fixed_outputs_for_tap_map(
        input_dir=Path(input_dir).resolve(), out_dir=Path(output_dir).resolve() / "fixed_5tap",
        coeff_map=h_coeff_5tap_map, tap_label="5tap", frac_bits=frac_bits, acc_bits=acc_bits,
        coeff_bits=coeff_bits, overwrite=overwrite, devices=devices, timings=timings)


def _build_argparser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Generate FIR 1D fixed output vectors for 3tap/5tap filters (GPU).")
    ap.add_argument("--input-dir", type=Path, default=DEFAULT_INPUT_DIR)
    ap.add_argument("--output-dir", type=Path, default=DEFAULT_OUTPUT_DIR)
    ap.add_argument("--tap", choices=("all", "3", "5"), default="all")
    ap.add_argument("--frac-bits", type=int, default=12)
    ap.add_argument("--acc-bits", type=int, default=32)
    ap.add_argument("--coeff-bits", type=int, default=16)
    ap.add_argument("--overwrite", action="store_true")
    ap.add_argument("--devices", default=None,
                    help="GPUs for the rows of each image: N (devices 0..N-1) or a comma list of ids")
    return ap


def main(argv=None) -> int:
    t0 = perf_counter()
    args = _build_argparser().parse_args(argv)
    in_dir, out_dir = args.input_dir.resolve(), args.output_dir.resolve()
    counts, expected = {"fixed_3tap": 0, "fixed_5tap": 0}, 0
    try:
        kw = dict(input_dir=in_dir, output_dir=out_dir, frac_bits=args.frac_bits, acc_bits=args.acc_bits,
                  coeff_bits=args.coeff_bits, overwrite=args.overwrite, devices=args.devices)
        if args.tap in ("all", "3"):
            expected += len(_iter_input_npy_files(in_dir)) * len(h_coeff_3tap_map)
            counts["fixed_3tap"] = generate_fixed_3tap_output_vector(**kw)
        if args.tap in ("all", "5"):
            expected += len(_iter_input_npy_files(in_dir)) * len(h_coeff_5tap_map)
            counts["fixed_5tap"] = generate_fixed_5tap_output_vector(**kw)
    except Exception as exc:
        # the default folder, as the reference prints (:246-253)
        print(f"[FAIL] gen_fixed_output file=gen_fixed_output.py generated=0 skipped=0 failed=1 "
              f"elapsed={perf_counter() - t0:.2f}s out={DEFAULT_OUTPUT_DIR.resolve()} error=\"{exc}\"")
        raise
    total = sum(counts.values())
    print(f"[OK] gen_fixed_output file=gen_fixed_output.py generated={total} "
          f"skipped={max(expected - total, 0)} failed=0 elapsed={perf_counter() - t0:.2f}s out={out_dir} "
          f"fixed_3tap={counts['fixed_3tap']} fixed_5tap={counts['fixed_5tap']}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
