"""Restore PNG images from ideal/fixed output vectors.

Mirror of the reference stage ``fir_1d/sim/vector/restore_images.py`` (same arguments,
file-name pattern, output sub-directories ``{kind}_{tap}tap[_{policy}]``, skip / strict
behaviour and summary dict).  The u8 conversions run on the GPU (``fir_restore_u8``,
SURVEY §8(f) 4) with the reference's arithmetic: ``clip`` = rint + clip to [0,255]
(:51-54), ``normalize`` = min/max rescale (:57-64); fixed outputs are already uint8.
PNG encoding is host I/O (Pillow, whose zlib step releases the GIL) and most of the stage's
time (7 s of single-core encoding for the pipeline's 112 images, 272 M pixels): the main thread
walks the inputs in the reference's order -- name checks, np.load, the u8 conversion, the
skip-if-exists check, each where the reference does them -- and hands every image to a pool of
PNG writers that takes the largest pending image first (stage_io.OrderedSaver on a
LargestFirstPool), so the 13.5 M-pixel images start early and the small ones fill the tail.  The
files are encoded under temporary names and renamed into place in the reference's order; the
first image whose encoding fails is redone as the reference's own save call, which raises its
error after every image before it and none after it.  The summary and its order are the
reference's.
"""
from __future__ import annotations

import argparse
import json
import os
import re
from datetime import datetime, timezone
from pathlib import Path
from time import perf_counter
from typing import Any

import numpy as np

import fir_hip

from . import stage_io

THIS_FILE = Path(__file__).resolve()
DEFAULT_VECTOR_OUTPUT_DIR = THIS_FILE.parent / "output"
DEFAULT_OUTPUT_IMG_DIR = THIS_FILE.parent.parent / "output_img"
VALID_KINDS = ("ideal", "fixed")
VALID_TAPS = ("3", "5")
IDEAL_POLICIES = ("clip", "normalize")
FILENAME_RE = re.compile(
    r"^(?P<case_stem>.+?)__(?P<coeff_name>.+)_(?P<kind>ideal|fixed)_(?P<tap>[35])tap_y_(?P<dtype_tag>f64|u8)\.npy$")


def _to_u8_clip(a: np.ndarray) -> np.ndarray:
    return fir_hip.restore_u8(a, fir_hip.RESTORE_CLIP)


def _to_u8_normalized(a: np.ndarray) -> np.ndarray:
    return fir_hip.restore_u8(a, fir_hip.RESTORE_NORMALIZE)


def _to_image_u8(a: np.ndarray, kind: str, ideal_policy: str) -> np.ndarray:
    if a.ndim != 2:
        raise ValueError(f"Expected 2D array for image restore, got shape={a.shape}")
    if kind == "fixed":
        return a if a.dtype == np.uint8 else _to_u8_clip(a.astype(np.float64, copy=False))
    if kind != "ideal":
        raise ValueError(f"Unsupported kind={kind}")
    if ideal_policy == "clip":
        return _to_u8_clip(a.astype(np.float64, copy=False))
    if ideal_policy == "normalize":
        return _to_u8_normalized(a)
    raise ValueError(f"Unsupported ideal_policy={ideal_policy}")


def _selected(value: str, valid: tuple[str, ...]) -> list[str]:
    return list(valid) if value == "all" else [value]


# Converted images waiting for (or in) their PNG encoding, at most this many pixels (bytes).
INFLIGHT_BYTES = int(os.environ.get("FIR_RESTORE_INFLIGHT_BYTES", str(1 << 30)))


def png_workers() -> int:
    """PNG encoder threads: FIR_RESTORE_WRITERS, else the CPUs this process may run on, at most 16."""
    env = os.environ.get("FIR_RESTORE_WRITERS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _png_write(f, img: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(img, mode="L").save(f, format="PNG")


def _png_redo(path: Path, img: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(img, mode="L").save(path)  # the reference's call (restore_images.py:194-195)


def _pixel_range(rec: dict, img: np.ndarray) -> None:
    rec["pixel_min"], rec["pixel_max"] = int(img.min()), int(img.max())


def restore_images(*, vector_output_dir: Path = DEFAULT_VECTOR_OUTPUT_DIR, output_img_dir: Path = DEFAULT_OUTPUT_IMG_DIR,
                   kind: str = "all", tap: str = "all", ideal_policy: str = "clip", overwrite: bool = False,
                   strict: bool = False) -> dict[str, Any]:
    vector_output_dir, output_img_dir = Path(vector_output_dir).resolve(), Path(output_img_dir).resolve()
    if not vector_output_dir.exists():
        raise FileNotFoundError(f"Vector output directory not found: {vector_output_dir}")
    kinds, taps = _selected(kind, VALID_KINDS), _selected(tap, VALID_TAPS)
    try:
        from PIL import Image  # noqa: F401 - the reference's backend check
    except ModuleNotFoundError as exc:
        raise RuntimeError("Pillow is required to write PNG images.") from exc
    converted, skipped = [], []
    made: list = []  # (items submitted before, directory) for each directory the walk created
    ranges: list = []
    saver = stage_io.OrderedSaver(workers=png_workers(), writer=_png_write, redo=_png_redo, largest_first=True)
    try:
        try:
            _restore_all(kinds, taps, vector_output_dir, output_img_dir, ideal_policy, overwrite, strict, saver,
                         converted, skipped, made, ranges)
        finally:  # every image before the walk's end (or its error) is put in place, in order
            saver.commit()
        for f in ranges:
            f.result()
    except BaseException:
        if saver.failed_index is not None:
            # the reference stopped at the failing image: the directories it never reached go
            for before, d in reversed(made):
                if before > saver.failed_index:
                    try:
                        d.rmdir()
                    except OSError:
                        pass
        raise
    finally:
        saver.close()
    return {"generated_at_utc": datetime.now(timezone.utc).isoformat(),
            "config": {"vector_output_dir": str(vector_output_dir), "output_img_dir": str(output_img_dir),
                       "kind": kind, "tap": tap, "ideal_policy": ideal_policy, "overwrite": bool(overwrite),
                       "strict": bool(strict)},
            "num_converted": len(converted), "num_skipped": len(skipped), "converted": converted, "skipped": skipped}


def _restore_all(kinds, taps, vector_output_dir, output_img_dir, ideal_policy, overwrite, strict, saver,
                 converted, skipped, made, ranges):
    """The reference's loop (restore_images.py:128-213) with the PNG writes handed to ``saver``."""
    pending: set[Path] = set()  # outputs written by earlier items (not yet renamed into place)
    for k in kinds:
        for t in taps:
            src = vector_output_dir / f"{k}_{t}tap"
            if not src.exists():
                skipped.append({"reason": "missing_input_subdir", "kind": k, "tap": f"{t}tap", "path": str(src)})
                if strict:
                    raise FileNotFoundError(f"Expected input subdir not found: {src}")
                continue
            dst = output_img_dir / (f"{k}_{t}tap_{ideal_policy}" if k == "ideal" and ideal_policy != "clip"
                                    else f"{k}_{t}tap")
            new = [a for a in [dst, *dst.parents] if not a.exists()]
            dst.mkdir(parents=True, exist_ok=True)
            made.extend((saver.submitted, a) for a in reversed(new))
            for p in sorted((q for q in src.glob("*.npy") if q.is_file()), key=lambda q: q.name.lower()):
                m = FILENAME_RE.match(p.name)
                if m is None:
                    skipped.append({"reason": "invalid_filename", "path": str(p)})
                    if strict:
                        raise ValueError(f"Invalid vector filename: {p.name}")
                    continue
                if m.group("kind") != k or m.group("tap") != t:
                    skipped.append({"reason": "kind_tap_mismatch", "path": str(p), "expected_kind": k,
                                    "expected_tap": t, "file_kind": m.group("kind"), "file_tap": m.group("tap")})
                    if strict:
                        raise ValueError(f"Kind/tap mismatch in filename={p.name}, expected {k}_{t}tap")
                    continue
                # load and convert first, as the reference does: an unreadable or non-2-D input
                # raises even where its image already exists
                img = _to_image_u8(np.load(p), k, ideal_policy)
                out = dst / f"{p.stem}.png"
                if (out.exists() or out in pending) and not overwrite:
                    skipped.append({"reason": "exists", "path": str(out)})
                    continue
                rec = {"input_npy": str(p), "output_img": str(out), "kind": k, "tap": f"{t}tap",
                       "ideal_policy": ideal_policy if k == "ideal" else "n/a",
                       "height": int(img.shape[0]), "width": int(img.shape[1]), "dtype": str(img.dtype),
                       "pixel_min": None, "pixel_max": None}
                while saver.items and saver.pending_size() + img.size > INFLIGHT_BYTES:
                    saver.wait_oldest()  # bounded memory: the reference holds one image at a time
                    saver.commit(ready_only=True)
                saver.submit(saver.submitted, out, img, size=img.size)
                if img.size:  # the writer pool fills the pixel range (NumPy's reductions release the GIL)
                    ranges.append(saver.pool.submit(_pixel_range, rec, img, size=img.size))
                pending.add(out)
                converted.append(rec)


def _build_argparser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Restore output images from FIR ideal/fixed vector .npy files.")
    ap.add_argument("--vector-output-dir", type=Path, default=DEFAULT_VECTOR_OUTPUT_DIR)
    ap.add_argument("--output-img-dir", type=Path, default=DEFAULT_OUTPUT_IMG_DIR)
    ap.add_argument("--kind", choices=("all",) + VALID_KINDS, default="all")
    ap.add_argument("--tap", choices=("all",) + VALID_TAPS, default="all")
    ap.add_argument("--ideal-policy", choices=IDEAL_POLICIES, default="clip")
    ap.add_argument("--overwrite", action="store_true")
    ap.add_argument("--strict", action="store_true")
    ap.add_argument("--summary-json", type=Path, default=None, help="optional path for the JSON summary")
    return ap


def main(argv=None) -> int:
    args = _build_argparser().parse_args(argv)
    t0 = perf_counter()
    try:
        res = restore_images(vector_output_dir=args.vector_output_dir, output_img_dir=args.output_img_dir,
                             kind=args.kind, tap=args.tap, ideal_policy=args.ideal_policy, overwrite=args.overwrite,
                             strict=args.strict)
        extra = ""
        if args.summary_json is not None:
            path = args.summary_json.resolve()
            path.parent.mkdir(parents=True, exist_ok=True)
            path.write_text(json.dumps(res, indent=2, ensure_ascii=False) + "\n", encoding="utf-8")
            extra = f" summary_json={path}"
    except Exception as exc:
        print(f"[FAIL] restore_images file=restore_images.py generated=0 skipped=0 failed=1 "
              f"elapsed={perf_counter() - t0:.2f}s out={args.output_img_dir.resolve()} error=\"{exc}\"")
        raise
    print(f"[OK] restore_images file=restore_images.py generated={res['num_converted']} "
          f"skipped={res['num_skipped']} failed=0 elapsed={perf_counter() - t0:.2f}s "
          f"out={args.output_img_dir.resolve()}{extra}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
