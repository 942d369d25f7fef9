"""Input vectors: grayscale uint8 images -> ``case_{idx:03d}_{stem}_x_u8.npy`` + preview JSON + manifest.

Mirror of the reference stage ``fir_1d/sim/vector/gen_input_vectors.py`` (same file names,
preview / manifest fields, skip-if-exists).  Image decoding is host I/O and out of the GPU
path's scope; it uses Pillow like the reference (``convert("L")``, :19-33).  Two
differences: the output directory is created before the first ``np.save`` (the reference
saves first and fails on a fresh checkout, :130 vs :42), and ``image_dir`` may also be an
``.npz`` archive of already-decoded uint8 images (``fir_1d/sim/img_u8.npz``), so the
pipeline runs without re-decoding JPEGs (libjpeg versions can differ).
"""
from __future__ import annotations

import argparse

import json
from pathlib import Path
from time import perf_counter

import numpy as np

THIS_FILE = Path(__file__).resolve()
DEFAULT_IMAGE_DIR = THIS_FILE.parent.parent / "img"
DEFAULT_OUTPUT_DIR = THIS_FILE.parent / "input"
SUPPORTED_EXTS = {".bmp", ".png", ".jpg", ".jpeg"}


def _decode_gray_u8(path: Path) -> np.ndarray:
    try:
        from PIL import Image
    except ModuleNotFoundError as exc:
        raise RuntimeError("Pillow is required to decode images (or pass an .npz of uint8 arrays).") from exc
    with Image.open(path) as img:
        arr = np.asarray(img.convert("L"), dtype=np.uint8)
    if arr.ndim != 2:
        raise ValueError(f"Expected 2D grayscale image, got shape={arr.shape}.")
    return arr


def _sources(image_dir: Path) -> list[tuple[str, str, str, callable]]:
    """(stem, image name, source path, loader) in the reference's order (case-insensitive file
    name); an .npz archive's arrays stand in for image files (stem = name = the key's image part)."""
    if image_dir.is_file() and image_dir.suffix == ".npz":
        with np.load(image_dir) as d:
            arrays = {k: d[k] for k in d.files}
        out = []
        for key in sorted(arrays, key=str.lower):
            stem = key.split("_", 2)[2] if key.startswith("case_") else key  # case_000_<stem>
            out.append((stem, stem, str(image_dir), (lambda a=arrays[key]: a)))
        return out
    files = sorted((p for p in image_dir.iterdir() if p.is_file() and p.suffix.lower() in SUPPORTED_EXTS),
                   key=lambda p: p.name.lower())
    return [(p.stem, p.name, str(p), (lambda p=p: _decode_gray_u8(p))) for p in files]


def _preview(a: np.ndarray, max_rows: int = 8, max_cols: int = 16) -> dict:
    h, w = a.shape
    pr, pc = min(h, max_rows), min(w, max_cols)
    return {"preview_kind": "top_left_patch", "preview_shape": [pr, pc], "preview_rows_u8": a[:pr, :pc].tolist(),
            "stats": {"min": int(a.min()), "max": int(a.max()), "mean": float(a.mean()), "std": float(a.std())}}


def _preview_text(payload: dict) -> str:
    """The reference's preview layout (gen_input_vectors.py:46-75): one ``"key": value,`` line per
    field, then every preview row on a line of its own."""
    lines = ["{"]
    lines += [f"  {json.dumps(k, ensure_ascii=False)}: {json.dumps(v, ensure_ascii=False)},"
              for k, v in payload.items() if k != "preview_rows_u8"]
    rows = payload["preview_rows_u8"]
    lines.append('  "preview_rows_u8": [')
    lines += [f"    {json.dumps(r, separators=(',', ':'), ensure_ascii=False)}{',' if i < len(rows) - 1 else ''}"
              for i, r in enumerate(rows)]
    lines += ["  ]", "}"]
    return "\n".join(lines) + "\n"


def generate_input_vector_jsons(image_dir: Path = DEFAULT_IMAGE_DIR, output_dir: Path = DEFAULT_OUTPUT_DIR, *,
                                overwrite: bool = False) -> dict:
    image_dir, output_dir = Path(image_dir).resolve(), Path(output_dir).resolve()
    if not image_dir.exists():
        raise FileNotFoundError(f"Image directory not found: {image_dir}")
    sources = _sources(image_dir)
    if not sources:
        raise FileNotFoundError(f"No image files found in: {image_dir}")
    output_dir.mkdir(parents=True, exist_ok=True)
    cases, generated, skipped = [], 0, 0
    for idx, (stem, name, source, load) in enumerate(sources):
        a = load()  # decoded first, as the reference does: an undecodable image raises even when skipped
        case = f"case_{idx:03d}_{stem}"
        data_file, preview_file = output_dir / f"{case}_x_u8.npy", output_dir / f"{case}_preview.json"
        if data_file.exists() and preview_file.exists() and not overwrite:
            skipped += 1
        else:
            np.save(data_file, a)
            payload = {"case_name": case, "image_name": name, "source_path": source, "width": a.shape[1],
                       "height": a.shape[0], "dtype": "uint8", "layout": "row_major_2d", "data_file": data_file.name,
                       **_preview(a)}
            preview_file.write_text(_preview_text(payload), encoding="utf-8")
            generated += 1
        cases.append({"case_name": case, "image_name": name, "width": int(a.shape[1]), "height": int(a.shape[0]),
                      "dtype": "uint8", "data_npy": data_file.name, "preview_json": preview_file.name})
    manifest = {"note": "FIR 1D input vectors: pixel data in .npy, small previews in .json.",
                "source_image_dir": str(image_dir), "output_dir": str(output_dir), "num_images": len(cases),
                "overwrite": bool(overwrite), "generated_cases": generated, "skipped_cases": skipped, "cases": cases}
    (output_dir / "input_vector_manifest.json").write_text(json.dumps(manifest, indent=2) + "\n", encoding="utf-8")
    return manifest


def _build_argparser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Generate FIR 1D input vectors (.npy) and preview/manifest JSON files.")
    ap.add_argument("--image-dir", type=Path, default=DEFAULT_IMAGE_DIR,
                    help="image folder, or a .npz of decoded uint8 images")
    ap.add_argument("--output-dir", type=Path, default=DEFAULT_OUTPUT_DIR)
    ap.add_argument("--overwrite", action="store_true")
    return ap


def main(argv=None) -> int:
    t0 = perf_counter()
    args = _build_argparser().parse_args(argv)
    try:
        m = generate_input_vector_jsons(image_dir=args.image_dir, output_dir=args.output_dir, overwrite=args.overwrite)
    except Exception as exc:
        # the default folder, as the reference prints (:208-214)
        print(f"[FAIL] gen_input_vectors file=gen_input_vectors.py generated=0 skipped=0 failed=1 "
              f"elapsed={perf_counter() - t0:.2f}s out={DEFAULT_OUTPUT_DIR.resolve()} error=\"{exc}\"")
        raise
    print(f"[OK] gen_input_vectors file=gen_input_vectors.py generated={m['generated_cases']} "
          f"skipped={m['skipped_cases']} failed=0 elapsed={perf_counter() - t0:.2f}s out={m['output_dir']}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
