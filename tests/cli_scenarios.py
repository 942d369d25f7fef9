"""Command-line scenarios: the vector stages run as programs, as a user of the reference runs them
(``python -m fir_1d.sim.vector.<stage> --flags``): input vectors from an image folder (PNG and BMP,
gray and RGB, names sorted case-insensitively), ideal and fixed outputs for each tap selection,
skip-if-exists and ``--overwrite`` runs, both comparison reports, image restore with its policies
and ``--summary-json``; and the failing invocations (a missing folder, an invalid bit width, a
strict restore over a missing sub-directory).

tests/golden/make_cli_contract.py runs every step through the REFERENCE's stage programs and stores
what each prints (the ``[OK]`` / ``[FAIL]`` line and the report summaries; elapsed times masked,
the scratch directory written as <ROOT> and the stage package's own directory as <PKG>), its exit
status and the last line of an uncaught exception, and then every file the run left: .npy bytes,
JSON documents (timestamps dropped, paths normalised), CSV text and PNG pixels.
tests/test_cli_contract.py (the device-free steps, CPU) and tests/test_gpu_cli_contract.py (all)
run the same steps through this repo's programs and demand the same.  This module only builds
inputs; it holds no reference code.
"""
from __future__ import annotations

import hashlib
import json
import re
from pathlib import Path

import numpy as np

V = "fir_1d.sim.vector."


def _chain(extra_restore=()):
    return [
        (V + "gen_input_vectors", ["--image-dir", "{ROOT}/img", "--output-dir", "{ROOT}/vec/input"]),
        (V + "gen_input_vectors", ["--image-dir", "{ROOT}/img", "--output-dir", "{ROOT}/vec/input"]),
        (V + "gen_ideal_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--tap", "3"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--tap", "5", "--overwrite"]),
        (V + "gen_3tap_compare_report", ["--ideal-dir", "{ROOT}/vec/output/ideal_3tap", "--fixed-dir",
                                         "{ROOT}/vec/output/fixed_3tap", "--report-dir",
                                         "{ROOT}/vec/output/report_3tap", "--top-k", "2"]),
        (V + "gen_5tap_compare_report", ["--ideal-dir", "{ROOT}/vec/output/ideal_5tap", "--fixed-dir",
                                         "{ROOT}/vec/output/fixed_5tap", "--report-dir",
                                         "{ROOT}/vec/output/report_5tap"]),
        (V + "restore_images", ["--vector-output-dir", "{ROOT}/vec/output", "--output-img-dir", "{ROOT}/out_img",
                                "--summary-json", "{ROOT}/out_img/summary.json"]),
        (V + "restore_images", ["--vector-output-dir", "{ROOT}/vec/output", "--output-img-dir", "{ROOT}/out_img"]),
        *extra_restore,
    ]


SCENARIOS = [
    {"name": "chain", "steps": _chain([
        (V + "restore_images", ["--vector-output-dir", "{ROOT}/vec/output", "--output-img-dir", "{ROOT}/out_img",
                                "--kind", "ideal", "--tap", "3", "--ideal-policy", "normalize", "--overwrite"]),
        (V + "gen_ideal_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--tap", "5"]),
    ])},
    {"name": "fixed_other_bits", "steps": [
        (V + "gen_input_vectors", ["--image-dir", "{ROOT}/img", "--output-dir", "{ROOT}/vec/input"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--frac-bits", "10", "--acc-bits", "20", "--coeff-bits", "16"]),
    ]},
    {"name": "failures", "steps": [
        (V + "gen_input_vectors", ["--image-dir", "{ROOT}/no_images", "--output-dir", "{ROOT}/vec/input"]),
        (V + "gen_input_vectors", ["--image-dir", "{ROOT}/img", "--output-dir", "{ROOT}/vec/input"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--coeff-bits", "7"]),
        (V + "gen_fixed_output", ["--input-dir", "{ROOT}/vec/input", "--output-dir", "{ROOT}/vec/output",
                                  "--frac-bits", "0"]),
        (V + "gen_3tap_compare_report", ["--ideal-dir", "{ROOT}/vec/output/ideal_3tap", "--fixed-dir",
                                         "{ROOT}/vec/output/fixed_3tap", "--report-dir",
                                         "{ROOT}/vec/output/report_3tap"]),
        (V + "restore_images", ["--vector-output-dir", "{ROOT}/vec/output", "--output-img-dir", "{ROOT}/out_img",
                                "--strict"]),
        (V + "restore_images", ["--vector-output-dir", "{ROOT}/vec/nothing", "--output-img-dir", "{ROOT}/out_img"]),
    ]},
]


def build(root: Path) -> None:
    """The image folder every scenario starts from."""
    from PIL import Image
    img = root / "img"
    img.mkdir(parents=True)
    rng = np.random.default_rng(2026)
    Image.fromarray(rng.integers(0, 256, (5, 7)).astype(np.uint8), mode="L").save(img / "b_small.png")
    Image.fromarray(rng.integers(0, 256, (3, 40)).astype(np.uint8), mode="L").save(img / "A_wide.PNG")
    Image.fromarray(rng.integers(0, 256, (6, 9, 3)).astype(np.uint8), mode="RGB").save(img / "c_rgb.bmp")
    Image.fromarray(rng.integers(0, 256, (12, 20)).astype(np.uint8), mode="L").save(img / "d_tall.png")
    (img / "notes.txt").write_text("not an image\n")
    # the input folder exists, as in the reference's tree: its input stage saves before it creates
    # the folder (gen_input_vectors.py:130 vs :42), which this repo's does first (a documented fix)
    (root / "vec" / "input").mkdir(parents=True)


_ELAPSED = re.compile(r"elapsed=\d+\.\d+s")


def normalise(text: str, root: Path, pkg: Path) -> str:
    for r in {str(root.resolve()), str(root)}:
        text = text.replace(r, "<ROOT>")
    for p in {str(pkg.resolve()), str(pkg)}:
        text = text.replace(p, "<PKG>")
    return _ELAPSED.sub("elapsed=<T>s", text)


def _norm_json(obj, root, pkg):
    if isinstance(obj, dict):
        return {k: _norm_json(v, root, pkg) for k, v in obj.items() if k != "generated_at_utc"}
    if isinstance(obj, list):
        return [_norm_json(v, root, pkg) for v in obj]
    if isinstance(obj, str):
        return normalise(obj, root, pkg)
    return obj


def snapshot(root: Path, pkg: Path) -> dict:
    """Every file the run left outside the image folder."""
    from PIL import Image
    out = {}
    for p in sorted(root.rglob("*")):
        rel = p.relative_to(root).as_posix()
        if rel == "img" or rel.startswith("img/"):
            continue
        if p.is_dir():
            out[rel + "/"] = None
        elif p.suffix == ".json":
            out[rel] = _norm_json(json.loads(p.read_text(encoding="utf-8")), root, pkg)
        elif p.suffix == ".csv":
            out[rel] = normalise(p.read_text(encoding="utf-8"), root, pkg)
        elif p.suffix == ".png":
            with Image.open(p) as im:
                im.load()
                out[rel] = {"mode": im.mode, "size": list(im.size),
                            "pixels": hashlib.sha256(np.asarray(im).tobytes()).hexdigest()}
        else:
            out[rel] = hashlib.sha256(p.read_bytes()).hexdigest()
    return out


def preview_text(root: Path) -> dict:
    """The preview JSON files' exact text (their row layout is part of the format)."""
    return {p.name: p.read_text(encoding="utf-8") for p in sorted((root / "vec" / "input").glob("*_preview.json"))}


def run(scn: dict, root: Path, pkg: Path, runner) -> dict:
    """Run the scenario's steps with runner(module, argv) -> (exit status, stdout, last line of an
    uncaught exception or None) and record the outcome."""
    build(root)
    steps = []
    for module, args in scn["steps"]:
        argv = [a.replace("{ROOT}", str(root)) for a in args]
        rc, out, exc = runner(module, argv)
        steps.append({"module": module.rsplit(".", 1)[1], "args": args, "rc": rc,
                      "stdout": normalise(out, root, pkg),
                      "exception": None if exc is None else normalise(exc, root, pkg)})
    rec = {"name": scn["name"], "steps": steps, "files": snapshot(root, pkg)}
    rec["preview_text"] = {k: normalise(v, root, pkg) for k, v in preview_text(root).items()} \
        if (root / "vec" / "input").exists() else {}
    return rec
