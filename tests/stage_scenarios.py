"""Stage-contract scenarios: a vector stage (fixed or ideal) run over a directory of inputs with
pre-existing outputs, odd inputs and failing coefficient sets, recorded as the files it leaves
and the exception it raises.

tests/golden/make_stage_contract.py runs every scenario through the REFERENCE's own stage
functions (fir_1d/sim/vector/gen_fixed_output.py:70-107, gen_ideal_output.py:60-88) and stores
the outcome in tests/golden/stage_contract.json; tests/test_gpu_stage_contract.py runs the same
scenarios through this repo's stages and demands the same outcome: return value, exception type
and text, and every output file byte for byte (SHA-256 of the .npy file).  This module only builds
inputs; it holds no reference code.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

import numpy as np

BANK3 = {"moving_avg": [1 / 3, 1 / 3, 1 / 3], "simple_lp": [0.25, 0.5, 0.25], "edge": [-1.0, 0.0, 1.0],
         "sharpen": [-0.125, 1.25, -0.125]}
BANK5 = {"moving_avg": [0.2] * 5, "simple_lp": [1 / 16, 4 / 16, 6 / 16, 4 / 16, 1 / 16],
         "edge": [-1 / 8, -2 / 8, 0.0, 2 / 8, 1 / 8], "sharpen": [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16]}
BAD3 = {"moving_avg": BANK3["moving_avg"], "simple_lp": BANK3["simple_lp"], "too_big": [9.0, 0.0, 0.0],
        "sharpen": BANK3["sharpen"]}
NAN3 = {"moving_avg": BANK3["moving_avg"], "not_finite": [0.25, float("nan"), 0.25], "sharpen": BANK3["sharpen"]}
MIXED = {"lp3": BANK3["simple_lp"], "lp5": BANK5["simple_lp"], "edge3": BANK3["edge"], "edge5": BANK5["edge"]}
SHAPES3 = [[4, 8], [3, 17], [5, 16]]
TEN = [[1, 1], [1, 17], [2, 33], [9, 4499], [16, 16], [5, 640], [3, 1280], [64, 64], [2, 4096], [1, 100000]]


def _imgs(shapes, kind="u8"):
    return [{"shape": s, "kind": kind} for s in shapes]


SCENARIOS = [
    {"name": "fixed_all_new", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BANK3"},
    {"name": "fixed_skip_some", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BANK3",
     "pre": [[1, "simple_lp"], [0, "edge"]]},
    {"name": "fixed_overwrite", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BANK3",
     "pre": [[1, "simple_lp"], [0, "edge"]], "overwrite": True},
    {"name": "fixed_all_exist", "stage": "fixed", "images": _imgs(SHAPES3[:1]), "coeff": "BANK3",
     "pre": [[0, "moving_avg"], [0, "simple_lp"], [0, "edge"], [0, "sharpen"]]},
    {"name": "fixed_load_error_3d", "stage": "fixed",
     "images": [{"shape": [4, 8], "kind": "u8"}, {"shape": [2, 3, 4], "kind": "u8"}, {"shape": [5, 16], "kind": "u8"}],
     "coeff": "BANK3"},
    {"name": "fixed_load_error_junk", "stage": "fixed",
     "images": [{"shape": [4, 8], "kind": "u8"}, {"shape": [3, 17], "kind": "u8"}, {"shape": [5, 16], "kind": "junk"}],
     "coeff": "BANK3"},
    {"name": "fixed_load_error_truncated", "stage": "fixed",
     "images": [{"shape": [4, 8], "kind": "u8"}, {"shape": [3, 17], "kind": "truncated"}], "coeff": "BANK3"},
    {"name": "fixed_bad_tap", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BAD3"},
    {"name": "fixed_bad_tap_skipped_in_first_image", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BAD3",
     "pre": [[0, "too_big"]]},
    {"name": "fixed_empty_images", "stage": "fixed", "images": _imgs([[0, 8], [3, 0], [2, 5]]), "coeff": "BANK3"},
    {"name": "fixed_empty_rows_then_bad_tap", "stage": "fixed", "images": _imgs([[0, 8], [2, 5]]), "coeff": "BAD3"},
    {"name": "fixed_non_u8_inputs", "stage": "fixed",
     "images": [{"shape": [3, 9], "kind": "f64"}, {"shape": [4, 7], "kind": "i16"}, {"shape": [5, 11], "kind": "u8F"},
                {"shape": [2, 6], "kind": "bool"}, {"shape": [3, 16], "kind": "u8"}], "coeff": "BANK3"},
    {"name": "fixed_q_range_error", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BANK3", "bits": [12, 32, 8]},
    {"name": "fixed_other_bits", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "BANK5", "bits": [10, 20, 16],
     "tap_label": "5tap"},
    {"name": "fixed_mixed_tap_lengths", "stage": "fixed", "images": _imgs(SHAPES3), "coeff": "MIXED"},
    {"name": "fixed_ten_images", "stage": "fixed", "images": _imgs(TEN), "coeff": "BANK3"},
    {"name": "fixed_ten_images_5tap", "stage": "fixed", "images": _imgs(TEN), "coeff": "BANK5", "tap_label": "5tap"},
    {"name": "ideal_all_new", "stage": "ideal", "images": _imgs(SHAPES3), "coeff": "BANK3"},
    {"name": "ideal_skip_some", "stage": "ideal", "images": _imgs(SHAPES3), "coeff": "BANK5",
     "pre": [[2, "edge"]], "tap_label": "5tap"},
    {"name": "ideal_bad_tap", "stage": "ideal", "images": _imgs(SHAPES3), "coeff": "NAN3"},
    {"name": "ideal_load_error_3d", "stage": "ideal",
     "images": [{"shape": [4, 8], "kind": "u8"}, {"shape": [2, 3, 4], "kind": "u8"}], "coeff": "BANK3"},
    {"name": "ideal_empty_images", "stage": "ideal", "images": _imgs([[0, 8], [3, 0], [2, 5]]), "coeff": "BANK3"},
    {"name": "ideal_non_u8_inputs", "stage": "ideal",
     "images": [{"shape": [3, 9], "kind": "f64"}, {"shape": [4, 7], "kind": "i16"}, {"shape": [5, 11], "kind": "u8F"}],
     "coeff": "BANK3"},
    {"name": "ideal_ten_images", "stage": "ideal", "images": _imgs(TEN), "coeff": "BANK5", "tap_label": "5tap"},
    {"name": "ideal_mixed_tap_lengths", "stage": "ideal", "images": _imgs(SHAPES3), "coeff": "MIXED"},
]
COEFF = {"BANK3": BANK3, "BANK5": BANK5, "BAD3": BAD3, "NAN3": NAN3, "MIXED": MIXED}


def _array(spec: dict, seed: int) -> np.ndarray | bytes:
    rng = np.random.default_rng(seed)
    shape, kind = tuple(spec["shape"]), spec["kind"]
    if kind in ("u8", "truncated", "junk"):
        return rng.integers(0, 256, shape, dtype=np.uint8)
    if kind == "u8F":
        return np.asfortranarray(rng.integers(0, 256, shape, dtype=np.uint8))
    if kind == "f64":  # in [0, 256): astype(uint8) truncates, well defined
        return rng.uniform(0.0, 255.99, shape)
    if kind == "i16":  # values past 255 wrap mod 256 under astype(uint8)
        return rng.integers(-600, 600, shape, dtype=np.int16)
    if kind == "bool":
        return rng.integers(0, 2, shape).astype(bool)
    raise ValueError(kind)


def input_name(i: int) -> str:
    return f"case_{i:03d}_img_{i}_x_u8.npy"


def build(scn: dict, root: Path) -> tuple[Path, Path]:
    """Write the scenario's inputs and pre-existing outputs under root; (input_dir, out_dir)."""
    inp, out = root / "input", root / "output"
    inp.mkdir(parents=True)
    stage = scn["stage"]
    label = scn.get("tap_label", "3tap")
    sub = out / f"{stage}_{label}"
    for i, spec in enumerate(scn["images"]):
        a = _array(spec, 1000 + i)
        p = inp / input_name(i)
        np.save(p, a)
        if spec["kind"] == "junk":
            p.write_bytes(b"this is not a .npy file\n" * 3)
        elif spec["kind"] == "truncated":
            p.write_bytes(p.read_bytes()[:-5])
    for i, coeff in scn.get("pre", []):
        sub.mkdir(parents=True, exist_ok=True)
        stem = input_name(i)[: -len("_x_u8.npy")]
        suffix = "fixed" if stage == "fixed" else "ideal"
        dt = np.uint8 if stage == "fixed" else np.float64
        np.save(sub / f"{stem}__{coeff}_{suffix}_{label}_y_{'u8' if stage == 'fixed' else 'f64'}.npy",
                np.full((2, 2), 7, dtype=dt))  # a sentinel: a skipped file keeps it
    return inp, out


def run(scn: dict, root: Path, fixed_fn, ideal_fn) -> dict:
    """Run the scenario with the given stage functions (the reference's or this repo's
    _generate_{fixed,ideal}_outputs_for_tap_map) and record the outcome."""
    inp, out = build(scn, root)
    label = scn.get("tap_label", "3tap")
    sub = out / f"{scn['stage']}_{label}"
    kw = dict(input_dir=inp.resolve(), out_dir=sub.resolve(), coeff_map=COEFF[scn["coeff"]], tap_label=label,
              overwrite=bool(scn.get("overwrite", False)))
    rec: dict = {"name": scn["name"]}
    try:
        if scn["stage"] == "fixed":
            f, a, c = scn.get("bits", [12, 32, 16])
            rec["returned"] = fixed_fn(frac_bits=f, acc_bits=a, coeff_bits=c, **kw)
        else:
            rec["returned"] = ideal_fn(**kw)
        rec["error"] = None
    except Exception as exc:  # noqa: BLE001 - the outcome under test
        rec["returned"] = None
        rec["error"] = [type(exc).__name__, str(exc).replace(str(root.resolve()), "<ROOT>").replace(str(root), "<ROOT>")]
    rec["files"] = {p.name: hashlib.sha256(p.read_bytes()).hexdigest()
                    for p in sorted(sub.iterdir())} if sub.exists() else {}
    return rec
