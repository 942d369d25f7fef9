"""Report-stage scenarios: the ideal-vs-fixed comparison report (fir_1d/sim/vector/
gen_3tap_compare_report.py:263-400, and its 5-tap twin) over directories holding matched pairs,
unmatched and misnamed files, shape mismatches, non-default dtypes and memory orders, 1-D and
empty arrays, NaN / inf values, files np.load refuses, with strict mode and top_k variants.

tests/golden/make_report_contract.py runs every scenario through the REFERENCE's report function
and stores what it returns or raises and the text of the CSV and JSON it writes (the JSON's
timestamp dropped, directories written as <ROOT>) in tests/golden/report_contract.json;
tests/test_report_contract.py (CPU, the oracle's metrics) and tests/test_gpu_report_contract.py
(the GPU metrics) run them through this repo's report and demand the same.  This module only
builds inputs; it holds no reference code.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np


def _pair(stem, coeff, shape, seed, tap="3tap", ideal_dtype="f8", fixed_dtype="u1", order="C", nan=False):
    return {"stem": stem, "coeff": coeff, "shape": shape, "seed": seed, "tap": tap, "ideal_dtype": ideal_dtype,
            "fixed_dtype": fixed_dtype, "order": order, "nan": nan}


BASE = [_pair("case_000_a", "edge", [4, 9], 1), _pair("case_000_a", "simple_lp", [4, 9], 2),
        _pair("case_001_b", "edge", [1, 33], 3), _pair("case_001_b", "simple_lp", [1, 33], 4),
        _pair("case_002_c", "edge", [7, 1], 5), _pair("case_002_c", "simple_lp", [7, 1], 6)]
WIDE = [_pair(f"case_{i:03d}_w", c, s, 10 + 2 * i + j) for i, s in enumerate([[2, 4499], [9, 640], [3, 1280], [1, 100003]])
        for j, c in enumerate(("moving_avg", "sharpen"))]

SCENARIOS = [
    {"name": "valid", "pairs": BASE},
    {"name": "valid_wide", "pairs": WIDE},
    {"name": "missing_and_misnamed", "pairs": BASE, "drop_fixed": ["case_001_b__edge"],
     "drop_ideal": ["case_002_c__simple_lp"], "extra": ["notes.npy", "case_009_z_fixed_3tap_y_u8.npy"]},
    {"name": "strict_error", "pairs": BASE, "drop_fixed": ["case_001_b__edge"], "strict": True},
    {"name": "shape_mismatch", "pairs": BASE, "fixed_shape": {"case_000_a__simple_lp": [4, 8]}},
    {"name": "shape_mismatch_strict", "pairs": BASE, "fixed_shape": {"case_000_a__simple_lp": [3, 9]}, "strict": True},
    {"name": "dtypes_and_orders", "pairs": [
        _pair("case_000_a", "edge", [5, 17], 21, fixed_dtype="i2"), _pair("case_000_a", "lp", [5, 17], 22, ideal_dtype="f4"),
        _pair("case_001_b", "edge", [6, 16], 23, order="F"), _pair("case_001_b", "lp", [6, 16], 24, fixed_dtype="f8"),
        _pair("case_002_c", "edge", [3, 10], 25, fixed_dtype="b1"), _pair("case_002_c", "lp", [3, 10], 26, ideal_dtype=">f8")]},
    {"name": "one_d_and_empty", "pairs": [_pair("case_000_a", "edge", [37], 31), _pair("case_001_b", "edge", [0, 5], 32),
                                          _pair("case_002_c", "edge", [0], 33), _pair("case_003_d", "edge", [2, 3, 4], 34)]},
    {"name": "nan_and_inf", "pairs": [_pair("case_000_a", "edge", [4, 20], 41, nan=True),
                                      _pair("case_001_b", "edge", [4, 20], 42)]},
    {"name": "junk_ideal_file", "pairs": BASE, "junk": ["case_001_b__simple_lp_ideal_3tap_y_f64.npy"]},
    {"name": "junk_fixed_file", "pairs": BASE, "junk": ["case_002_c__edge_fixed_3tap_y_u8.npy"]},
    {"name": "no_pairs", "pairs": BASE, "drop_fixed": [f"{p['stem']}__{p['coeff']}" for p in BASE]},
    {"name": "top_k_zero", "pairs": BASE, "top_k": 0},
    {"name": "top_k_large", "pairs": BASE, "top_k": 100},
    {"name": "five_tap", "pairs": [dict(p, tap="5tap") for p in BASE], "tap": "5tap"},
]


def _arrays(p: dict):
    rng = np.random.default_rng(p["seed"])
    shape = tuple(p["shape"])
    ideal = rng.uniform(-60.0, 320.0, shape)
    if ideal.size:
        flat = ideal.reshape(-1)
        flat[::7] = np.round(flat[::7])  # exact hits: zero differences
    if p["nan"] and ideal.size > 3:
        flat = ideal.reshape(-1)
        flat[1], flat[2], flat[3] = np.nan, np.inf, -np.inf
    fixed = np.clip(np.round(np.nan_to_num(ideal, nan=0.0, posinf=255.0, neginf=0.0)) + rng.integers(-2, 3, shape),
                    0, 255)
    dt = {"u1": np.uint8, "i2": np.int16, "f8": np.float64, "b1": bool}[p["fixed_dtype"]]
    fixed = (fixed > 127) if dt is bool else (fixed + (rng.integers(-300, 300, shape) if dt == np.int16 else 0)).astype(dt)
    ideal = ideal.astype(np.dtype(p["ideal_dtype"]))
    if p["order"] == "F":
        ideal, fixed = np.asfortranarray(ideal), np.asfortranarray(fixed)
    return ideal, fixed


def build(scn: dict, root: Path) -> tuple[Path, Path, Path]:
    """Write the scenario's files; returns (ideal_dir, fixed_dir, report_dir)."""
    tap = scn.get("tap", "3tap")
    idir, fdir, rdir = root / f"ideal_{tap}", root / f"fixed_{tap}", root / f"report_{tap}"
    idir.mkdir(parents=True)
    fdir.mkdir(parents=True)
    for p in scn["pairs"]:
        key = f"{p['stem']}__{p['coeff']}"
        yi, yf = _arrays(p)
        if key in scn.get("fixed_shape", {}):
            yf = np.zeros(tuple(scn["fixed_shape"][key]), dtype=yf.dtype)
        if key not in scn.get("drop_ideal", []):
            np.save(idir / f"{key}_ideal_{p['tap']}_y_f64.npy", yi)
        if key not in scn.get("drop_fixed", []):
            np.save(fdir / f"{key}_fixed_{p['tap']}_y_u8.npy", yf)
    for name in scn.get("extra", []):
        np.save(idir / name, np.zeros(3))
        np.save(fdir / name, np.zeros(3, np.uint8))
    for name in scn.get("junk", []):
        d = idir if "_ideal_" in name else fdir
        (d / name).write_bytes(b"not a .npy file\n" * 4)
    return idir, fdir, rdir


def run(scn: dict, root: Path, report_fn) -> dict:
    """Run the scenario through report_fn (the reference's generate_{3,5}tap_compare_report or
    this repo's) and record the outcome with <ROOT> for the scratch directory."""
    idir, fdir, rdir = build(scn, root)
    norm = lambda s: s.replace(str(root.resolve()), "<ROOT>").replace(str(root), "<ROOT>")  # noqa: E731
    rec = {"name": scn["name"]}
    try:
        ret = report_fn(ideal_dir=idir, fixed_dir=fdir, report_dir=rdir, top_k=scn.get("top_k", 5),
                        strict=bool(scn.get("strict", False)))
        rec["returned"] = json.loads(norm(json.dumps(ret)))
        rec["error"] = None
    except Exception as exc:  # noqa: BLE001 - the outcome under test
        rec["returned"] = None
        rec["error"] = [type(exc).__name__, norm(str(exc))]
    tap = scn.get("tap", "3tap")
    csv_p, json_p = rdir / f"compare_{tap}_cases.csv", rdir / f"compare_{tap}_summary.json"
    rec["csv"] = csv_p.read_text() if csv_p.exists() else None
    if json_p.exists():
        payload = json.loads(norm(json_p.read_text()))
        payload.pop("generated_at_utc", None)
        rec["json"] = payload
    else:
        rec["json"] = None
    return rec
