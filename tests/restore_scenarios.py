"""Restore-stage scenarios: PNG restore of the pipeline's output vectors
(fir_1d/sim/vector/restore_images.py:104-213) over vector trees holding every kind / tap
sub-directory or only some, misnamed and misplaced files, inputs np.load refuses, 1-D / 3-D /
empty arrays, non-default dtypes, byte orders and memory orders, NaN / inf values, constant
arrays, outputs that already exist (kept, or replaced with overwrite) -- under both ideal
policies, every kind / tap selection, strict and not.

tests/golden/make_restore_contract.py runs every scenario through the REFERENCE's restore_images
and stores what it returns or raises and every file it leaves in the image tree (bytes SHA-256,
and for PNGs the decoded mode, size and pixel SHA-256), the summary's timestamp dropped and the
scratch directory written as <ROOT>; tests/test_restore_contract.py (CPU, the oracle's
conversions) and tests/test_gpu_restore_contract.py (the GPU conversions) run them through this
repo's restore_images and demand the same.  This module only builds inputs; it holds no
reference code.
"""
from __future__ import annotations

import hashlib
import json
import warnings
from pathlib import Path

import numpy as np

TAPS = ("3", "5")
# name pieces of a vector file: <stem>__<coeff>_<kind>_<tap>tap_y_<tag>.npy
STEMS = ("case_000_a", "case_001_b", "case_002_c")
COEFFS = ("edge", "simple_lp")


def _fname(stem, coeff, kind, tap):
    return f"{stem}__{coeff}_{kind}_{tap}tap_y_{'f64' if kind == 'ideal' else 'u8'}.npy"


def _ideal(shape, seed, dtype="f8", special=None, order="C"):
    rng = np.random.default_rng(seed)
    a = rng.uniform(-60.0, 320.0, shape)
    if a.size:
        flat = a.reshape(-1)
        flat[::5] = np.floor(flat[::5]) + 0.5  # ties: rint goes to even
        flat[1::9] = np.round(flat[1::9])
    if special == "nan" and a.size > 4:
        flat = a.reshape(-1)
        flat[1], flat[2], flat[3] = np.nan, np.inf, -np.inf
    if special == "inf" and a.size > 4:
        flat = a.reshape(-1)
        flat[2], flat[3] = np.inf, -np.inf
    if special == "const":
        a[...] = 77.25
    if np.dtype(dtype).kind in "iu":
        a = np.clip(a, np.iinfo(dtype).min, np.iinfo(dtype).max)
    a = a.astype(np.dtype(dtype))
    return np.asfortranarray(a) if order == "F" else a


def _fixed(shape, seed, dtype="u1", order="C"):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt == np.uint8:
        a = rng.integers(0, 256, shape).astype(np.uint8)
    elif dt == bool:
        a = rng.integers(0, 2, shape).astype(bool)
    elif dt.kind == "f":
        a = rng.uniform(-40.0, 300.0, shape)
        if a.size:
            a.reshape(-1)[::4] = np.floor(a.reshape(-1)[::4]) + 0.5
        a = a.astype(dt)
    else:
        a = rng.integers(-400, 700, shape)
        if dt.kind == "u":
            a = np.abs(a)
        a = a.astype(dt)
    return np.asfortranarray(a) if order == "F" else a


def tree(kinds=("ideal", "fixed"), taps=TAPS, shapes=((4, 9), (1, 33), (7, 1)), seed=0, **kw):
    """Files of a plain vector tree: {relpath: array spec}."""
    files = {}
    for ki, kind in enumerate(kinds):
        for ti, tap in enumerate(taps):
            for si, stem in enumerate(STEMS[:len(shapes)]):
                for ci, coeff in enumerate(COEFFS):
                    s = seed + 1000 * ki + 100 * ti + 10 * si + ci
                    spec = {"gen": kind, "shape": list(shapes[si]), "seed": s}
                    spec.update(kw.get(kind, {}))
                    files[f"{kind}_{tap}tap/{_fname(stem, coeff, kind, tap)}"] = spec
    return files


def _with(files, **extra):
    out = dict(files)
    out.update(extra)
    return out


BASE = tree()
SCENARIOS = [
    {"name": "all_clip", "files": BASE},
    {"name": "all_normalize", "files": _with(BASE, **{
        "ideal_3tap/case_003_d__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [3, 6], "seed": 7, "special": "const"}}),
     "ideal_policy": "normalize"},
    {"name": "ideal_only_tap3", "files": BASE, "kind": "ideal", "tap": "3"},
    {"name": "fixed_only_tap5", "files": BASE, "kind": "fixed", "tap": "5"},
    {"name": "ideal_only_normalize_tap5", "files": BASE, "kind": "ideal", "tap": "5", "ideal_policy": "normalize"},
    {"name": "missing_subdirs", "files": tree(kinds=("fixed",), taps=("3",))},
    {"name": "missing_subdir_strict", "files": tree(kinds=("ideal",), taps=("3",)), "strict": True},
    {"name": "invalid_names", "files": _with(tree(kinds=("ideal",), taps=("3",)), **{
        "ideal_3tap/notes.npy": {"gen": "ideal", "shape": [2, 2], "seed": 1},
        "ideal_3tap/case_009_z__edge_ideal_7tap_y_f64.npy": {"gen": "ideal", "shape": [2, 2], "seed": 2},
        "ideal_3tap/CASE_00A__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [2, 3], "seed": 3},
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_u8.npy": {"gen": "ideal", "shape": [2, 2], "seed": 4},
        "ideal_3tap/readme.txt": {"text": "not a vector\n"},
        "ideal_3tap/dir.npy/": {"dir": True}})},
    {"name": "invalid_names_strict", "files": _with(tree(kinds=("ideal",), taps=("3",)), **{
        "ideal_3tap/case_001_b__zz.npy": {"gen": "ideal", "shape": [2, 2], "seed": 1}}), "strict": True},
    {"name": "kind_tap_mismatch", "files": _with(tree(kinds=("fixed",), taps=("3", "5")), **{
        "fixed_3tap/case_001_b__lp_fixed_5tap_y_u8.npy": {"gen": "fixed", "shape": [2, 2], "seed": 1},
        "fixed_5tap/case_001_b__lp_ideal_5tap_y_f64.npy": {"gen": "ideal", "shape": [2, 2], "seed": 2}})},
    {"name": "kind_tap_mismatch_strict", "files": _with(tree(kinds=("fixed",), taps=("3",)), **{
        "fixed_3tap/case_001_b__lp_fixed_5tap_y_u8.npy": {"gen": "fixed", "shape": [2, 2], "seed": 1}}),
     "strict": True, "kind": "fixed", "tap": "3"},
    {"name": "exists_kept", "files": BASE, "existing": [
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.png", "fixed_5tap/case_000_a__simple_lp_fixed_5tap_y_u8.png"]},
    {"name": "exists_overwrite", "files": BASE, "overwrite": True, "existing": [
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.png", "fixed_5tap/case_000_a__simple_lp_fixed_5tap_y_u8.png"]},
    {"name": "exists_normalize_dir", "files": BASE, "ideal_policy": "normalize", "existing": [
        "ideal_3tap/case_000_a__edge_ideal_3tap_y_f64.png",
        "ideal_3tap_normalize/case_000_a__edge_ideal_3tap_y_f64.png"]},
    {"name": "exists_but_unreadable_input", "files": _with(BASE, **{
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.npy": {"junk": True}}),
     "existing": ["ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.png"]},
    {"name": "exists_but_1d", "files": _with(BASE, **{
        "fixed_3tap/case_002_c__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [40], "seed": 3}}),
     "existing": ["fixed_3tap/case_002_c__edge_fixed_3tap_y_u8.png"]},
    {"name": "unreadable_input_midway", "files": _with(BASE, **{
        "ideal_5tap/case_001_b__edge_ideal_5tap_y_f64.npy": {"junk": True}})},
    {"name": "truncated_input", "files": _with(BASE, **{
        "fixed_3tap/case_001_b__simple_lp_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [30, 40], "seed": 5,
                                                                "truncate": 200}})},
    {"name": "three_d_array", "files": _with(BASE, **{
        "ideal_3tap/case_002_c__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [2, 3, 4], "seed": 3}})},
    {"name": "empty_array_midway", "files": _with(BASE, **{
        "fixed_3tap/case_001_b__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [0, 5], "seed": 3}})},
    {"name": "empty_array_normalize", "files": _with(BASE, **{
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 0], "seed": 3}}),
     "ideal_policy": "normalize"},
    {"name": "fixed_dtypes", "files": tree(kinds=("fixed",), taps=("3",), shapes=((5, 17), (6, 16), (3, 10))) | {
        "fixed_3tap/case_010_i2__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 11, "dtype": "i2"},
        "fixed_3tap/case_011_f8__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 12, "dtype": "f8"},
        "fixed_3tap/case_012_b1__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 13, "dtype": "b1"},
        "fixed_3tap/case_013_f4__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 14, "dtype": "f4"},
        "fixed_3tap/case_014_u2__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 15, "dtype": "u2"},
        "fixed_3tap/case_015_be__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [5, 11], "seed": 16, "dtype": ">i4"},
        "fixed_3tap/case_016_fo__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [6, 7], "seed": 17, "order": "F"},
        "fixed_3tap/case_017_i8__edge_fixed_3tap_y_u8.npy": {"gen": "fixed", "shape": [4, 9], "seed": 18, "dtype": "i8"}}},
    {"name": "ideal_dtypes", "files": {
        "ideal_3tap/case_000_f4__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 21, "dtype": "f4"},
        "ideal_3tap/case_001_be__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 22, "dtype": ">f8"},
        "ideal_3tap/case_002_i2__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 23, "dtype": "i2"},
        "ideal_3tap/case_003_u1__edge_ideal_3tap_y_f64.npy": {"gen": "fixed", "shape": [5, 11], "seed": 24},
        "ideal_3tap/case_004_fo__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [6, 7], "seed": 25, "order": "F"},
        "ideal_3tap/case_005_f2__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 9], "seed": 26, "dtype": "f2"}}},
    {"name": "ideal_dtypes_normalize", "files": {
        "ideal_5tap/case_000_f4__edge_ideal_5tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 31, "dtype": "f4"},
        "ideal_5tap/case_001_be__edge_ideal_5tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 32, "dtype": ">f8"},
        "ideal_5tap/case_002_i2__edge_ideal_5tap_y_f64.npy": {"gen": "ideal", "shape": [5, 11], "seed": 33, "dtype": "i2"},
        "ideal_5tap/case_003_fo__edge_ideal_5tap_y_f64.npy": {"gen": "ideal", "shape": [6, 7], "seed": 34, "order": "F"}},
     "ideal_policy": "normalize"},
    {"name": "nan_inf_clip", "files": {
        "ideal_3tap/case_000_a__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 20], "seed": 41, "special": "nan"},
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 20], "seed": 42, "special": "inf"},
        "fixed_3tap/case_000_a__edge_fixed_3tap_y_u8.npy": {"gen": "ideal", "shape": [4, 20], "seed": 43, "special": "nan"}}},
    {"name": "nan_inf_normalize", "files": {
        "ideal_3tap/case_000_a__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 20], "seed": 41, "special": "nan"},
        "ideal_3tap/case_001_b__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [4, 20], "seed": 42, "special": "inf"},
        "ideal_3tap/case_002_c__edge_ideal_3tap_y_f64.npy": {"gen": "ideal", "shape": [3, 6], "seed": 44, "special": "const"}},
     "ideal_policy": "normalize"},
    {"name": "wide_rows", "files": tree(kinds=("ideal", "fixed"), taps=("3",), shapes=((2, 4499), (3, 1280), (1, 20011)))},
    {"name": "no_vector_dir", "files": BASE, "vector_dir": "missing"},
]


def _array(spec: dict) -> np.ndarray:
    if spec["gen"] == "ideal":
        return _ideal(tuple(spec["shape"]), spec["seed"], spec.get("dtype", "f8"), spec.get("special"),
                      spec.get("order", "C"))
    return _fixed(tuple(spec["shape"]), spec["seed"], spec.get("dtype", "u1"), spec.get("order", "C"))


def _existing_png(path: Path, seed: int) -> None:
    from PIL import Image
    path.parent.mkdir(parents=True, exist_ok=True)
    a = np.random.default_rng(seed).integers(0, 256, (3, 5)).astype(np.uint8)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        Image.fromarray(a, mode="L").save(path)


def build(scn: dict, root: Path) -> tuple[Path, Path]:
    """Write the scenario's vector tree (and its pre-existing images); returns (vector_dir, img_dir)."""
    vec, img = root / "vector", root / "img"
    vec.mkdir(parents=True)
    for rel, spec in scn["files"].items():
        p = vec / rel.rstrip("/")
        p.parent.mkdir(parents=True, exist_ok=True)
        if spec.get("dir"):
            p.mkdir()
        elif "text" in spec:
            p.write_text(spec["text"])
        elif spec.get("junk"):
            p.write_bytes(b"not a .npy file\n" * 4)
        else:
            np.save(p, _array(spec))
            if spec.get("truncate"):
                data = p.read_bytes()
                p.write_bytes(data[:spec["truncate"]])
    for i, rel in enumerate(scn.get("existing", [])):
        _existing_png(img / rel, 1000 + i)
    if scn.get("vector_dir") == "missing":
        vec = root / "no_such_vector_dir"
    return vec, img


def snapshot(img: Path) -> dict:
    """Every entry under the image tree: directories as None, files as their bytes' SHA-256 plus,
    for PNGs, the decoded mode, size and pixel SHA-256."""
    from PIL import Image
    out = {}
    if not img.exists():
        return out
    for p in sorted(img.rglob("*")):
        rel = p.relative_to(img).as_posix()
        if p.is_dir():
            out[rel + "/"] = None
            continue
        data = p.read_bytes()
        rec = {"sha256": hashlib.sha256(data).hexdigest()}
        if p.suffix == ".png":
            with Image.open(p) as im:
                im.load()
                rec.update(mode=im.mode, size=list(im.size),
                           pixels=hashlib.sha256(np.asarray(im).tobytes()).hexdigest())
        out[rel] = rec
    return out


def run(scn: dict, root: Path, restore_fn) -> dict:
    """Run the scenario through restore_fn (the reference's restore_images or this repo's) and
    record the outcome with <ROOT> for the scratch directory."""
    vec, img = build(scn, root)
    norm = lambda s: s.replace(str(root.resolve()), "<ROOT>").replace(str(root), "<ROOT>")  # noqa: E731
    rec = {"name": scn["name"]}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # NumPy's cast warnings and Pillow's mode deprecation
        try:
            ret = restore_fn(vector_output_dir=vec, output_img_dir=img, kind=scn.get("kind", "all"),
                             tap=scn.get("tap", "all"), ideal_policy=scn.get("ideal_policy", "clip"),
                             overwrite=bool(scn.get("overwrite", False)), strict=bool(scn.get("strict", False)))
            ret = json.loads(norm(json.dumps(ret)))
            ret.pop("generated_at_utc", None)
            rec["returned"] = ret
            rec["error"] = None
        except Exception as exc:  # noqa: BLE001 - the outcome under test
            rec["returned"] = None
            rec["error"] = [type(exc).__name__, norm(str(exc))]
    rec["images"] = snapshot(img)
    return rec
