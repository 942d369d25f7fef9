"""Ideal-vs-fixed comparison report, shared by the 3-tap and 5-tap stages.

Mirrors the reference's twin modules ``fir_1d/sim/vector/gen_{3,5}tap_compare_report.py``
(identical except the tap literal): the same file pairing (``{case}__{coeff}_ideal_Ntap_y_f64.npy``
with ``..._fixed_Ntap_y_u8.npy``), validation lists and strict-mode error, CSV columns,
summary-JSON sections (config / validation / overall / by_coeff / worst_cases_by_rmse /
cases), console summary and return value.  The per-case metrics (:67-112 there) are one
fused GPU reduction (``fir_hip.compare_metrics``) instead of seven NumPy passes, every value
bit-identical to the reference's (the float64 sums added in NumPy's order).  The reference
np.loads each pair in turn (:303-304); here a plain pair (C-order float64 ideal, uint8 fixed of
the same shape, as the pipeline's stages write them) is read straight from its files into
page-locked staging by a pool of readers running ahead of the metrics calls, so the ideal
arrays' 544 MB per stage are neither page-faulted into fresh arrays nor staged again for the
upload; any other file goes through np.load at its turn, so a file np.load refuses raises the
reference's error in the reference's order (no report file is written before that point in
either).  Pinned against 15 scenarios run through the reference's own report functions
(tests/golden/report_contract.json).
"""
from __future__ import annotations

import csv
import json
import re
import time
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from pathlib import Path
from typing import Any

import numpy as np

import fir_hip
from fir_1d.sim.vector import stage_io

THIS_FILE = Path(__file__).resolve()
DEFAULT_OUTPUT_DIR = THIS_FILE.parent / "output"

CSV_FIELDS = ["key", "case_stem", "coeff_name", "height", "width", "num_samples", "max_abs_err", "mae", "rmse",
              "mean_err", "sat_low_ratio", "sat_high_ratio", "sat_ratio", "clip_needed_ratio", "ideal_file",
              "fixed_file"]
_AVG_COLS = ["max_abs_err", "mae", "rmse", "mean_err", "sat_low_ratio", "sat_high_ratio", "sat_ratio",
             "clip_needed_ratio"]
_MAX_COLS = ["max_abs_err", "mae", "rmse", "sat_ratio"]
_VALIDATION_KEYS = ["invalid_ideal_filenames", "invalid_fixed_filenames", "duplicate_ideal_keys",
                    "duplicate_fixed_keys", "missing_ideal_keys", "missing_fixed_keys", "shape_mismatch_cases"]


def name_patterns(tap: str) -> tuple[re.Pattern, re.Pattern]:
    return (re.compile(rf"^(?P<case_stem>.+?)__(?P<coeff_name>.+)_ideal_{tap}_y_f64\.npy$"),
            re.compile(rf"^(?P<case_stem>.+?)__(?P<coeff_name>.+)_fixed_{tap}_y_u8\.npy$"))


def _collect(directory: Path, pattern: re.Pattern):
    found, invalid, dups = {}, [], []
    for path in sorted((p for p in directory.glob("*.npy") if p.is_file()), key=lambda p: p.name.lower()):
        m = pattern.match(path.name)
        if m is None:
            invalid.append(path.name)
            continue
        key = (m.group("case_stem"), m.group("coeff_name"))
        if key in found:
            dups.append(f"{key[0]}__{key[1]}")
        else:
            found[key] = path
    return found, invalid, sorted(dups)


def compute_metrics(y_ideal: np.ndarray, y_fixed: np.ndarray) -> dict[str, float | int]:
    """Per-case metrics (reference gen_3tap_compare_report.py:67-112) on the GPU, for the fixed
    array as loaded: any integer / bool / float dtype, as the reference's astype(np.float64) (:85)
    takes it (no cast to uint8: int16 / int32 / float outputs keep their values)."""
    if y_ideal.shape != y_fixed.shape:
        raise ValueError(f"Shape mismatch: ideal={y_ideal.shape}, fixed={y_fixed.shape}")
    return fir_hip.compare_metrics(y_ideal, y_fixed)


class _Pair:
    """One matched (ideal, fixed) pair of the report, planned in key order."""

    def __init__(self, key, ip: Path, fp: Path):
        self.key, self.ip, self.fp = key, ip, fp
        self.yi = self.yf = None  # arrays (np.load, or views of the staging once read)
        self.shapes = None  # (ideal shape, fixed shape) when the headers alone decide a mismatch
        self.plain = None  # (shape, ideal offset, fixed offset): read into staging
        self.reads = None


def _plan_pair(key, ip: Path, fp: Path) -> _Pair:
    """Headers first; np.load (the reference's call, raising its error) for anything but a plain pair."""
    pr = _Pair(key, ip, fp)
    hi, hf = stage_io.npy_header(ip), stage_io.npy_header(fp)
    if hi is not None and hf is not None and not hi[1] and not hf[1] and hi[2] == np.dtype(np.float64) \
            and hf[2] == np.dtype(np.uint8):
        if hi[0] == hf[0]:
            pr.plain = (hi[0], hi[3], hf[3])
        else:
            pr.shapes = (hi[0], hf[0])
        return pr
    pr.yi, pr.yf = np.load(ip), np.load(fp)
    return pr


def _pairs(shared, ideal_map, fixed_map, timings: dict | None):
    """Yield the planned pairs in key order with their arrays in place: windows of at most
    stage_io.BATCH_BYTES of plain pairs are read by a reader pool into page-locked staging
    (float64 ideal arrays in one buffer, uint8 fixed arrays in another) while the metrics of the
    pairs before them run."""
    planned = [_plan_pair(k, ideal_map[k], fixed_map[k]) for k in shared]
    t_read = 0.0
    with ThreadPoolExecutor(max_workers=stage_io.save_workers()) as pool:
        i0 = 0
        while i0 < len(planned):
            i1, nbytes = i0, 0
            while i1 < len(planned):
                pl = planned[i1].plain
                b = 9 * stage_io._align(int(np.prod(pl[0], dtype=np.int64))) if pl else 0
                if i1 > i0 and nbytes + b > stage_io.BATCH_BYTES:
                    break
                nbytes += b
                i1 += 1
            window = planned[i0:i1]
            sizes = [int(np.prod(pr.plain[0], dtype=np.int64)) if pr.plain else 0 for pr in window]
            ar = stage_io.arena()  # the ideal stage's output staging, reused: no new pinned memory
            ibuf = ar.take("out", sum(stage_io._align(8 * n) for n in sizes))
            fbuf = ar.take("aux", sum(stage_io._align(n) for n in sizes))
            oi = of = 0
            for pr, n in zip(window, sizes):
                if pr.plain is None:
                    continue
                pr.yi = ibuf[oi:oi + 8 * n].view(np.float64).reshape(pr.plain[0])
                pr.yf = fbuf[of:of + n].reshape(pr.plain[0])
                oi += stage_io._align(8 * n)
                of += stage_io._align(n)
                pr.reads = (pool.submit(stage_io.read_into, pr.ip, pr.plain[1], pr.yi),
                            pool.submit(stage_io.read_into, pr.fp, pr.plain[2], pr.yf))
            for pr in window:
                if pr.reads is not None:
                    t0 = time.perf_counter()
                    ok = all(f.result() for f in pr.reads)
                    t_read += time.perf_counter() - t0
                    if not ok:  # the data did not come: np.load judges the files, as the reference would
                        pr.yi, pr.yf = np.load(pr.ip), np.load(pr.fp)
                yield pr
            i0 = i1
    if timings is not None:
        timings["read_wait_ms"] = round(t_read * 1e3, 3)


def summarize_rows(rows: list[dict[str, Any]]) -> dict[str, Any]:
    out: dict[str, Any] = {"num_cases": len(rows),
                           "num_samples_total": int(sum(int(r["num_samples"]) for r in rows))}
    for c in _AVG_COLS:
        out[f"avg_{c}"] = float(np.mean([float(r[c]) for r in rows])) if rows else 0.0
    for c in _MAX_COLS:
        out[f"max_{c}"] = float(np.max([float(r[c]) for r in rows])) if rows else 0.0
    return out


def generate_compare_report(tap: str, *, ideal_dir: Path, fixed_dir: Path, report_dir: Path, top_k: int = 5,
                            strict: bool = False, verbose: bool = True, timings: dict | None = None) -> dict[str, Any]:
    """The report stage (gen_3tap_compare_report.py:263-400).  ``timings`` (a dict) receives
    read_wait_ms (time the metrics calls waited for file reads), metrics_ms and wall_ms."""
    t_start = time.perf_counter()
    ideal_dir, fixed_dir, report_dir = Path(ideal_dir).resolve(), Path(fixed_dir).resolve(), Path(report_dir).resolve()
    if not ideal_dir.exists():
        raise FileNotFoundError(f"Ideal output directory not found: {ideal_dir}")
    if not fixed_dir.exists():
        raise FileNotFoundError(f"Fixed output directory not found: {fixed_dir}")
    ideal_re, fixed_re = name_patterns(tap)
    ideal_map, bad_ideal, dup_ideal = _collect(ideal_dir, ideal_re)
    fixed_map, bad_fixed, dup_fixed = _collect(fixed_dir, fixed_re)
    shared = sorted(set(ideal_map) & set(fixed_map))
    if not shared:
        raise ValueError(f"No matched {tap} ideal/fixed pairs found. ideal_dir={ideal_dir}, fixed_dir={fixed_dir}")

    rows, mismatched = [], []
    t_metrics = 0.0
    for pr in _pairs(shared, ideal_map, fixed_map, timings):
        key, ip, fp = pr.key, pr.ip, pr.fp
        name = f"{key[0]}__{key[1]}"
        si, sf = pr.shapes if pr.shapes is not None else (pr.yi.shape, pr.yf.shape)
        if si != sf:
            mismatched.append({"key": name, "ideal_shape": list(si), "fixed_shape": list(sf),
                               "ideal_file": ip.name, "fixed_file": fp.name})
            continue
        yi, yf = pr.yi, pr.yf
        t0 = time.perf_counter()
        m = compute_metrics(yi, yf)
        t_metrics += time.perf_counter() - t0
        pr.yi = pr.yf = None
        h, w = (int(yi.shape[0]), int(yi.shape[1])) if yi.ndim >= 2 else (1, int(yi.shape[0]))
        rows.append({"key": name, "case_stem": key[0], "coeff_name": key[1], "height": h, "width": w, **m,
                     "ideal_file": ip.name, "fixed_file": fp.name})
    rows.sort(key=lambda r: (str(r["case_stem"]), str(r["coeff_name"])))

    validation = {
        "invalid_ideal_filenames": sorted(bad_ideal), "invalid_fixed_filenames": sorted(bad_fixed),
        "duplicate_ideal_keys": dup_ideal, "duplicate_fixed_keys": dup_fixed,
        "missing_ideal_keys": [f"{a}__{b}" for a, b in sorted(set(fixed_map) - set(ideal_map))],
        "missing_fixed_keys": [f"{a}__{b}" for a, b in sorted(set(ideal_map) - set(fixed_map))],
        "shape_mismatch_cases": mismatched,
    }
    has_issue = any(len(validation[k]) > 0 for k in _VALIDATION_KEYS)
    if strict and has_issue:
        raise ValueError(
            "Validation failed in strict mode. "
            f"missing_ideal={len(validation['missing_ideal_keys'])}, "
            f"missing_fixed={len(validation['missing_fixed_keys'])}, "
            f"shape_mismatch={len(validation['shape_mismatch_cases'])}, "
            f"invalid_ideal_names={len(validation['invalid_ideal_filenames'])}, "
            f"invalid_fixed_names={len(validation['invalid_fixed_filenames'])}, "
            f"duplicate_ideal_keys={len(validation['duplicate_ideal_keys'])}, "
            f"duplicate_fixed_keys={len(validation['duplicate_fixed_keys'])}")

    overall = summarize_rows(rows)
    groups: dict[str, list] = {}
    for r in rows:
        groups.setdefault(str(r["coeff_name"]), []).append(r)
    by_coeff = {c: summarize_rows(rs) for c, rs in sorted(groups.items())}
    worst = sorted(rows, key=lambda r: (-float(r["rmse"]), str(r["key"])))[:max(top_k, 0)]

    report_dir.mkdir(parents=True, exist_ok=True)
    csv_path = report_dir / f"compare_{tap}_cases.csv"
    json_path = report_dir / f"compare_{tap}_summary.json"
    with csv_path.open("w", encoding="utf-8", newline="") as f:
        wr = csv.DictWriter(f, fieldnames=CSV_FIELDS)
        wr.writeheader()
        for r in rows:
            wr.writerow({k: r.get(k, "") for k in CSV_FIELDS})
    payload = {
        "generated_at_utc": datetime.now(timezone.utc).isoformat(),
        "config": {"ideal_dir": str(ideal_dir), "fixed_dir": str(fixed_dir), "report_dir": str(report_dir),
                   "top_k": int(top_k), "strict": bool(strict),
                   "comparison_note": "Metrics are computed on fixed(uint8 clipped) - ideal(float64 raw)."},
        "validation": validation, "overall": overall, "by_coeff": by_coeff, "worst_cases_by_rmse": worst,
        "cases": rows,
    }
    json_path.write_text(json.dumps(payload, indent=2, ensure_ascii=False) + "\n", encoding="utf-8")
    if verbose:
        print(f"[{tap} compare summary]")
        for k in ("num_cases", "num_samples_total"):
            print(f"- {k}: {overall[k]}")
        for k in ("avg_mae", "avg_rmse", "max_max_abs_err", "avg_sat_ratio"):
            print(f"- {k}: {overall[k]:.6f}")
        print("[validation]")
        for k in _VALIDATION_KEYS:
            print(f"- {k}: {len(validation[k])}")
        if worst:
            print("[worst cases by rmse]")
            for i, r in enumerate(worst, start=1):
                print(f"{i}. key={r['key']}, rmse={r['rmse']:.6f}, mae={r['mae']:.6f}, "
                      f"max_abs_err={r['max_abs_err']:.6f}")
        print(f"[reports]\n- csv: {csv_path}\n- json: {json_path}")
    if timings is not None:
        timings["metrics_ms"] = round(t_metrics * 1e3, 3)
        timings["wall_ms"] = round((time.perf_counter() - t_start) * 1e3, 3)
    return {"csv_path": str(csv_path), "json_path": str(json_path), "num_cases": overall["num_cases"],
            "num_samples_total": overall["num_samples_total"], "validation_has_issue": has_issue}


def run_cli(tap: str, generate, defaults: tuple[Path, Path, Path], argv=None) -> int:
    """The report programs' command line (gen_3tap_compare_report.py:404-475 and its 5-tap twin):
    flags, the console summary, and the ``[OK]`` / ``[FAIL]`` status line, which names the CSV on
    success and the report folder on failure; the error is raised after its line."""
    import argparse

    ap = argparse.ArgumentParser(description=f"Generate {tap} ideal/fixed comparison report (CSV/JSON + console summary).")
    ap.add_argument("--ideal-dir", type=Path, default=defaults[0])
    ap.add_argument("--fixed-dir", type=Path, default=defaults[1])
    ap.add_argument("--report-dir", type=Path, default=defaults[2])
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--strict", action="store_true")
    a = ap.parse_args(argv)
    name = f"gen_{tap}_compare_report"
    t0 = time.perf_counter()
    try:
        r = generate(ideal_dir=a.ideal_dir, fixed_dir=a.fixed_dir, report_dir=a.report_dir, top_k=a.top_k,
                     strict=a.strict)
    except Exception as exc:
        print(f"[FAIL] {name} file={name}.py generated=0 skipped=0 failed=1 "
              f"elapsed={time.perf_counter() - t0:.2f}s out={a.report_dir.resolve()} error=\"{exc}\"")
        raise
    print(f"[OK] {name} file={name}.py generated={r['num_cases']} skipped=0 failed=0 "
          f"elapsed={time.perf_counter() - t0:.2f}s out={r['csv_path']} validation_has_issue={r['validation_has_issue']}")
    return 0
