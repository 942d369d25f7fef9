"""3-tap ideal-vs-fixed comparison report (mirror of the reference module of the same name).

Same entry point, defaults, outputs (``report_3tap/compare_3tap_cases.csv``,
``compare_3tap_summary.json``) and return value; the shared implementation (with the
GPU metrics reduction) is fir_1d.sim.vector.gen_compare_report.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any

from fir_1d.sim.vector.gen_compare_report import DEFAULT_OUTPUT_DIR, generate_compare_report, run_cli

DEFAULT_IDEAL_3TAP_DIR = DEFAULT_OUTPUT_DIR / "ideal_3tap"
DEFAULT_FIXED_3TAP_DIR = DEFAULT_OUTPUT_DIR / "fixed_3tap"
DEFAULT_REPORT_DIR = DEFAULT_OUTPUT_DIR / "report_3tap"


def generate_3tap_compare_report(*, ideal_dir: Path = DEFAULT_IDEAL_3TAP_DIR,
                                  fixed_dir: Path = DEFAULT_FIXED_3TAP_DIR, report_dir: Path = DEFAULT_REPORT_DIR,
                                  top_k: int = 5, strict: bool = False) -> dict[str, Any]:
    return generate_compare_report("3tap", ideal_dir=ideal_dir, fixed_dir=fixed_dir, report_dir=report_dir,
                                   top_k=top_k, strict=strict)


def main(argv=None) -> int:
    return run_cli("3tap", generate_3tap_compare_report,
                   (DEFAULT_IDEAL_3TAP_DIR, DEFAULT_FIXED_3TAP_DIR, DEFAULT_REPORT_DIR), argv)


if __name__ == "__main__":
    raise SystemExit(main())
