"""Generate tests/golden/report_contract.json by running the REFERENCE's comparison report.

Runs only in the build container (reference at /root/reference, override with FIR_REFERENCE).
Every scenario of tests/report_scenarios.py is built in a scratch directory and run through the
reference's own report functions:

  fir_1d/sim/vector/gen_3tap_compare_report.py:263   generate_3tap_compare_report
  fir_1d/sim/vector/gen_5tap_compare_report.py:263   generate_5tap_compare_report

and the outcome stored as data: the returned dict or the exception's type and text, the CSV text
and the summary JSON (timestamp dropped, the scratch directory written as <ROOT>).  No reference
source text is copied.

Usage:  python tests/golden/make_report_contract.py
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("FIR_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(OUT.parent))

import report_scenarios as S  # noqa: E402


def main() -> None:
    sys.path.insert(0, str(REF))
    from fir_1d.sim.vector import gen_3tap_compare_report as r3  # the reference's modules
    from fir_1d.sim.vector import gen_5tap_compare_report as r5

    assert Path(r3.__file__).resolve().is_relative_to(REF.resolve()), r3.__file__
    recs = []
    for scn in S.SCENARIOS:
        fn = r5.generate_5tap_compare_report if scn.get("tap") == "5tap" else r3.generate_3tap_compare_report
        with tempfile.TemporaryDirectory(prefix="report_contract_") as tmp, \
                contextlib.redirect_stdout(io.StringIO()):
            rec = S.run(scn, Path(tmp), fn)
        print(rec["name"], rec["error"], None if rec["returned"] is None else rec["returned"]["num_cases"])
        recs.append(rec)
    meta = {"numpy": np.__version__, "python": sys.version.split()[0],
            "generator": "tests/golden/make_report_contract.py", "scenarios": "tests/report_scenarios.py"}
    (OUT / "report_contract.json").write_text(json.dumps({"meta": meta, "scenarios": recs}, indent=1) + "\n")


if __name__ == "__main__":
    main()
