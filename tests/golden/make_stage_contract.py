"""Generate tests/golden/stage_contract.json by running the REFERENCE's vector stages.

Runs only in the build container, where the read-only reference is mounted at /root/reference
(override with FIR_REFERENCE).  Every scenario of tests/stage_scenarios.py (inputs, pre-existing
outputs, coefficient maps, bit widths, overwrite) is built in a scratch directory and run through
the reference's own stage functions:

  fir_1d/sim/vector/gen_fixed_output.py:70   _generate_fixed_outputs_for_tap_map
  fir_1d/sim/vector/gen_ideal_output.py:60   _generate_ideal_outputs_for_tap_map

and the outcome stored as data: the return value, or the exception's type and text, and the
SHA-256 of every file left in the output directory.  No reference source text is copied.

Usage:  python tests/golden/make_stage_contract.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("FIR_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(OUT.parent))

import stage_scenarios as S  # noqa: E402


def main() -> None:
    sys.path.insert(0, str(REF))
    from fir_1d.sim.vector import gen_fixed_output as gf  # the reference's modules
    from fir_1d.sim.vector import gen_ideal_output as gi

    assert Path(gf.__file__).resolve().is_relative_to(REF.resolve()), gf.__file__
    recs = []
    for scn in S.SCENARIOS:
        with tempfile.TemporaryDirectory(prefix="stage_contract_") as tmp:
            rec = S.run(scn, Path(tmp), gf._generate_fixed_outputs_for_tap_map, gi._generate_ideal_outputs_for_tap_map)
        print(rec["name"], rec["returned"], rec["error"], len(rec["files"]))
        recs.append(rec)
    meta = {"numpy": np.__version__, "python": sys.version.split()[0],
            "generator": "tests/golden/make_stage_contract.py", "scenarios": "tests/stage_scenarios.py"}
    (OUT / "stage_contract.json").write_text(json.dumps({"meta": meta, "scenarios": recs}, indent=1) + "\n")


if __name__ == "__main__":
    main()
