"""Generate tests/golden/restore_contract.json by running the REFERENCE's image restore.

Runs only in the build container (reference at /root/reference, override with FIR_REFERENCE).
Every scenario of tests/restore_scenarios.py is built in a scratch directory and run through the
reference's own stage function:

  fir_1d/sim/vector/restore_images.py:104   restore_images

and the outcome stored as data: the returned summary (timestamp dropped, the scratch directory
written as <ROOT>) or the exception's type and text, and every file and directory left in the
image tree (bytes SHA-256; for PNGs the decoded mode, size and pixel SHA-256).  No reference
source text is copied.

Usage:  python tests/golden/make_restore_contract.py
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

import restore_scenarios as S  # noqa: E402


def main() -> None:
    sys.path.insert(0, str(REF))
    from fir_1d.sim.vector import restore_images as ref  # the reference's module
    import PIL

    assert Path(ref.__file__).resolve().is_relative_to(REF.resolve()), ref.__file__
    recs = []
    for scn in S.SCENARIOS:
        with tempfile.TemporaryDirectory(prefix="restore_contract_") as tmp:
            rec = S.run(scn, Path(tmp), ref.restore_images)
        print(rec["name"], rec["error"], None if rec["returned"] is None else rec["returned"]["num_converted"],
              len(rec["images"]))
        recs.append(rec)
    meta = {"numpy": np.__version__, "pillow": PIL.__version__, "python": sys.version.split()[0],
            "generator": "tests/golden/make_restore_contract.py", "scenarios": "tests/restore_scenarios.py"}
    (OUT / "restore_contract.json").write_text(json.dumps({"meta": meta, "scenarios": recs}, indent=1) + "\n")


if __name__ == "__main__":
    main()
