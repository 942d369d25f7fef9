"""Generate tests/golden/cli_contract.json by running the REFERENCE's stage programs.

Runs only in the build container (reference at /root/reference, override with FIR_REFERENCE).
Every step of tests/cli_scenarios.py runs as ``python -m fir_1d.sim.vector.<stage> <flags>`` with
the reference on PYTHONPATH, in a scratch directory; the outcome is stored as data (printed lines
with elapsed times masked and paths normalised, exit status, the uncaught exception's last line,
and the files left).  No reference source text is copied.

Usage:  python tests/golden/make_cli_contract.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("FIR_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(OUT.parent))

import cli_scenarios as S  # noqa: E402


def runner(module: str, argv: list[str]):
    env = dict(os.environ, PYTHONPATH=str(REF), PYTHONDONTWRITEBYTECODE="1")
    p = subprocess.run([sys.executable, "-m", module, *argv], capture_output=True, text=True, env=env,
                       cwd=tempfile.gettempdir(), timeout=600)
    exc = None
    if p.returncode != 0:
        lines = [ln for ln in p.stderr.strip().splitlines() if ln.strip()]
        exc = lines[-1] if lines else ""
    return p.returncode, p.stdout, exc


def main() -> None:
    import PIL

    recs = []
    for scn in S.SCENARIOS:
        with tempfile.TemporaryDirectory(prefix="cli_contract_") as tmp:
            rec = S.run(scn, Path(tmp), REF, runner)
        for st in rec["steps"]:
            print(scn["name"], st["module"], st["rc"], st["stdout"].strip().splitlines()[-1:] if st["stdout"] else "",
                  st["exception"])
        recs.append(rec)
    meta = {"numpy": np.__version__, "pillow": PIL.__version__, "python": sys.version.split()[0],
            "generator": "tests/golden/make_cli_contract.py", "scenarios": "tests/cli_scenarios.py"}
    (OUT / "cli_contract.json").write_text(json.dumps({"meta": meta, "scenarios": recs}, indent=1) + "\n")


if __name__ == "__main__":
    main()
