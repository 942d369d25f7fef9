#!/usr/bin/env python3
"""Per-CALL HBM traffic of an entry point that issues several launches per call (the exact
metrics: part launches of metrics_blocks, then metrics_final): FETCH_SIZE / WRITE_SIZE summed
over every dispatch whose kernel name matches `kernels`, divided by the number of dispatches of
the `marker` kernel (one per call).  gfx950 correction as tools/pmc_summary.py (FETCH_SIZE x2).

Usage: tools/pmc_call_summary.py <dir with pmc_<wl>_FETCH_SIZE/ and _WRITE_SIZE/> <wl> <kernels regex>
                                 <marker substring> <algorithmic bytes per call> <out.json>"""
from __future__ import annotations

import csv
import json
import re
import sys
from pathlib import Path


def total(path: Path, counter: str, kernels: str, marker: str) -> tuple[float, int]:
    s, calls = 0.0, 0
    with path.open() as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            if re.search(kernels, r["Kernel_Name"]):
                s += float(r["Counter_Value"])
            if marker in r["Kernel_Name"]:
                calls += 1
    if not calls:
        raise SystemExit(f"no {marker} dispatches in {path}")
    return s, calls


def main() -> None:
    root, wl, kernels, marker, alg, out = Path(sys.argv[1]), sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), Path(sys.argv[6])
    f, nf = total(root / f"pmc_{wl}_FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE", kernels, marker)
    w, nw = total(root / f"pmc_{wl}_WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE", kernels, marker)
    rd, wr = f / nf * 1024 * 2, w / nw * 1024
    summary = {"kernel": kernels, "calls": {"FETCH_SIZE": nf, "WRITE_SIZE": nw},
               "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
               "hbm_bytes_per_launch": round(rd + wr), "algorithmic_bytes_per_launch": alg,
               "traffic_over_algorithmic": round((rd + wr) / alg, 4),
               "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced streaming reads), WRITE_SIZE x1",
               "per": f"call (all dispatches matching {kernels!r} / dispatches of {marker!r})",
               "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace, separate passes, python bench.py "
                         f"--workload {wl} --steps 10 --warmup 2 (tools/gpu_round.sh pmc_{wl})"}
    out.write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
