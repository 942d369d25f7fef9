#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into the per-launch HBM traffic that bench.py reports.

Input: the two separate passes `rocprofv3 --pmc FETCH_SIZE --kernel-trace ...` and
`rocprofv3 --pmc WRITE_SIZE --kernel-trace ...` (tools/gpu_round.sh step `pmc`), each a
run_counter_collection.csv.  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.

The summary records the build id of the library the passes ran (fir_hip.build_id(), i.e. the
source hash the .so was built from): bench.py attaches a summary's traffic only to runs of that
same build.  Run it on the box, in the same call as the passes.

Usage: tools/pmc_summary.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <kernel substring>
                            <algorithmic bytes per launch> <out.json> [dir prefix, default pmc_]
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from pathlib import Path


def per_launch(path: Path, counter: str, kernel: str) -> list[float]:
    vals = []
    with path.open() as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel {kernel!r} in {path}")
    return vals


def build_id() -> str:
    repo = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(repo / "warmup-fir-filter_amd"))
    import fir_hip

    return fir_hip.build_id()


def main() -> None:
    root, kernel, alg, out = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3]), Path(sys.argv[4])
    pre = sys.argv[5] if len(sys.argv) > 5 else "pmc_"
    fetch = per_launch(root / f"{pre}FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE", kernel)
    write = per_launch(root / f"{pre}WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE", kernel)
    fetch_b = statistics.median(fetch) * 1024 * 2  # KiB -> B, x2 gfx950 correction
    write_b = statistics.median(write) * 1024
    summary = {
        "kernel": kernel,
        "launches": {"FETCH_SIZE": len(fetch), "WRITE_SIZE": len(write)},
        "fetch_size_kib_median": statistics.median(fetch),
        "write_size_kib_median": statistics.median(write),
        "read_bytes_per_launch": int(fetch_b),
        "write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 4),
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced streaming reads), WRITE_SIZE x1",
        "source": str(root),
        "build_id": build_id(),
    }
    out.write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
