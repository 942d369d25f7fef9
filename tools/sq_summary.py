"""Summarise a rocprofv3 SQ counter pass (run_counter_collection.csv): per kernel, the median
over launches of each counter, and the wave-cycle split WAIT_ANY / WAIT_INST_ANY / ACTIVE
(SQ counters count quad-cycles; MI355X_MICROARCH.md).  Usage: tools/sq_summary.py <csv> [kernel substring]"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            vals[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        print(k)
        for c in sorted(med):
            print(f"  {c:28s} {med[c]:16.0f}")
        w = med.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in med:
                    print(f"  {c + ' / WAVE_CYCLES':40s} {med[c] / w:6.3f}")


if __name__ == "__main__":
    main()
