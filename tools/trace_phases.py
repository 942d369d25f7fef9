#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace (run_kernel_trace.csv) into the bench's phases -- runs of
back-to-back dispatches separated by idle gaps longer than --gap us (each host synchronise between
phases leaves one) -- and print per phase: launches, mean / median / stdev / min / max duration,
and every launch slower than --slow x the median with its neighbours' times and gaps.

Usage: python tools/trace_phases.py <run_kernel_trace.csv> [--kernel SUBSTR] [--gap 20] [--slow 2]
"""
import argparse
import csv
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--slow", type=float, default=2.0)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    s = [(int(r["Start_Timestamp"]) - t0) / 1e3 for r in rows]
    e = [(int(r["End_Timestamp"]) - t0) / 1e3 for r in rows]
    d = [b - a_ for a_, b in zip(s, e)]
    queues = sorted({(r["Agent_Id"], r["Queue_Id"], r["Stream_Id"]) for r in rows})
    names = sorted({r["Kernel_Name"][:70] for r in rows})
    print(f"{len(rows)} dispatches, queues {queues}, kernels {names}")
    cuts = [0] + [i for i in range(1, len(rows)) if s[i] - e[i - 1] > a.gap] + [len(rows)]
    med_all = st.median(d)
    for p, (i0, i1) in enumerate(zip(cuts, cuts[1:])):
        x = d[i0:i1]
        gap = s[i0] - e[i0 - 1] if i0 else 0.0
        print(f"phase {p}: dispatches {i0}..{i1 - 1} ({i1 - i0}), idle gap before {gap:.1f} us: mean {st.mean(x):.2f} "
              f"median {st.median(x):.2f} stdev {st.pstdev(x):.2f} min {min(x):.1f} max {max(x):.1f} us")
    for i, v in enumerate(d):
        if v > a.slow * med_all:
            print(f"slow dispatch {i}: {v:.1f} us ({v / med_all:.1f}x the median), starts {s[i]:.1f} us")
            for k in range(max(0, i - 3), min(len(rows), i + 4)):
                gap = s[k] - e[k - 1] if k else 0.0
                print(f"   {k}: start {s[k]:.1f} end {e[k]:.1f} dur {d[k]:.1f} gap_before {gap:.1f}")


if __name__ == "__main__":
    main()
