#!/usr/bin/env python3
"""Mean duration of a kernel's LAST n launches in a rocprofv3 kernel trace: the roofline loop
bench.py runs last (n = --steps back-to-back launches), to set beside roofline.kernel_avg_us.
The --stats average also includes the warmup and the timed steps (launched between host-side
step work, slightly slower under the profiler).  Usage: prof_tail.py <run_kernel_trace.csv> <kernel substr> [n]"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[3]) if len(sys.argv) > 3 else 200
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
tail = d[-n:]
print(f"{sys.argv[2]}: {len(d)} launches, all-launch mean {statistics.mean(d):.2f} us, "
      f"last {len(tail)} (roofline loop) mean {statistics.mean(tail):.2f} us, median {statistics.median(tail):.2f} us")
