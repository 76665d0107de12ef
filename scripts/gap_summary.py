#!/usr/bin/env python
"""Per-kernel durations and the idle gaps before each launch, from a
rocprofv3 --kernel-trace CSV (scripts/gap_probe.py, bench.py):
    python scripts/gap_summary.py <run_kernel_trace.csv> [last N launches]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
    prev = None
    for r in rows[-last:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        print(f"gap {gap:8.1f} us  dur {(e - s) / 1000:8.1f} us  {r['Kernel_Name'][:70]}")
        prev = e


if __name__ == "__main__":
    main()
