#!/usr/bin/env python3
"""Per-step GPU time by kernel from a rocprofv3 --stats kernel_stats.csv.
    python tools/kstats.py <run_kernel_stats.csv> <steps> [top]"""
import csv
import sys


def main():
    path, steps = sys.argv[1], float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print("%8.1f us/step %6d calls %9.1f avg_us  %s" % (float(r["TotalDurationNs"]) / 1e3 / steps, int(r["Calls"]),
                                                           float(r["AverageNs"]) / 1e3, r["Name"][:110]))
    print("all kernels: %.3f ms per step (%g steps)" % (tot / 1e6 / steps, steps))


if __name__ == "__main__":
    main()
