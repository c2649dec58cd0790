#!/usr/bin/env python3
"""Per-depth digit-pass durations and the bucket phase from a bench kernel trace
(rocprofv3 --kernel-trace of `bench.py`): mean over the sorts of each depth's
4-bit pass, the counting kernel and the retry / LSD list launches.
    python tools/pass_split.py <rocprof output dir>"""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
acc = defaultdict(list)
depth = None
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n.startswith("void lsort::k_rsv_sample<"):
        depth = 0
    elif "k_tile_pass<4, 256, 16, unsigned int, lsort::NoValue" in n and depth is not None:
        acc["pass%d" % depth].append(d)
        depth = depth + 1 if depth < 3 else None  # (the hybrid's 4 passes after its sampler)
    elif "k_bucket_count<256, 17" in n:
        acc["count"].append(d)
    elif "k_bucket_count<256, 23" in n:
        acc["retry"].append(d)
    elif "k_bucket_sort<4, 256, 23" in n:
        acc["lsdlist"].append(d)
print(sys.argv[1], "  ".join("%s %.1f (x%d)" % (k, sum(v) / len(v), len(v)) for k, v in sorted(acc.items())))
