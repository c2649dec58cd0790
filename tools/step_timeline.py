#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 kernel trace: the launches of the
last step (from the last `rsv_sample` / first-kernel marker to the next), each
with its duration and the gap before it, and the per-step totals averaged over
the steps found.  tools/step_timeline.py TRACE.csv [FIRST_KERNEL_REGEX]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_rsv_sample<")
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first.search(r["Kernel_Name"])]
steps = []
for a, b in zip(starts, starts[1:] + [len(rows)]):
    steps.append(rows[a:b])


def short(n):
    n = n.replace("void ", "").replace("lsort::", "")
    return n[:n.find("(")][:95] if "(" in n else n[:95]


tot_busy, tot_span = [], []
for s in steps[1:]:
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
    span = int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])
    tot_busy.append(busy)
    tot_span.append(span)
last = steps[-2] if len(steps) > 2 else steps[-1]
prev_end = None
for r in last:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev_end) / 1e3 if prev_end else 0.0
    print("%8.1f us  gap %6.1f  %s" % ((en - st) / 1e3, gap, short(r["Kernel_Name"])))
    prev_end = en
if tot_busy:
    print("steps %d: kernel busy %.1f us, first start -> last end %.1f us (averages)"
          % (len(tot_busy), sum(tot_busy) / len(tot_busy) / 1e3, sum(tot_span) / len(tot_span) / 1e3))
