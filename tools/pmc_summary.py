#!/usr/bin/env python3
"""Average PMC value per dispatch, per kernel, from tools/pmc.sh output."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/*/run_counter_collection.csv") + glob.glob(root + "/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        short = name.split("<")[0].replace("void lsort::", "").replace("lsort::", "")
        tmpl = name[name.find("<"):name.find(">") + 1] if "<" in name else ""
        acc[short + tmpl[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k)
    for c, v in sorted(d.items()):
        print("   %-24s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
