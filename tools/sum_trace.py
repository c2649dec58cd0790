import csv, sys, collections
for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
    tot = collections.Counter(); cnt = collections.Counter()
    for r in rows:
        name = r["Kernel_Name"]
        key = "copy" if "copyBuffer" in name or "Copy" in name else ("fill" if "fill" in name else "libsort")
        if "at::" in name: key = "torch"
        tot[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"]); cnt[key] += 1
    print(d, {k: (cnt[k], round(tot[k] / 1e6, 2)) for k in tot})
