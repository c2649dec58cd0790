#!/usr/bin/env python3
"""Turns gpurun_out/prof_TAG into committed summaries under profiles/:
  profiles/TAG_kernel_stats.csv      rocprofv3 --stats of the bench command
  profiles/TAG_bench.json            the bench line
  profiles/TAG_bw_probe.txt          HBM ceiling probes (tools/bw_probe)
  profiles/pmc_<kernel>.json         HBM bytes per launch from FETCH_SIZE /
                                     WRITE_SIZE (read by bench.py as `traffic`)
gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the
bytes of a streaming read, verified on this box with tools/calib_copy for
both 4-byte and 16-byte loads; WRITE_SIZE is exact.  Both are in KiB."""
import csv
import glob
import json
import pathlib
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = pathlib.Path("gpurun_out") / ("prof_" + tag)
dst = pathlib.Path("profiles")
dst.mkdir(exist_ok=True)
for f in glob.glob(str(src / "stats" / "*kernel_stats.csv")):
    shutil.copy(f, dst / ("%s_kernel_stats.csv" % tag))
if (src / "bench.json").exists():
    shutil.copy(src / "bench.json", dst / ("%s_bench.json" % tag))
if (src / "calib.txt").exists():
    shutil.copy(src / "calib.txt", dst / ("%s_calib_copy_rocprim.txt" % tag))
if (src / "bw_probe.txt").exists():
    shutil.copy(src / "bw_probe.txt", dst / ("%s_bw_probe.txt" % tag))


def per_kernel(counter):
    out = {}
    for f in glob.glob(str(src / ("pmc_" + counter) / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            key = ("tilepass" if "tile_pass" in name else "onesweep" if "onesweep" in name else
                   "downsweep" if "downsweep" in name else "tilecounts" if "tile_counts" in name else None)
            if key:
                out.setdefault(key, []).append(float(r["Counter_Value"]))
    return out


fetch, write = per_kernel("FETCH_SIZE"), per_kernel("WRITE_SIZE")
stats = {}
for f in glob.glob(str(src / "stats" / "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        stats[r["Name"]] = r
for k in sorted(set(fetch) & set(write)):
    fr = sum(fetch[k]) / len(fetch[k]) * 1024 * 2  # corrected read bytes
    wr = sum(write[k]) / len(write[k]) * 1024
    rec = {"kernel": k, "launches_sampled": len(fetch[k]), "read_bytes_per_launch": fr,
           "write_bytes_per_launch": wr, "hbm_bytes_per_launch": fr + wr,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "`bench.py --steps 5 --warmup 2`; read = 2 x FETCH_SIZE (gfx950, calibrated with "
                     "tools/calib_copy), write = WRITE_SIZE; KiB -> bytes",
           "round": tag}
    (dst / ("pmc_%s.json" % k)).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))
