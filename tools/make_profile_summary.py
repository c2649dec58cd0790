#!/usr/bin/env python3
"""Turns gpurun_out/prof_TAG (tools/collect_profiles.sh) into committed
summaries under profiles/ -- all of the driver's exact bench command:
  TAG_kernel_stats.csv        rocprofv3 --stats
  TAG_rocprof_tilepass.json   average duration of the headline pass kernel
                              (4-bit k_tile_pass on the 2^28-key workload) in
                              the kernel trace: all its launches, and the
                              timed steps' launches (bench.py reads this)
  TAG_pmc_tilepass.json       HBM bytes per launch of the same launches from
                              FETCH_SIZE / WRITE_SIZE (bench.py's `traffic`)
  TAG_legs.json               the same (rocprof average + FETCH/WRITE bytes per
                              launch) for the other legs' dominant kernels:
                              configs[2]'s 8-bit passes and bucket counter,
                              configs[4]'s pair passes (16384-pair depth 0,
                              8192-pair table depths) and k_bucket_pairs, the
                              gpuPartial legs' 8-bit pass (bench.py reads it)
  TAG_bench.json, TAG_bw_probe.txt, TAG_calib_copy_rocprim.txt
gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the
bytes of a streaming read (verified on the box with tools/calib_copy, 4- and
16-byte loads); WRITE_SIZE is exact.  Both are in KiB."""
import csv
import glob
import json
import pathlib
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
src = pathlib.Path("gpurun_out") / ("prof_" + tag)
dst = pathlib.Path("profiles")
cmd = (src / "cmd.txt").read_text().strip() if (src / "cmd.txt").exists() else "?"
for f in glob.glob(str(src / "stats" / "**" / "*kernel_stats.csv"), recursive=True):
    shutil.copy(f, dst / ("%s_kernel_stats.csv" % tag))
for name, out in (("bench.json", "bench.json"), ("calib.txt", "calib_copy_rocprim.txt"),
                  ("bw_probe.txt", "bw_probe.txt")):
    if (src / name).exists():
        shutil.copy(src / name, dst / ("%s_%s" % (tag, out)))

KEYS = 1 << 28
HEADLINE = "k_tile_pass<4, 256, 16, unsigned int, lsort::NoValue"


def _groups(row):
    gx = int(float(row.get("Grid_Size_X", row.get("Grid_Size", 0)) or 0))
    wx = int(float(row.get("Workgroup_Size_X", row.get("Workgroup_Size", 256)) or 256))
    return gx // wx if gx >= wx * 1024 else gx  # grid in work-items or in workgroups


def headline(row):
    """The bench's headline pass: 4-bit keys-only RadixDigit k_tile_pass over
    the 2^28-key workload -- the MSD hybrid's four digit passes, whose grids
    are the 65536 tiles plus at most one partial tile per segment (16, 256,
    4096 segments at depths 1-3), or at depth 1 after the reserved depth 0
    the slices' capacity tiles (~75K)."""
    name = row.get("Kernel_Name", "")
    if HEADLINE not in name or "BiasedDigit" in name or "LutDigit" in name:
        return False
    # the hybrid's passes (ANY_ORDER, the last template argument), not the
    # LSD variant's (variants.lsd runs after the timed steps)
    if not name.split(">(")[0].endswith("true"):
        return False
    # depth 1 after the reserved depth 0: tiles numbered by slice capacity
    # (radix_kernels.hip rsv_capacity_bound + one partial tile per slice)
    rsv_bound = (KEYS + KEYS // 8 + KEYS // 64 + 8 * 16 * 4096 + 1024 + 4095) // 4096 + 128
    return KEYS // 4096 <= _groups(row) <= max(KEYS // 4096 + 4096, rsv_bound)


def bucketsort(row):
    """The headline's bucket sort: the counting placement's first-size launch
    over the 65536 buckets (round 4: its own kernel, k_bucket_count), not
    variants.bucket_lsd_steps' LSD steps (k_bucket_sort)."""
    name = row.get("Kernel_Name", "")
    return "k_bucket_count<256," in name and _groups(row) == 65536  # (configs[2]'s are 1024-thread blocks)


trace = sorted(glob.glob(str(src / "stats" / "**" / "*kernel_trace.csv"), recursive=True))
durs = []
for f in trace:
    for r in csv.DictReader(open(f)):
        if headline(r):
            durs.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
durs.sort()
if durs:
    us = [d for _, d in durs]
    # the command's warm-up and timed steps, digit passes per sort (MSD hybrid:
    # 16 bits / 4); the hybrid's launches in trace order are the warm-up
    # sorts', the timed sorts', then the later steps' and variants'
    warm, steps, per = 5, 20, 4
    timed = us[warm * per:(warm + steps) * per]
    rec = {"kernel": "k_tile_pass<4,...> (4-bit keys-only digit pass of the MSD hybrid, 65536+ tiles)", "cmd": cmd,
           "launches": len(timed), "avg_launch_us": sum(timed) / len(timed),
           "all_launches": len(us), "avg_all_us": sum(us) / len(us),
           "min_us": min(us), "max_us": max(us),
           "note": "avg_launch_us = launches 21-100 of the hybrid's 4-bit passes in trace order (the 20 timed sorts, "
                   "after the 5 warm-up sorts' 20); avg_all_us = every such launch (warm-up, timed, the 2 breakdown "
                   "steps, variants.bucket_lsd_steps)"}
    (dst / ("%s_rocprof_tilepass.json" % tag)).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))


def pmc(counter, pick=None):
    pick = pick or headline
    vals = []
    for f in glob.glob(str(src / ("pmc_" + counter) / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pick(r):
                vals.append(float(r["Counter_Value"]))
    return vals


fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
if fetch and write:
    fr = sum(fetch) / len(fetch) * 1024 * 2
    wr = sum(write) / len(write) * 1024
    rec = {"kernel": "tilepass", "launches_sampled": len(fetch), "read_bytes_per_launch": fr,
           "write_bytes_per_launch": wr, "hbm_bytes_per_launch": fr + wr, "algorithmic_bytes_per_launch": 8.0 * KEYS,
           "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of `%s`; "
                     "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; KiB -> bytes; headline pass launches only" % cmd,
           "round": tag}
    (dst / ("%s_pmc_tilepass.json" % tag)).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))


# the bucket sort (the MSD hybrid's last step: one HBM read and write per key)
fetch, write = pmc("FETCH_SIZE", bucketsort), pmc("WRITE_SIZE", bucketsort)
bs = []
bs_name = "k_bucket_count"
for f in trace:
    for r in csv.DictReader(open(f)):
        if bucketsort(r):
            bs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            nm = r["Kernel_Name"]
            bs_name = "k_bucket_count" + nm[nm.find("<"):nm.find(">") + 1].replace("lsort::", "")
if fetch and write and bs:
    fr = sum(fetch) / len(fetch) * 1024 * 2
    wr = sum(write) / len(write) * 1024
    rec = {"kernel": "%s (2^16 buckets of the 2^28-key workload)" % bs_name, "cmd": cmd,
           "launches": len(bs), "avg_launch_us": sum(bs) / len(bs), "read_bytes_per_launch": fr,
           "write_bytes_per_launch": wr, "algorithmic_bytes_per_launch": 8.0 * KEYS,
           "method": "same runs as %s_pmc_tilepass.json" % tag, "round": tag}
    (dst / ("%s_bucketsort.json" % tag)).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))


# ---------------------------------------------------------------------------
# the other legs of the N = 1 line (bench.py variants.c3 / c5 / partial*)
# ---------------------------------------------------------------------------
def _name(r):
    return r.get("Kernel_Name", "")


def _wg(r):
    return int(float(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0))


LEGS = {
    # configs[2]: 2^30 u32 keys, the MSD hybrid at 8-bit digits (depth 0 reserved, depth 1 from the table)
    "c3_pass": (lambda r: "k_tile_pass<8, 512, 16, unsigned int, lsort::NoValue" in _name(r)
                and _name(r).split(">(")[0].endswith("true") and _groups(r) >= (1 << 30) // 8192,
                8.0 * (1 << 30), "k_tile_pass<8,512,16,u32> (configs[2] hybrid digit passes, 2^30 keys)"),
    "c3_bucket": (lambda r: "k_bucket_count<1024," in _name(r), 8.0 * (1 << 30),
                  "k_bucket_count<1024,17,...> (configs[2] bucket counter, 2^30 keys)"),
    "c3_counts": (lambda r: "k_tile_counts<8, 512, 16, unsigned int" in _name(r) and _groups(r) >= (1 << 30) // 8192,
                  4.0 * (1 << 30), "k_tile_counts<8,...,u32> (configs[2] depth-1 count read, 2^30 keys)"),
    # configs[4] per-GPU share: 2^28 (u64, u32) pairs
    "c5_pass_depth0": (lambda r: "k_tile_pass<8," in _name(r) and "unsigned long, unsigned int" in _name(r)
                       and _wg(r) == 1024, 24.0 * (1 << 28),
                       "k_tile_pass<8,1024,...,u64,u32> (configs[4] depth 0, 16384-pair tiles)"),
    "c5_pass_table": (lambda r: "k_tile_pass<8," in _name(r) and "unsigned long, unsigned int" in _name(r)
                      and _wg(r) == 512, 24.0 * (1 << 28),
                      "k_tile_pass<8,512,...,u64,u32> (configs[4] table depth, 8192-pair tiles)"),
    "c5_bucket": (lambda r: "k_bucket_pairs<" in _name(r), 24.0 * (1 << 28),
                  "k_bucket_pairs<1024,...> (configs[4] bucket sort, 2^28 pairs)"),
    # gpuPartial at the reference's workload (2^28 keys, stable LSD 8-bit passes)
    "partial_pass": (lambda r: "k_tile_pass<8, 512, 16, unsigned int, lsort::NoValue" in _name(r)
                     and _name(r).split(">(")[0].endswith("false")
                     and (1 << 28) // 8192 <= _groups(r) <= (1 << 28) // 8192 + 1, 8.0 * (1 << 28),
                     "k_tile_pass<8,512,16,u32> stable LSD pass (gpuPartial legs, 2^28 keys)"),
}
legs = {}
for leg, (pick, alg, label) in LEGS.items():
    ds = []
    for f in trace:
        for r in csv.DictReader(open(f)):
            if pick(r):
                ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not ds:
        continue
    rec = {"kernel": label, "launches": len(ds), "avg_launch_us": sum(ds) / len(ds),
           "algorithmic_bytes_per_launch": alg,
           "frac_rocprof": round(alg / (sum(ds) / len(ds) * 1e-6) / 1e9 / 8000.0, 4)}
    fetch, write = pmc("FETCH_SIZE", pick), pmc("WRITE_SIZE", pick)
    if fetch and write:
        rec["read_bytes_per_launch"] = sum(fetch) / len(fetch) * 1024 * 2
        rec["write_bytes_per_launch"] = sum(write) / len(write) * 1024
        rec["hbm_bytes_per_launch"] = rec["read_bytes_per_launch"] + rec["write_bytes_per_launch"]
        rec["traffic_over_algorithmic"] = round(rec["hbm_bytes_per_launch"] / alg, 4)
    legs[leg] = rec
if legs:
    out = {"cmd": cmd, "round": tag, "method": "rocprofv3 kernel trace (durations) and --pmc FETCH_SIZE / WRITE_SIZE "
           "in separate runs of the same command; read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE, KiB -> bytes",
           "legs": legs}
    (dst / ("%s_legs.json" % tag)).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))
