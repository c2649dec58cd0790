#!/usr/bin/env python3
"""Kernel resource table from `make asm` remarks: tools/kres.py LOG [REGEX]"""
import re, subprocess, sys
log = open(sys.argv[1]).read().splitlines()
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cur, rows = None, []
for ln in log:
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, lab in (("VGPRs: ", "vgpr"), ("Occupancy [waves/SIMD]: ", "occ"), ("LDS Size [bytes/block]: ", "lds")):
        if cur is not None and key in ln and "AGPR" not in ln:
            cur[lab] = ln.split(key)[1].split()[0]
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
for r, d in zip(rows, dem):
    d = d.replace("lsort::", "").replace("unsigned int", "u32").replace("unsigned long", "u64")
    if pat and not pat.search(d):
        continue
    print("%4s vgpr  occ %2s  lds %6s  %s" % (r.get("vgpr", "?"), r.get("occ", "?"), r.get("lds", "?"), d[:150]))
