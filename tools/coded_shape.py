#!/usr/bin/env python3
"""GPU work per rank of the C engine's schedules at configs[3]'s per-rank size
(2^29 keys) with R ranks sharing ONE MI355X (device-copy exchanges): the
top-digit rounds (msd, 24-bit wire at 4-bit digits) and the gap-coded rounds
(msdz, LIBSORT_DISTRIB_CODED), each step's wall time / R and the bytes each
rank sends (libsortDistribLastBytes).  The inputs of DESIGN.md section 7's
N = 2 / 4 / 8 model (tools/scale_model.py).

    python tools/coded_shape.py [R ...]          (default 2 4)
    CODED_PROFILE=R,sched python tools/coded_shape.py   (rocprofv3: 2 + 5 steps)
"""
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    torch.cuda.set_device(0)
    pylibsort.setDigitBits(4)
    lg = int(os.environ.get("CODED_LG", "29"))
    n = 1 << lg
    flags = {"msd": D.LIBSORT_DISTRIB_COPY, "msdz": D.LIBSORT_DISTRIB_COPY | D.LIBSORT_DISTRIB_CODED,
             "msd32": D.LIBSORT_DISTRIB_COPY | D.LIBSORT_DISTRIB_WIRE32}
    prof = os.environ.get("CODED_PROFILE")
    Rs = [int(prof.split(",")[0])] if prof else ([int(a) for a in sys.argv[1:]] or [2, 4])
    for R in Rs:
        shards = [D.populate_u32(n, first=r * n) for r in range(R)]
        torch.cuda.synchronize()
        if prof:
            f = flags[prof.split(",")[1]]
            for _ in range(7):
                D.distrib_sort_u32(shards, f)
            torch.cuda.synchronize()
            print({"profile": prof, "steps": 5, "warmup": 2})
            return
        res = {"R": R, "keys_per_rank": n}
        for name, f in flags.items():
            for _ in range(2):
                D.distrib_sort_u32(shards, f)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                D.distrib_sort_u32(shards, f)
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t0) / reps
            sent = D.distrib_last_bytes(R)
            res[name] = {"step_ms_all_ranks": round(ms, 3), "gpu_ms_per_rank": round(ms / R, 3),
                         "sent_bytes_per_rank": [int(b) for b in sent],
                         "bits_per_sent_key": round(8 * sum(sent) / ((R - 1) / R * n * R), 2)}
        print(json.dumps(res), flush=True)
        del shards
        pylibsort.lib().libsortReleaseWorkspace()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
