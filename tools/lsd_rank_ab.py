#!/usr/bin/env python3
"""Timing only (no check): gpuPartial's device-resident call at the
reference's workload (2^28 keys, width 8 / 16, 8-bit digits) and the 8-pass
LSD full sort, 10 reps each, with per-kernel pass timing -- for A/B builds
(LIBSORT_PATH) whose LSD rank differs.  python tools/lsd_rank_ab.py"""
import json
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
    pylibsort.setDigitBits(8)
    n = 1 << 28
    keys = D.populate_u32(n)
    out, tmp = torch.empty_like(keys), torch.empty_like(keys)
    res = {"lib": pylibsort._state.path.split("/")[-1]}
    for w in (8, 16, 32):
        b = torch.empty(1 << w, dtype=torch.int32, device="cuda") if w < 32 else None
        prev = pylibsort.setHybrid("off") if w == 32 else None

        def step():
            D.sort_keys_u32(keys, out=out, tmp=tmp, offset=0, width=w, boundaries=b)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        D.timing_reset()
        D.timing_filter("tilepass")
        D.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / 10
        D.timing_enable(False)
        l, tms, _ = D.timing_query("tilepass")
        res["w%d" % w] = {"ms": round(ms, 4), "pass_us": round(1e3 * tms / max(l, 1), 1)}
        if prev is not None:
            pylibsort.setHybrid(prev)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
