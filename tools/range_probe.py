#!/usr/bin/env python3
"""Kernel-level comparison of the full sort and the range-restricted sort
(the round sorts of the msd schedule) at 2^28 keys: run under
rocprofv3 --kernel-trace.  python tools/range_probe.py"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    pylibsort.setDigitBits(4)
    n = 1 << 28
    keys = D.populate_u32(n)
    lo = 1 << 28
    narrow = ((keys >> 5) & ((1 << 27) - 1)) + lo
    out = torch.empty_like(keys)
    tmp = torch.empty_like(keys)
    for name, fn in (("full", lambda: D.sort_keys_u32(keys, out=out, tmp=tmp)),
                     ("range27", lambda: D.sort_keys_range_u32(narrow, lo, lo + (1 << 27), out=out, tmp=tmp)),
                     ("full_narrow", lambda: D.sort_keys_u32(narrow, out=out, tmp=tmp))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        print(name, "%.3f ms" % ((time.perf_counter() - t0) / 5 * 1e3))


if __name__ == "__main__":
    main()
