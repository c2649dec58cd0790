#!/usr/bin/env python3
"""LSD vs MSD hybrid (forced) across sizes, one MI355X: u32 keys (4/8-bit),
(u64, u32) pairs and u64 keys (8-bit).  python tools/hyb_sizes.py [lg ...]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def timed(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    lgs = [int(a) for a in sys.argv[1:]] or [23, 24, 25, 26, 27]
    for lg in lgs:
        n = 1 << lg
        k32 = D.populate_u32(n)
        o32, t32 = torch.empty_like(k32), torch.empty_like(k32)
        w = D.populate_u32(2 * n, first=7).to(torch.int64) & 0xFFFFFFFF
        k64 = (w[0::2] << 32) | w[1::2]
        del w
        v32 = torch.arange(n, dtype=torch.int32, device="cuda")
        o64, t64, ov, tv = torch.empty_like(k64), torch.empty_like(k64), torch.empty_like(v32), torch.empty_like(v32)
        cases = [
            ("u32 keys 4-bit", 4, lambda: D.sort_keys_u32(k32, out=o32, tmp=t32)),
            ("u32 keys 8-bit", 8, lambda: D.sort_keys_u32(k32, out=o32, tmp=t32)),
            ("u64+u32 pairs 8-bit", 8, lambda: D.sort_pairs_u64_u32(k64, v32, out_keys=o64, out_vals=ov,
                                                                     tmp_keys=t64, tmp_vals=tv)),
            ("u64 keys 8-bit", 8, lambda: D.sort_keys_u64(k64, out=o64, tmp=t64)),
        ]
        for name, bits, fn in cases:
            pylibsort.setDigitBits(bits)
            r = {}
            for mode in ("off", "force"):
                prev = pylibsort.setHybrid(mode)
                r[mode] = timed(fn)
                pylibsort.setHybrid(prev)
            print("2^%d %-20s lsd %7.3f ms  hybrid %7.3f ms  (%.2fx)" % (lg, name, r["off"], r["force"],
                                                                     r["off"] / r["force"]), flush=True)
        del k32, o32, t32, k64, o64, t64, ov, tv, v32


if __name__ == "__main__":
    main()
