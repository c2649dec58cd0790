#!/usr/bin/env python3
"""Does a working set that fits the 256 MiB Infinity Cache sort faster per key?

1. size sweep: device-resident full sort at 2^20..2^28 keys (4- and 8-bit
   digits), microseconds per key-pass;
2. MSD emulation at 2^28 keys: one stable partition by the top B bits
   (libsortPartitionLutU32), then each bucket sorted on its own by the
   range-restricted sort (digits of key - lo), bucket after bucket, so every
   bucket's passes run on a 2^(28-B)-key working set.

python tools/mall_probe.py   (one GPU)"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def timeit(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    for bits in (4, 8):
        pylibsort.setDigitBits(bits)
        passes = 32 // bits
        for lg in range(20, 29):
            n = 1 << lg
            keys = D.populate_u32(n)
            out = torch.empty_like(keys)
            tmp = torch.empty_like(keys)
            t = timeit(lambda: D.sort_keys_u32(keys, out=out, tmp=tmp))
            print("sweep bits=%d n=2^%d sort %.3f ms  %.3f ns/key-pass  %.1f Gkeys/s" %
                  (bits, lg, t * 1e3, t * 1e9 / n / passes, n / t / 1e9), flush=True)
    n = 1 << 28
    keys = D.populate_u32(n)
    ref = D.sort_keys_u32(keys)
    for bits in (4, 8):
        pylibsort.setDigitBits(bits)
        for B in (2, 3, 4, 5, 6):
            nb = 1 << B
            lut_shift = 20
            lut = (torch.arange(1 << 12, device="cuda", dtype=torch.int32) >> (12 - B)).to(torch.uint8)
            part = torch.empty_like(keys)
            out = torch.empty_like(keys)
            tmp = torch.empty_like(keys)
            _, bounds = D.partition_lut_u32(keys, lut, lut_shift, nb, out=part)
            b = bounds.cpu().tolist() + [n]
            span = 1 << (32 - B)

            def run():
                D.partition_lut_u32(keys, lut, lut_shift, nb, out=part, bounds=bounds)
                for i in range(nb):
                    a, e = b[i], b[i + 1]
                    if e > a:
                        D.sort_keys_range_u32(part[a:e], i * span, (i + 1) * span, out=out[a:e], tmp=tmp[a:e])

            def part_only():
                D.partition_lut_u32(keys, lut, lut_shift, nb, out=part, bounds=bounds)
            t = timeit(run, reps=5)
            tp = timeit(part_only, reps=5)
            ok = torch.equal(out, ref)
            print("msd bits=%d B=%d buckets=%d: %.3f ms total (partition %.3f ms) %.1f Gkeys/s %s" %
                  (bits, B, nb, t * 1e3, tp * 1e3, n / t / 1e9, "ok" if ok else "MISMATCH"), flush=True)


if __name__ == "__main__":
    main()
