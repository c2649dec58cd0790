#!/usr/bin/env python3
"""Times the range sorts of the msd schedule's rounds at 8 GPUs (2^29 keys
per rank, K = 4 rounds growing x1.2: ~100M / 120M / 144M / 173M keys, each
spanning its share of the rank's 2^29 key values) on one MI355X.  Run with
LIBSORT_HYBRID=0 / LIBSORT_HYB_MIN_LOG2=... for A/B.  python tools/round_sorts.py"""
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
    w = [1.2 ** i for i in range(4)]
    fr = [x / sum(w) for x in w]
    total = 0.0
    for f in fr:
        n = int(f * (1 << 29))
        span = int(f * (1 << 29))
        lo = 0x20000000
        x = D.populate_u32(n, first=7)
        y = (((x.to(torch.int64) & 0xFFFFFFFF) * span >> 32) + lo).to(torch.int32)  # < 2^31
        out = torch.empty_like(y)
        tmp = torch.empty_like(y)
        fn = lambda: D.sort_keys_range_u32(y, lo, lo + span, out=out, tmp=tmp)
        fn()
        torch.cuda.synchronize()
        D.timing_enable(True)
        D.timing_reset()
        fn()
        torch.cuda.synchronize()
        nbs, npass = D.timing_query("bucketsort")[0], D.timing_query("tilepass")[0]
        D.timing_enable(False)
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        total += ms
        print("n %d span 2^%.2f: %.3f ms (bucket sorts %d, passes %d)" % (n, float(torch.tensor(span).log2()), ms, nbs, npass))
    print("rounds total %.3f ms" % total)


if __name__ == "__main__":
    main()
