#!/usr/bin/env python3
"""Times the single-GPU pieces of the multi-GPU "msd" schedule at 2^28 keys:
the sampled top-bit histogram, the table partition (16 / 32 / 64 buckets),
and the local sort done as K round-sized sorts (K = 1, 2, 4, 8), so the
critical path of an R-GPU run can be estimated next to the exchange time.

    python tools/msd_parts.py [--keys-log2 28] [--digit-bits 4]
"""
import argparse
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def timed(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys-log2", type=int, default=28)
    ap.add_argument("--digit-bits", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    import pylibsort
    import pylibsort.device as D
    from pylibsort import distrib
    pylibsort.setDigitBits(a.digit_bits)
    n = 1 << a.keys_log2
    keys = D.populate_u32(n)
    ops = distrib.HipOps()
    res = {}
    res["sample_hist_ms"] = timed(lambda: ops.histogram(ops.sample(keys, 16), 20, 12))
    res["full_hist_ms"] = timed(lambda: ops.histogram(keys, 20, 12))
    out = torch.empty_like(keys)
    for nb in (16, 32, 64):
        H = np.ones((1, 4096))
        lut, _ = distrib.plan_rounds(H, nb, 1)
        t = torch.from_numpy(lut).cuda()
        b = torch.empty(nb, dtype=torch.int32, device="cuda")
        res["partition_%d_ms" % nb] = timed(lambda: D.partition_lut_u32(keys, t, 20, nb, out=out, bounds=b))
    tmp = torch.empty_like(keys)
    for K in (1, 2, 4, 8):
        m = n // K

        def rounds():
            for i in range(K):
                D.sort_keys_u32(keys[i * m:(i + 1) * m], out=out[i * m:(i + 1) * m], tmp=tmp[:m])
        res["sort_%d_rounds_ms" % K] = timed(rounds, reps=5)
    lo = 1 << 28                             # a round's range at R*K = 32: [lo, lo + 2^27)
    narrow = ((keys >> 5) & ((1 << 27) - 1)) + lo
    for K in (1, 4, 8):
        m = n // K

        def rounds_range():
            for i in range(K):
                D.sort_keys_range_u32(narrow[i * m:(i + 1) * m], lo, lo + (1 << 27), out=out[i * m:(i + 1) * m],
                                      tmp=tmp[:m])
        res["range27_sort_%d_rounds_ms" % K] = timed(rounds_range, reps=5)
    for K in (4, 6, 8, 12):                  # K equal rounds of a rank's 2^29-wide range (R = 8)
        m = n // K
        span = (1 << 29) // K
        narrowK = (keys % span) + lo

        def rounds_k():
            for i in range(K):
                D.sort_keys_range_u32(narrowK[i * m:(i + 1) * m], lo, lo + span, out=out[i * m:(i + 1) * m],
                                      tmp=tmp[:m])
        res["r8_equal_%d_rounds_ms" % K] = timed(rounds_k, reps=5)
    print({k: round(v, 3) for k, v in res.items()})


if __name__ == "__main__":
    main()
