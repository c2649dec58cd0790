#!/usr/bin/env python3
"""GPU work of the C engine's one- vs two-part partition: R ranks sharing
the one GPU (device-copy exchanges, so nothing overlaps and the time is the
sum of the work), keys and pairs, median of reps.  Run once per
LIBSORT_DISTRIB_PARTS value (read once per process).
    LIBSORT_DISTRIB_PARTS=1 python3 tools/parts_ab.py [R] [log2 keys per rank]"""
import os
import sys
import time

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "gpu-radix-sort_amd")]
import pylibsort.device as D  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 26
n = 1 << lg
sh = [D.populate_u32(n, first=r * n) for r in range(R)]
ks = [((D.populate_u32(n, first=(R + r) * n).to(torch.int64) << 32) | (s.to(torch.int64) & 0xFFFFFFFF)) for r, s in
      enumerate(sh)]
vs = [torch.arange(r * n, (r + 1) * n, device="cuda", dtype=torch.int64).to(torch.int32) for r in range(R)]
COPY = getattr(D, "LIBSORT_DISTRIB_COPY", 2)


def med(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * sorted(ts)[len(ts) // 2]


tk = med(lambda: D.distrib_sort_u32(sh, COPY))
tp = med(lambda: D.distrib_sort_pairs_u64_u32(ks, vs, COPY))
print("parts=%s R=%d 2^%d per rank: keys %.3f ms, pairs %.3f ms" % (os.environ.get("LIBSORT_DISTRIB_PARTS", "2"), R,
                                                                    lg, tk, tp))
