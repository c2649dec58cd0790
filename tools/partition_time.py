#!/usr/bin/env python3
"""Times the stable 256-bucket partition of the multi-GPU engine (count +
scatter; libsortPartitionLut*), (u64, u32) pairs and u32 keys, 2^28 each,
identity table on the top byte, and checks the pairs' output against a
stable argsort of the digits.  LIBSORT_PATH selects the library (A/B).
    python3 tools/partition_time.py [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "gpu-radix-sort_amd")]
import pylibsort.device as D  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = 1 << 28
g = torch.Generator(device="cuda").manual_seed(5)
k = torch.randint(-(1 << 62), 1 << 62, (n,), device="cuda", dtype=torch.int64, generator=g)
v = torch.arange(n, device="cuda", dtype=torch.int64).to(torch.int32)
lut = torch.arange(256, device="cuda", dtype=torch.int32).to(torch.uint8)
ok_, ov = torch.empty_like(k), torch.empty_like(v)
u = torch.randint(-(1 << 31), 1 << 31, (n,), device="cuda", dtype=torch.int64, generator=g).to(torch.int32)
uo = torch.empty_like(u)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * sorted(ts)[len(ts) // 2]


tp = timed(lambda: D.partition_lut_pairs_u64_u32(k, v, lut, 24, 256, out_keys=ok_, out_vals=ov))
tk = timed(lambda: D.partition_lut_u32(u, lut, 24, 256, out=uo))
# check: the pairs stably partitioned by the top byte of the key's high word
kk = k.cpu().numpy().view(np.uint64)
dig = (kk >> np.uint64(56)).astype(np.int64)
order = np.argsort(dig, kind="stable")
good = np.array_equal(ok_.cpu().numpy().view(np.uint64), kk[order]) and \
    np.array_equal(ov.cpu().numpy().view(np.uint32), order.astype(np.uint32))
print("pairs 2^28: %.3f ms (%s)   u32 keys 2^28: %.3f ms   lib %s" % (
    tp, "exact" if good else "WRONG", tk, os.environ.get("LIBSORT_PATH", "in-tree")))
