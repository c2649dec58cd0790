#!/usr/bin/env python3
"""configs[4]'s per-GPU pair sort (2^28 (u64, u32) pairs, 8-bit digits) with
its six buffers either as torch tensors (the bench's allocation) or carved
out of ONE hipMalloc slab at 2 MiB-aligned offsets -- the test of round 5's
hypothesis that the pair pass's box-to-box swing is the driver's page
fragmentation of the depth-0 output (depth 0 misses
UTCL1 ~1.28e6 times per dispatch against 2.4e3 at depth 1).

    python tools/pair_slab_ab.py torch|slab [reps]
Run under rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS for the TLB side."""
import ctypes
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
    mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    torch.cuda.set_device(0)
    pylibsort.setDigitBits(8)
    n = 1 << 28
    w = D.populate_u32(2 * n).view(n, 2).to(torch.int64)
    keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
    del w
    vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32)
    torch.cuda.synchronize()
    L = pylibsort.lib()
    stream = torch.cuda.current_stream().cuda_stream
    if mode == "torch":
        ok_, ov = torch.empty_like(keys), torch.empty_like(vals)
        tk, tv = torch.empty_like(keys), torch.empty_like(vals)
        ptrs = [keys.data_ptr(), vals.data_ptr(), ok_.data_ptr(), ov.data_ptr(), tk.data_ptr(), tv.data_ptr()]
        hold = (ok_, ov, tk, tv)
    else:
        hip = ctypes.CDLL("libamdhip64.so")
        align = 2 << 20
        sizes = [8 * n, 4 * n, 8 * n, 4 * n, 8 * n, 4 * n]
        offs, at = [], 0
        for sz in sizes:
            offs.append(at)
            at += (sz + align - 1) // align * align
        base = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(base), ctypes.c_size_t(at + align)) == 0
        b0 = (base.value + align - 1) // align * align
        ptrs = [b0 + o for o in offs]
        hip.hipMemcpy(ctypes.c_void_p(ptrs[0]), ctypes.c_void_p(keys.data_ptr()), ctypes.c_size_t(8 * n), 3)
        hip.hipMemcpy(ctypes.c_void_p(ptrs[1]), ctypes.c_void_p(vals.data_ptr()), ctypes.c_size_t(4 * n), 3)
        hold = base
    args = [ctypes.c_void_p(p) for p in ptrs] + [ctypes.c_size_t(n), ctypes.c_uint32(0), ctypes.c_uint32(64),
                                                  ctypes.c_void_p(stream)]

    def step():
        if L.libsortSortPairsU64U32(*args) != 1:
            raise RuntimeError(pylibsort.last_error())
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    D.timing_reset()
    D.timing_filter("tilepass")
    D.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / reps
    D.timing_enable(False)
    launches, tms, _ = D.timing_query("tilepass")
    print(json.dumps({"mode": mode, "ms_per_sort": round(ms, 4), "pass_launches": launches,
                      "pass_avg_us": round(1e3 * tms / max(launches, 1), 2),
                      "buffers_2MiB_aligned": mode == "slab",
                      "addresses": [hex(p) for p in ptrs]}), flush=True)
    del hold


if __name__ == "__main__":
    main()
