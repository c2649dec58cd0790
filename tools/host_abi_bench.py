#!/usr/bin/env python3
"""End-to-end timing of the host-pointer C ABI (providedGpu / gpuPartial on a
pageable host buffer: H2D + sort + D2H), i.e. what the reference's callers
see.  Not the bench `value` (which is device-resident)."""
import ctypes
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]

import numpy as np  # noqa: E402

import pylibsort  # noqa: E402

n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 28
pylibsort.require_gpu()
L = pylibsort.lib()
x = np.frombuffer(pylibsort.generateInputs(n), dtype=np.uint32)
for bits in (4, 8):
    pylibsort.setDigitBits(bits)
    for name, call in (("providedGpu", lambda b: L.providedGpu(b.ctypes.data, b.size)),
                       ("gpuPartial w8", lambda b: L.gpuPartial(b.ctypes.data, ctypes.addressof(bnd), b.size, 0, 8)),
                       ("gpuPartial w16", lambda b: L.gpuPartial(b.ctypes.data, ctypes.addressof(bnd16), b.size, 0, 16))):
        bnd = (ctypes.c_uint32 * 256)()
        bnd16 = (ctypes.c_uint32 * 65536)()
        ts = []
        for _ in range(4):
            b = x.copy()
            t0 = time.perf_counter()
            assert call(b) == 1, pylibsort.last_error()
            ts.append(time.perf_counter() - t0)
        t = min(ts[1:])
        print("%-15s digit%d n=2^%d: %.1f ms  %.2f Gkeys/s (host buffers, PCIe-inclusive)"
              % (name, bits, n.bit_length() - 1, t * 1e3, n / t / 1e9))
        if name == "providedGpu":
            assert np.array_equal(b, np.sort(x))
