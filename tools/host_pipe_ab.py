#!/usr/bin/env python3
"""providedGpu on a pageable host buffer of 2^28 keys (PCIe-inclusive), min
of 4 calls: for A/B of the pipelined host sort's knobs (LIBSORT_PIPE_CHUNKS,
LIBSORT_PIPE_GROUPS, LIBSORT_HOST_PIPELINE_MIN=0 for the unpipelined path)."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]
import numpy as np  # noqa: E402

import pylibsort  # noqa: E402

n = 1 << 28
pylibsort.require_gpu()
L = pylibsort.lib()
x = np.frombuffer(pylibsort.generateInputs(n), dtype=np.uint32)
ts = []
for _ in range(5):
    b = x.copy()
    t0 = time.perf_counter()
    assert L.providedGpu(b.ctypes.data, b.size) == 1, pylibsort.last_error()
    ts.append(time.perf_counter() - t0)
assert np.array_equal(b, np.sort(x))
print("%s providedGpu 2^28: %.2f ms" % (" ".join(sys.argv[1:]), 1e3 * min(ts[1:])))
