"""ctypes front end of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker (never as the thing measured or shipped).  See
oracle.cpp for the reference file:line each function restates.
"""
import ctypes
import pathlib
import subprocess

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
_LIB = _HERE / "liboracle.so"
_lib = None

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.run(["make", "-C", str(_HERE), "liboracle.so"], check=True,
                   stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not _LIB.exists():
            build()
        L = ctypes.CDLL(str(_LIB))
        L.oracle_pcg_fill.argtypes = [_u32p, ctypes.c_size_t, _u64p]
        L.oracle_pcg_initial_state.restype = ctypes.c_uint64
        L.oracle_sort_u32.argtypes = [_u32p, ctypes.c_size_t]
        L.oracle_partial_u32.argtypes = [_u32p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_ref_step_u32.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_ref_boundaries.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _u32p]
        L.oracle_distrib_local_u32.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_uint32]
        L.oracle_distrib_bsp_u32.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _u64p]
        L.oracle_stable_sort_kv64.argtypes = [_u64p, _u32p, ctypes.c_size_t]
        L.oracle_stable_sort_kv32.argtypes = [_u32p, _u32p, ctypes.c_size_t]
        L.oracle_sort_u64.argtypes = [_u64p, ctypes.c_size_t]
        L.oracle_stable_sort_kv64v64.argtypes = [_u64p, _u64p, ctypes.c_size_t]
        L.oracle_pcg_value_counts.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        L.oracle_pcg_value_counts.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _p32(a):
    return a.ctypes.data_as(_u32p)


def _p64(a):
    return a.ctypes.data_as(_u64p)


class Pcg:
    """The reference populateInput stream with its process-wide state
    (utils.cu:65-80); a fresh instance = a fresh process."""

    def __init__(self, skip=0):
        self.state = ctypes.c_uint64(lib().oracle_pcg_initial_state())
        if skip:
            self.take(skip)

    def take(self, n):
        out = np.empty(n, dtype=np.uint32)
        lib().oracle_pcg_fill(_p32(out), n, ctypes.byref(self.state))
        return out


def pcg(n, first=0):
    """Elements [first, first+n) of a fresh-process populateInput stream."""
    g = Pcg()
    if first:
        # advance in bounded chunks
        left = first
        while left:
            k = min(left, 1 << 24)
            g.take(k)
            left -= k
    return g.take(n)


def sort_u32(a):
    b = np.array(a, dtype=np.uint32, copy=True)
    lib().oracle_sort_u32(_p32(b), b.size)
    return b


def partial_u32(a, offset, width):
    """(data, boundaries) of the gpuPartial contract."""
    b = np.array(a, dtype=np.uint32, copy=True)
    bounds = np.zeros(1 << width, dtype=np.uint32)
    lib().oracle_partial_u32(_p32(b), _p32(bounds), b.size, offset, width)
    return b, bounds


def ref_step_u32(a, offset, width):
    """Exact emulation of the reference SortState::Step kernels."""
    b = np.array(a, dtype=np.uint32, copy=True)
    lib().oracle_ref_step_u32(_p32(b), b.size, offset, width)
    return b


def ref_boundaries(sorted_a, offset, width):
    """The reference GetBoundaries output, quirk included."""
    s = np.ascontiguousarray(sorted_a, dtype=np.uint32)
    b = np.zeros(1 << width, dtype=np.uint32)
    lib().oracle_ref_boundaries(_p32(s), s.size, offset, width, _p32(b))
    return b


def distrib_local_u32(a, width=8):
    b = np.array(a, dtype=np.uint32, copy=True)
    lib().oracle_distrib_local_u32(_p32(b), b.size, width)
    return b


def distrib_bsp_u32(a, nworker, width=8):
    """(concatenated result, per-worker final lengths) of SortDistribFromArr."""
    b = np.array(a, dtype=np.uint32, copy=True)
    lens = np.zeros(nworker, dtype=np.uint64)
    lib().oracle_distrib_bsp_u32(_p32(b), b.size, nworker, width, _p64(lens))
    return b, lens


def stable_sort_kv64(k, v):
    kk = np.array(k, dtype=np.uint64, copy=True)
    vv = np.array(v, dtype=np.uint32, copy=True)
    lib().oracle_stable_sort_kv64(_p64(kk), _p32(vv), kk.size)
    return kk, vv


def stable_sort_kv32(k, v):
    kk = np.array(k, dtype=np.uint32, copy=True)
    vv = np.array(v, dtype=np.uint32, copy=True)
    lib().oracle_stable_sort_kv32(_p32(kk), _p32(vv), kk.size)
    return kk, vv


def sort_u64(k):
    kk = np.array(k, dtype=np.uint64, copy=True)
    lib().oracle_sort_u64(_p64(kk), kk.size)
    return kk


def stable_sort_kv64v64(k, v):
    kk = np.array(k, dtype=np.uint64, copy=True)
    vv = np.array(v, dtype=np.uint64, copy=True)
    lib().oracle_stable_sort_kv64v64(_p64(kk), _p64(vv), kk.size)
    return kk, vv


def sorted_pcg_sha256(n, first=0, chunk_values=1 << 24, shift=0):
    """sha256 (hex) of std::sort of elements [first, first+n) of the
    populateInput stream, little-endian uint32, without sorting: a one-byte
    count per value (4 GiB), expanded in value order chunk by chunk.
    shift > 0: of the keys x >> shift instead (a monotone map, so the sorted
    stream is the sorted one shifted)."""
    import hashlib
    counts = np.zeros(1 << 32, dtype=np.uint8)
    mx = lib().oracle_pcg_value_counts(counts.ctypes.data, n, first)
    if mx >= 255:
        raise RuntimeError("a value occurs 255+ times: one-byte counts saturate")
    h = hashlib.sha256()
    total = 0
    for a in range(0, 1 << 32, chunk_values):
        c = counts[a:a + chunk_values]
        nz = np.nonzero(c)[0]
        if nz.size:
            vals = np.repeat(((nz + a) >> shift).astype(np.uint32), c[nz])
            total += vals.size
            h.update(vals.astype("<u4").tobytes())
    assert total == n
    return h.hexdigest()
