"""Host-buffer sort API, mirroring faasTest/pylibsort/sort.py:94-126 and
data.py:313-317 (same names, argument meaning and errors), plus the result
checkers of sort.py:36-89 (checkPartial restated so that it checks against
the boundaries themselves; the reference's variant is broken).
"""
import ctypes

import numpy as np

from . import _state, require_gpu

__all__ = [
    "sortException", "sortResultException", "groupBits", "bytesToInts", "checkOrder",
    "checkSortFull", "checkPartial", "sortFull", "sortFullDistrib", "sortPartial", "generateInputs",
    "boundariesToCaps", "setDigitBits", "getDigitBits", "setAlgorithm", "setHybrid",
]


class sortException(Exception):
    def __init__(self, msg):
        self.msg = msg

    def __str__(self):
        return "Sort error: {}".format(self.msg)


class sortResultException(Exception):
    def __init__(self, idx, expect, got, msg=None):
        self.idx = idx
        self.expect = expect
        self.got = got
        self.msg = msg

    def __str__(self):
        desc = "Sorted Incorrectly at index {}, Expected {:#08x}, Got {:#08x}".format(
            self.idx, self.expect, self.got)
        if self.msg is not None:
            desc += " ({})".format(self.msg)
        return desc


def groupBits(v, pos, width):
    """Group id of v for `width` bits starting at `pos` (sort.py:36-37)."""
    return (v >> pos) & ((1 << width) - 1)


def bytesToInts(barr):
    """View a bytes-like object as little-endian uint32 (sort.py:40-41)."""
    return np.frombuffer(barr, dtype=np.uint32)


def checkOrder(arr):
    """Raise sortResultException unless arr is non-decreasing."""
    a = np.asarray(arr)
    if a.size < 2:
        return
    bad = np.nonzero(a[1:] < a[:-1])[0]
    if bad.size:
        i = int(bad[0]) + 1
        raise sortResultException(i, int(a[i - 1]), int(a[i]), "value should be >= to expected")


def checkSortFull(new, orig):
    """Raise unless `new` equals sorted(orig)."""
    ref = np.sort(np.asarray(orig, dtype=np.uint32), kind="stable")
    got = np.asarray(new, dtype=np.uint32)
    bad = np.nonzero(ref != got)[0]
    if bad.size:
        i = int(bad[0])
        raise sortResultException(i, int(ref[i]), int(got[i]))


def checkPartial(refBytes, testBytes, boundaries, pos, width):
    """Check a partial sort: every element of group g lies in
    [boundaries[g], boundaries[g+1]) and the multiset is unchanged.
    (Reference sort.py:67-89 takes byte `caps` and ignores `pos`.)"""
    ref = bytesToInts(refBytes)
    test = bytesToInts(testBytes)
    b = np.asarray(boundaries, dtype=np.int64)
    if len(ref) != len(test):
        raise sortException("test length doesnt match reference: expected {}, got {}".format(
            len(ref), len(test)))
    if len(b) != (1 << width):
        raise sortException("Not enough output buckets: expected {}, got {}".format(
            1 << width, len(b)))
    sizes = np.diff(np.append(b, len(test)))
    if np.any(sizes < 0):
        raise sortException("boundaries are not monotone")
    expect = np.repeat(np.arange(len(b), dtype=np.uint64), sizes)
    got = (test.astype(np.uint64) >> np.uint64(pos)) & np.uint64((1 << width) - 1)
    if not np.array_equal(expect, got):
        raise sortException("Output does not have expected groups")
    if not np.array_equal(np.sort(ref), np.sort(test)):
        raise sortException("Test does not contain same elements as ref")


def boundariesToCaps(boundaries, nbytes):
    """Bucket capacities in bytes from element boundaries, as the FaaS worker
    derives them (data.py:301-304: caps = diff(b*4, append=len))."""
    caps = np.array(boundaries, dtype=np.int64) * 4
    return np.diff(caps, append=nbytes)


def sortFull(buf: bytearray):
    """Interpret buf as an array of C uint32s and sort it in place (sort.py:94-105)."""
    require_gpu()
    nElem = int(len(buf) / 4)
    if nElem == 0:
        return
    cRaw = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    res = _state.sortLib.providedGpu(ctypes.addressof(cRaw), ctypes.c_size_t(nElem))
    if not res:
        raise RuntimeError("Libsort had an internal error")


def sortFullDistrib(buf: bytearray, ngpu=0):
    """Sort buf (C uint32s) in place across ngpu GPUs of the device pool
    (gpuDistribSort; ngpu <= 0: all of them)."""
    require_gpu()
    nElem = int(len(buf) / 4)
    if nElem == 0:
        return
    cRaw = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    if not _state.sortLib.gpuDistribSort(ctypes.addressof(cRaw), ctypes.c_size_t(nElem), ctypes.c_int(ngpu)):
        raise RuntimeError("Libsort had an internal error")


def sortPartial(buf: bytearray, offset, width):
    """Partial sort of buf in place (width bits starting at bit offset); returns
    the list of int boundaries between radix groups (sort.py:108-126)."""
    require_gpu()
    nElem = int(len(buf) / 4)
    boundaries = (ctypes.c_uint32 * (1 << width))()
    if nElem == 0:
        return list(boundaries)
    cRaw = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    res = _state.sortLib.gpuPartial(ctypes.addressof(cRaw), ctypes.addressof(boundaries),
                                    ctypes.c_size_t(nElem), ctypes.c_uint32(offset),
                                    ctypes.c_uint32(width))
    if not res:
        raise RuntimeError("Libsort had an internal error")
    return list(boundaries)


def generateInputs(n):
    """n PCG32 integers from the process-wide populateInput stream (data.py:313-317)."""
    b = bytearray(n * 4)
    if n:
        cInts = (ctypes.c_uint32 * n).from_buffer(b)
        _state.sortLib.populateInput(ctypes.addressof(cInts), n)
    return b


def setDigitBits(bits):
    prev = _state.sortLib.libsortSetDigitBits(int(bits))
    if prev < 0:
        raise ValueError("unsupported digit width %r (4 or 8)" % bits)
    return prev


def getDigitBits():
    return _state.sortLib.libsortGetDigitBits()


_ALGOS = {"auto": 0, "onesweep": 1, "rts": 2, "tiles": 3}
_HYBRID = {"off": 0, "auto": 1, "force": 2}


def setHybrid(name):
    """MSD hybrid for full 32-bit key sorts: "auto" (default), "off" or
    "force" (every full sort of >= 1024 keys); returns the previous name."""
    prev = _state.sortLib.libsortSetHybrid(_HYBRID[name])
    if prev < 0:
        raise ValueError(name)
    return {v: k for k, v in _HYBRID.items()}[prev]


def setAlgorithm(name):
    """Select the pass algorithm ("auto", "onesweep", "rts" or "tiles"); returns the previous name."""
    prev = _state.sortLib.libsortSetAlgorithm(_ALGOS[name])
    if prev < 0:
        raise ValueError(name)
    return {v: k for k, v in _ALGOS.items()}[prev]
