"""pylibsort -- Python host side of the MI355X libsort.

Mirrors the reference binding faasTest/pylibsort (__init__.py:5-26, sort.py,
data.py:313-317): the same module-level functions (sortFull, sortPartial,
generateInputs, checkPartial, ...) over the same C ABI, loaded with ctypes.
On top of that it exposes the device-resident entry points for torch tensors
(pylibsort.device), the multi-GPU driver (pylibsort.distrib), the file
distributed arrays of data.py (pylibsort.data) and the FaaS worker of
faasTest/f.py (pylibsort.faas).

Library lookup order: $LIBSORT_PATH, the in-tree build
(gpu-radix-sort_amd/libsort.so), then the reference's own lookup,
ctypes.util._findLib_ld("sort") on LD_LIBRARY_PATH (__init__.py:13).

Like the reference, initLibSort() is called once at import.  On a machine
without a HIP device it fails; the GPU entry points then raise RuntimeError
instead of silently running anything else.
"""
import ctypes
import ctypes.util
import importlib.util
import os
import pathlib
import types

_HERE = pathlib.Path(__file__).resolve().parent
_INTREE = _HERE.parent / "libsort.so"

# (name, restype, argtypes)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_SIGS = [
    # Part 1 -- reference ABI (libsort/libsort.h:14-32)
    ("initLibSort", ctypes.c_int, []),
    ("gpuPartial", ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]),
    ("providedGpu", ctypes.c_int, [_vp, ctypes.c_size_t]),
    ("providedCpu", ctypes.c_int, [_vp, ctypes.c_size_t]),
    ("populateInput", None, [_vp, ctypes.c_size_t]),
    ("gpuPartialProfile", ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]),
    ("providedGpuProfile", ctypes.c_int, [_vp, ctypes.c_size_t]),
    # Part 2 -- additive
    ("gpuFullSort", ctypes.c_int, [_vp, ctypes.c_size_t]),
    ("gpuPartialSort", ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]),
    ("libsortSortKeysU32", ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortSortKeysRangeU32", ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, _vp]),
    ("libsortSortPiecesU32", ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_size_t, _u64p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
      _vp]),
    ("libsortSortPairsU64U32", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortSortKeysU64", ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortSortPairsU64U64", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortSortPairsU32U32", ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortHistogramU32", ctypes.c_int,
     [_vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionU32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, _u32p, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionLutU32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionLutU64U32", ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionLutCountU32", ctypes.c_int,
     [_vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionLutScatterU32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortPartitionLutCountU64U32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionLutScatterU64U32", ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortPartitionRangeCountU32", ctypes.c_int,
     [_vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionRangeScatterU32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ("libsortPartitionRangeCountU64U32", ctypes.c_int,
     [_vp, _vp, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, _vp, _vp]),
    ("libsortPartitionRangeScatterU64U32", ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, _vp]),
    ("libsortMinMaxU32", ctypes.c_int, [_vp, ctypes.c_size_t, _vp, _vp]),
    ("libsortMinMaxU64", ctypes.c_int, [_vp, ctypes.c_size_t, _vp, _vp]),
    ("libsortSortPiecesRangeU32", ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_size_t, _u64p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, _vp]),
    ("libsortSegmentCopyU32", ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _u64p, _u64p, _u64p, _vp]),
    ("libsortDeltaMaxGapU32", ctypes.c_int, [_vp, ctypes.c_size_t, _vp, _vp]),
    ("libsortDeltaPackU32", ctypes.c_int, [_vp, ctypes.c_size_t, _vp, _vp, _vp]),
    ("libsortDeltaUnpackU32", ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_uint32, _vp, _vp]),
    ("libsortMergeU32", ctypes.c_int, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, _vp]),
    ("gpuDistribSort", ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_int]),
    ("libsortDistribSortU32", ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32]),
    ("libsortDistribSortPairsU64U32", ctypes.c_int,
     [ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32]),
    ("libsortDistribLastBytes", ctypes.c_int, [ctypes.c_int, _u64p]),
    ("libsortSetDistribTrace", ctypes.c_int, [ctypes.c_int]),
    ("libsortDistribOverlapProbe", ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_uint32, _vp]),
    ("libsortDistribPlanDigits", ctypes.c_int,
     [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, _vp, _vp]),
    ("libsortDistribRangeDigit", ctypes.c_int,
     [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, _u64p, _u32p]),
    ("libsortPopulateDevice", ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_uint64, _vp]),
    ("libsortSetDigitBits", ctypes.c_int, [ctypes.c_int]),
    ("libsortGetDigitBits", ctypes.c_int, []),
    ("libsortSetAlgorithm", ctypes.c_int, [ctypes.c_int]),
    ("libsortSetHybrid", ctypes.c_int, [ctypes.c_int]),
    ("libsortSetBucketMode", ctypes.c_int, [ctypes.c_int]),
    ("libsortSetBoundaryMode", ctypes.c_int, [ctypes.c_int]),
    ("libsortTimingEnable", None, [ctypes.c_bool]),
    ("libsortTimingReset", None, []),
    ("libsortTimingFilter", None, [ctypes.c_char_p]),
    ("libsortTimingSample", None, [ctypes.c_uint32]),
    ("libsortTimingQuery", ctypes.c_int,
     [ctypes.c_char_p, _u64p, ctypes.POINTER(ctypes.c_double), _u64p]),
    ("libsortReleaseWorkspace", ctypes.c_int, []),
    ("libsortLastError", ctypes.c_char_p, []),
    ("libsortDeviceErrors", ctypes.c_uint32, []),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]


def library_path():
    """Path of the libsort.so this package binds to (None if not found)."""
    env = os.environ.get("LIBSORT_PATH")
    if env:
        return env
    if _INTREE.exists():
        return str(_INTREE)
    return ctypes.util._findLib_ld("sort")


def _preload_torch_hip():
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so, soname
    libamdhip64.so.7).  If libsort.so were loaded first it would bring in
    /opt/rocm's copy, torch would later load its own, and with two HIP
    runtimes in the process torch sees no GPU ("No HIP GPUs are available").
    Loading torch's copy first (global, without importing torch) makes
    libsort.so bind to it: one runtime, whichever of torch and pylibsort is
    imported first.  Without torch installed this does nothing;
    LIBSORT_HIP_RUNTIME=system keeps the image's runtime (a process that never
    imports torch, e.g. the reference's FaaS worker flow)."""
    if os.environ.get("LIBSORT_HIP_RUNTIME", "torch") == "system":
        return
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.origin:
        return
    hip = pathlib.Path(spec.origin).parent / "lib" / "libamdhip64.so"
    if hip.exists():
        ctypes.CDLL(str(hip), mode=ctypes.RTLD_GLOBAL)


def _setup():
    s = types.SimpleNamespace()
    _preload_torch_hip()
    path = library_path()
    if path is None:
        raise RuntimeError("libsort could not be located: build it (python __graft_entry__.py build) "
                           "or put libsort.so on LD_LIBRARY_PATH / $LIBSORT_PATH")
    s.path = path
    s.sortLib = ctypes.cdll.LoadLibrary(path)
    # (LIBSORT_AB_MISSING_OK=1: an older build in an A/B run may lack newer
    # entry points; they then stay unbound)
    missing_ok = os.environ.get("LIBSORT_AB_MISSING_OK") == "1"
    for name, res, args in _SIGS:
        fn = getattr(s.sortLib, name, None)
        if fn is None:
            if missing_ok:
                continue
            raise AttributeError("%s lacks %s" % (path, name))
        fn.restype = res
        fn.argtypes = args
    # Must be called exactly once per process (reference __init__.py:19-20).
    s.gpu_ready = bool(s.sortLib.initLibSort())
    return s


_state = _setup()


def lib():
    """The loaded ctypes library."""
    return _state.sortLib


def gpu_ready():
    """True when initLibSort() found at least one HIP device."""
    return _state.gpu_ready


def last_error():
    msg = _state.sortLib.libsortLastError()
    return msg.decode() if msg else ""


def require_gpu():
    if not _state.gpu_ready:
        raise RuntimeError("libsort: no HIP device (initLibSort failed: %s)" % last_error())


from .data import *  # noqa: E402,F401,F403
from .sort import *  # noqa: E402,F401,F403
