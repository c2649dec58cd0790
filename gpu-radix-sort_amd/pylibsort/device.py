"""Device-resident entry points of libsort on torch tensors.

torch is plumbing here: it owns the HBM buffers and the current HIP stream;
every computation runs in libsort.so's HIP kernels (there is no torch or CPU
fallback -- a missing GPU or library raises).

uint32 keys travel in int32 tensors and uint64 keys in int64 tensors (same
bits); torch's uint32/uint64 dtypes are accepted too.
"""
import ctypes

import numpy as np
import torch

from . import _state, last_error

_U32 = (torch.int32, torch.uint32)
_U64 = (torch.int64, torch.uint64)


def _lib():
    return _state.sortLib


def _check(ok, what):
    if not ok:
        raise RuntimeError("%s failed: %s" % (what, last_error()))


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need(t, dtypes, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("%s must be a CUDA (HIP) tensor" % name)
    if t.dtype not in dtypes:
        raise TypeError("%s has dtype %s, expected one of %s" % (name, t.dtype, dtypes))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)


def sort_keys_u32(keys, out=None, tmp=None, offset=0, width=None, boundaries=None):
    """Stable LSD sort of bits [offset, offset+width) of uint32 keys (int32
    carrier).  Returns `out`.  `boundaries` (optional int32 tensor of 2**width)
    receives the gpuPartial group boundaries."""
    _need(keys, _U32, "keys")
    n = keys.numel()
    if width is None:
        width = 32 - offset
    out = torch.empty_like(keys) if out is None else out
    tmp = torch.empty_like(keys) if tmp is None else tmp
    _need(out, _U32, "out")
    _need(tmp, _U32, "tmp")
    if boundaries is not None:
        _need(boundaries, _U32, "boundaries")
        if boundaries.numel() != (1 << width):
            raise ValueError("boundaries must hold 2**width entries")
    _check(_lib().libsortSortKeysU32(_ptr(keys), _ptr(out), _ptr(tmp), n, offset, width,
                                     _ptr(boundaries), _stream()), "libsortSortKeysU32")
    return out


def sort_keys_range_u32(keys, lo, hi, out=None, tmp=None):
    """Full sort of uint32 keys known to lie in [lo, hi): digits of key - lo,
    so fewer passes when the range is narrow."""
    _need(keys, _U32, "keys")
    out = torch.empty_like(keys) if out is None else out
    tmp = torch.empty_like(keys) if tmp is None else tmp
    _need(out, _U32, "out")
    _need(tmp, _U32, "tmp")
    _check(_lib().libsortSortKeysRangeU32(_ptr(keys), _ptr(out), _ptr(tmp), keys.numel(), int(lo), int(hi),
                                          _stream()), "libsortSortKeysRangeU32")
    return out


def sort_pieces_u32(keys, off, lens, segs, nseg, bits, out=None, tmp=None, bias=None):
    """Sort of pre-partitioned uint32 keys (libsortSortPiecesU32): piece p =
    keys[off[p] : off[p] + lens[p]] of segment segs[p] (host arrays, pieces in
    non-decreasing segment order); every key of segment s shares its bits
    [bits, 32), increasing with s.  Returns `out` holding the sum(lens) keys
    sorted (out and tmp distinct from keys).  bias (range-digit pieces,
    libsortSortPiecesRangeU32): the shared bits are those of key - bias."""
    _need(keys, _U32, "keys")
    o = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    sg = np.ascontiguousarray(segs, dtype=np.uint32)
    if not (o.size == ln.size == sg.size):
        raise ValueError("piece tables differ in length")
    if o.size and int((o + ln).max()) > keys.numel():
        raise ValueError("piece out of range")
    n = int(ln.sum())
    out = torch.empty(n, dtype=keys.dtype, device=keys.device) if out is None else out
    tmp = torch.empty(n, dtype=keys.dtype, device=keys.device) if tmp is None else tmp
    _need(out, _U32, "out")
    _need(tmp, _U32, "tmp")
    if out.numel() < n or tmp.numel() < n:
        raise ValueError("out / tmp smaller than the pieces")
    p64 = ctypes.POINTER(ctypes.c_uint64)
    tabs = (o.ctypes.data_as(p64), ln.ctypes.data_as(p64), sg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    if bias is None:
        _check(_lib().libsortSortPiecesU32(_ptr(keys), _ptr(out), _ptr(tmp), n, *tabs, o.size, int(nseg), int(bits),
                                           _stream()), "libsortSortPiecesU32")
    else:
        _check(_lib().libsortSortPiecesRangeU32(_ptr(keys), _ptr(out), _ptr(tmp), n, *tabs, o.size, int(nseg),
                                                int(bits), int(bias) & 0xFFFFFFFF, _stream()),
               "libsortSortPiecesRangeU32")
    return out


def sort_pairs_u64_u32(keys, vals, out_keys=None, out_vals=None, tmp_keys=None, tmp_vals=None,
                       offset=0, width=None):
    """Stable sort of (uint64 key, uint32 payload) pairs by key bits."""
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    if keys.numel() != vals.numel():
        raise ValueError("keys and vals differ in length")
    if width is None:
        width = 64 - offset
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    tk = torch.empty_like(keys) if tmp_keys is None else tmp_keys
    tv = torch.empty_like(vals) if tmp_vals is None else tmp_vals
    _check(_lib().libsortSortPairsU64U32(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), _ptr(tk),
                                         _ptr(tv), keys.numel(), offset, width, _stream()),
           "libsortSortPairsU64U32")
    return ok_, ov


def sort_keys_u64(keys, out=None, tmp=None, offset=0, width=None):
    """Stable LSD sort of bits [offset, offset+width) of uint64 keys (int64
    carrier).  Returns `out`."""
    _need(keys, _U64, "keys")
    if width is None:
        width = 64 - offset
    out = torch.empty_like(keys) if out is None else out
    tmp = torch.empty_like(keys) if tmp is None else tmp
    _need(out, _U64, "out")
    _need(tmp, _U64, "tmp")
    _check(_lib().libsortSortKeysU64(_ptr(keys), _ptr(out), _ptr(tmp), keys.numel(), offset, width, _stream()),
           "libsortSortKeysU64")
    return out


def sort_pairs_u64_u64(keys, vals, out_keys=None, out_vals=None, tmp_keys=None, tmp_vals=None,
                       offset=0, width=None):
    """Stable sort of (uint64 key, uint64 payload) pairs by key bits."""
    _need(keys, _U64, "keys")
    _need(vals, _U64, "vals")
    if keys.numel() != vals.numel():
        raise ValueError("keys and vals differ in length")
    if width is None:
        width = 64 - offset
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    tk = torch.empty_like(keys) if tmp_keys is None else tmp_keys
    tv = torch.empty_like(vals) if tmp_vals is None else tmp_vals
    _check(_lib().libsortSortPairsU64U64(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), _ptr(tk),
                                         _ptr(tv), keys.numel(), offset, width, _stream()),
           "libsortSortPairsU64U64")
    return ok_, ov


def sort_pairs_u32_u32(keys, vals, out_keys=None, out_vals=None, tmp_keys=None, tmp_vals=None,
                       offset=0, width=None):
    """Stable sort of (uint32 key, uint32 payload) pairs by key bits."""
    _need(keys, _U32, "keys")
    _need(vals, _U32, "vals")
    if keys.numel() != vals.numel():
        raise ValueError("keys and vals differ in length")
    if width is None:
        width = 32 - offset
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    tk = torch.empty_like(keys) if tmp_keys is None else tmp_keys
    tv = torch.empty_like(vals) if tmp_vals is None else tmp_vals
    _check(_lib().libsortSortPairsU32U32(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), _ptr(tk),
                                         _ptr(tv), keys.numel(), offset, width, _stream()),
           "libsortSortPairsU32U32")
    return ok_, ov


def histogram_u32(keys, shift, bits, out=None):
    """Counts of (key >> shift) & (2**bits-1) into an int32 tensor of 2**bits."""
    _need(keys, _U32, "keys")
    out = torch.empty(1 << bits, dtype=torch.int32, device=keys.device) if out is None else out
    _check(_lib().libsortHistogramU32(_ptr(keys), keys.numel(), shift, bits, _ptr(out), _stream()),
           "libsortHistogramU32")
    return out


def partition_u32(keys, splitters, out=None, counts=None):
    """Stable range partition: bucket(x) = #{s in splitters : x >= s}."""
    _need(keys, _U32, "keys")
    sp = [int(s) for s in splitters]
    arr = (ctypes.c_uint32 * max(1, len(sp)))(*sp)
    out = torch.empty_like(keys) if out is None else out
    counts = (torch.empty(len(sp) + 1, dtype=torch.int32, device=keys.device)
              if counts is None else counts)
    _check(_lib().libsortPartitionU32(_ptr(keys), _ptr(out), keys.numel(), arr, len(sp),
                                      _ptr(counts), _stream()), "libsortPartitionU32")
    return out, counts


def partition_lut_u32(keys, lut, lut_shift, nbuckets, out=None, bounds=None):
    """Stable partition by bucket = lut[key >> lut_shift] (lut: uint8 CUDA
    tensor of 2**(32 - lut_shift) entries, each < nbuckets).  Returns (out,
    bounds) with bounds = int32 tensor of the nbuckets bucket starts."""
    _need(keys, _U32, "keys")
    if lut.dtype != torch.uint8 or not lut.is_cuda or lut.numel() != 1 << (32 - lut_shift):
        raise ValueError("lut must be a uint8 CUDA tensor of 2**(32 - lut_shift) entries")
    lut = lut.contiguous()
    out = torch.empty_like(keys) if out is None else out
    _need(out, _U32, "out")
    bounds = torch.empty(nbuckets, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionLutU32(_ptr(keys), _ptr(out), keys.numel(), _ptr(lut), lut_shift, nbuckets,
                                         _ptr(bounds), _stream()), "libsortPartitionLutU32")
    return out, bounds


def partition_lut_pairs_u64_u32(keys, vals, lut, lut_shift, nbuckets, out_keys=None, out_vals=None,
                                bounds=None):
    """Stable partition of (uint64 key, uint32 payload) pairs by bucket =
    lut[(key >> 32) >> lut_shift].  Returns (out_keys, out_vals, bounds)."""
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    if keys.numel() != vals.numel():
        raise ValueError("keys and vals differ in length")
    if lut.dtype != torch.uint8 or not lut.is_cuda or lut.numel() != 1 << (32 - lut_shift):
        raise ValueError("lut must be a uint8 CUDA tensor of 2**(32 - lut_shift) entries")
    lut = lut.contiguous()
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    bounds = torch.empty(nbuckets, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionLutU64U32(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), keys.numel(), _ptr(lut),
                                            lut_shift, nbuckets, _ptr(bounds), _stream()),
           "libsortPartitionLutU64U32")
    return ok_, ov, bounds


def _lut_check(lut, lut_shift):
    if lut.dtype != torch.uint8 or not lut.is_cuda or lut.numel() != 1 << (32 - lut_shift):
        raise ValueError("lut must be a uint8 CUDA tensor of 2**(32 - lut_shift) entries")
    return lut.contiguous()


def partition_lut_count_u32(keys, lut, lut_shift, nbuckets, bounds=None):
    """First half of partition_lut_u32: counts + scan, bucket starts (int32
    tensor).  partition_lut_scatter_u32 with the same arguments must follow."""
    _need(keys, _U32, "keys")
    lut = _lut_check(lut, lut_shift)
    bounds = torch.empty(nbuckets, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionLutCountU32(_ptr(keys), keys.numel(), _ptr(lut), lut_shift, nbuckets, _ptr(bounds),
                                              _stream()), "libsortPartitionLutCountU32")
    return bounds


def partition_lut_scatter_u32(keys, lut, lut_shift, nbuckets, out=None):
    """Second half of partition_lut_u32: the data movement."""
    _need(keys, _U32, "keys")
    lut = _lut_check(lut, lut_shift)
    out = torch.empty_like(keys) if out is None else out
    _need(out, _U32, "out")
    _check(_lib().libsortPartitionLutScatterU32(_ptr(keys), _ptr(out), keys.numel(), _ptr(lut), lut_shift, nbuckets,
                                                _stream()), "libsortPartitionLutScatterU32")
    return out


def partition_lut_pairs_count_u64_u32(keys, vals, lut, lut_shift, nbuckets, bounds=None):
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    lut = _lut_check(lut, lut_shift)
    bounds = torch.empty(nbuckets, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionLutCountU64U32(_ptr(keys), _ptr(vals), keys.numel(), _ptr(lut), lut_shift, nbuckets,
                                                 _ptr(bounds), _stream()), "libsortPartitionLutCountU64U32")
    return bounds


def partition_lut_pairs_scatter_u64_u32(keys, vals, lut, lut_shift, nbuckets, out_keys=None, out_vals=None):
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    lut = _lut_check(lut, lut_shift)
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    _check(_lib().libsortPartitionLutScatterU64U32(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), keys.numel(),
                                                   _ptr(lut), lut_shift, nbuckets, _stream()),
           "libsortPartitionLutScatterU64U32")
    return ok_, ov


def partition_range_count_u32(keys, bias, shift, bounds=None):
    """Count half of the range-digit partition (digit = (key - bias) >> shift,
    256 buckets): the bucket starts (int32 tensor) while nothing has moved.
    partition_range_scatter_u32 with the same arguments must follow."""
    _need(keys, _U32, "keys")
    bounds = torch.empty(256, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionRangeCountU32(_ptr(keys), keys.numel(), int(bias) & 0xFFFFFFFF, int(shift),
                                                _ptr(bounds), _stream()), "libsortPartitionRangeCountU32")
    return bounds


def partition_range_scatter_u32(keys, bias, shift, out=None):
    _need(keys, _U32, "keys")
    out = torch.empty_like(keys) if out is None else out
    _need(out, _U32, "out")
    _check(_lib().libsortPartitionRangeScatterU32(_ptr(keys), _ptr(out), keys.numel(), int(bias) & 0xFFFFFFFF,
                                                  int(shift), _stream()), "libsortPartitionRangeScatterU32")
    return out


def partition_range_pairs_count_u64_u32(keys, vals, bias, shift, bounds=None):
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    bounds = torch.empty(256, dtype=torch.int32, device=keys.device) if bounds is None else bounds
    _check(_lib().libsortPartitionRangeCountU64U32(_ptr(keys), _ptr(vals), keys.numel(), int(bias), int(shift),
                                                   _ptr(bounds), _stream()), "libsortPartitionRangeCountU64U32")
    return bounds


def partition_range_pairs_scatter_u64_u32(keys, vals, bias, shift, out_keys=None, out_vals=None):
    _need(keys, _U64, "keys")
    _need(vals, _U32, "vals")
    ok_ = torch.empty_like(keys) if out_keys is None else out_keys
    ov = torch.empty_like(vals) if out_vals is None else out_vals
    _check(_lib().libsortPartitionRangeScatterU64U32(_ptr(keys), _ptr(vals), _ptr(ok_), _ptr(ov), keys.numel(),
                                                     int(bias), int(shift), _stream()),
           "libsortPartitionRangeScatterU64U32")
    return ok_, ov


def minmax_u32(keys, out=None):
    """(smallest, largest) key as a 2-element int32 tensor holding uint32 bits
    (n == 0: 0xFFFFFFFF, 0)."""
    _need(keys, _U32, "keys")
    out = torch.empty(2, dtype=torch.int32, device=keys.device) if out is None else out
    _check(_lib().libsortMinMaxU32(_ptr(keys), keys.numel(), _ptr(out), _stream()), "libsortMinMaxU32")
    return out


def minmax_u64(keys, out=None):
    """(smallest, largest) uint64 key as a 2-element int64 tensor of the bits."""
    _need(keys, _U64, "keys")
    out = torch.empty(2, dtype=torch.int64, device=keys.device) if out is None else out
    _check(_lib().libsortMinMaxU64(_ptr(keys), keys.numel(), _ptr(out), _stream()), "libsortMinMaxU64")
    return out


def segment_copy_u32(src, dst, src_off, dst_off, lens):
    """dst[dst_off[i] + j] = src[src_off[i] + j] for j < lens[i]."""
    _need(src, _U32, "src")
    _need(dst, _U32, "dst")
    so = np.ascontiguousarray(src_off, dtype=np.uint64)
    do = np.ascontiguousarray(dst_off, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    if not (so.size == do.size == ln.size):
        raise ValueError("segment tables differ in length")
    if so.size and (int((so + ln).max()) > src.numel() or int((do + ln).max()) > dst.numel()):
        raise ValueError("segment out of range")
    p = ctypes.POINTER(ctypes.c_uint64)
    _check(_lib().libsortSegmentCopyU32(_ptr(src), _ptr(dst), so.size, so.ctypes.data_as(p),
                                        do.ctypes.data_as(p), ln.ctypes.data_as(p), _stream()),
           "libsortSegmentCopyU32")
    return dst


DELTA_GROUP = 64  # keys per coded group (radix_kernels.hip kDeltaGroup)


def delta_bits(maxgap):
    """Bit width of the coded gaps for a run whose largest in-group gap is maxgap."""
    return int(maxgap).bit_length()


def delta_words(n, bits):
    """uint32 words of a delta-coded run of n keys with gap width `bits`."""
    return -(-int(n) // DELTA_GROUP) * (1 + 2 * int(bits))


def delta_maxgap_u32(keys, out=None):
    """Largest gap between neighbours inside each 64-key group of the sorted
    run `keys`, as a one-element int32 tensor on the device."""
    _need(keys, _U32, "keys")
    out = torch.empty(1, dtype=torch.int32, device=keys.device) if out is None else out
    _check(_lib().libsortDeltaMaxGapU32(_ptr(keys), keys.numel(), _ptr(out), _stream()), "libsortDeltaMaxGapU32")
    return out


def delta_pack_u32(keys, maxgap, out=None, capacity=None):
    """Delta-code the sorted run `keys` with the gap width implied by the
    device word `maxgap` (delta_maxgap_u32).  `out` must hold the coded size
    (delta_words); without it, a buffer of `capacity` words (default: the
    32-bit worst case) is allocated."""
    _need(keys, _U32, "keys")
    _need(maxgap, _U32, "maxgap")
    if out is None:
        out = torch.empty(capacity if capacity is not None else delta_words(keys.numel(), 32),
                          dtype=torch.int32, device=keys.device)
    _need(out, _U32, "out")
    _check(_lib().libsortDeltaPackU32(_ptr(keys), keys.numel(), _ptr(maxgap), _ptr(out), _stream()),
           "libsortDeltaPackU32")
    return out


def delta_unpack_u32(coded, n, bits, out=None):
    """Decode n keys from a delta-coded run with gap width `bits`."""
    _need(coded, _U32, "coded")
    if coded.numel() < delta_words(n, bits):
        raise ValueError("coded run holds %d words, %d needed" % (coded.numel(), delta_words(n, bits)))
    out = torch.empty(n, dtype=torch.int32, device=coded.device) if out is None else out
    _need(out, _U32, "out")
    _check(_lib().libsortDeltaUnpackU32(_ptr(coded), int(n), int(bits), _ptr(out), _stream()), "libsortDeltaUnpackU32")
    return out


def merge_u32(a, b, out=None):
    """Merge two sorted uint32 runs into `out` (distinct from both)."""
    _need(a, _U32, "a")
    _need(b, _U32, "b")
    out = torch.empty(a.numel() + b.numel(), dtype=torch.int32, device=a.device) if out is None else out
    _need(out, _U32, "out")
    if out.numel() != a.numel() + b.numel():
        raise ValueError("out must hold len(a) + len(b) keys")
    _check(_lib().libsortMergeU32(_ptr(a), a.numel(), _ptr(b), b.numel(), _ptr(out), _stream()), "libsortMergeU32")
    return out


LIBSORT_DISTRIB_LSD, LIBSORT_DISTRIB_COPY, LIBSORT_DISTRIB_SELF_RCCL, LIBSORT_DISTRIB_WIRE32 = 1, 2, 4, 8
LIBSORT_DISTRIB_CODED = 16


def distrib_last_bytes(nranks):
    """Bytes each rank sent to the others in the last distributed sort
    (libsortDistribLastBytes), as a list of ints."""
    arr = (ctypes.c_uint64 * nranks)()
    _check(_lib().libsortDistribLastBytes(int(nranks), arr), "libsortDistribLastBytes")
    return [int(x) for x in arr]


def distrib_sort_u32(shards, flags=0):
    """libsortDistribSortU32: the single-process multi-GPU sort over the
    shards' devices (tensors may share a device).  Returns rank r's shard of
    the sorted whole (keys [r*S, (r+1)*S), S = ceil(N/R)) on shard r's device.
    Synchronous; the shards' producers are waited for first."""
    R = len(shards)
    devs = []
    for i, t in enumerate(shards):
        _need(t, _U32, "shards[%d]" % i)
        devs.append(t.device.index)
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)
    N = sum(t.numel() for t in shards)
    S = -(-N // R) if R else 0
    outs = [torch.empty(max(S, 1), dtype=torch.int32, device=t.device) for t in shards]
    arr_dev = (ctypes.c_int * R)(*devs)
    arr_in = (ctypes.c_void_p * R)(*[t.data_ptr() for t in shards])
    arr_n = (ctypes.c_size_t * R)(*[t.numel() for t in shards])
    arr_out = (ctypes.c_void_p * R)(*[t.data_ptr() for t in outs])
    arr_nout = (ctypes.c_size_t * R)()
    _check(_lib().libsortDistribSortU32(R, arr_dev, arr_in, arr_n, arr_out, arr_nout, flags),
           "libsortDistribSortU32")
    return [o[:int(arr_nout[r])] for r, o in enumerate(outs)]


def distrib_sort_pairs_u64_u32(key_shards, val_shards, flags=0):
    """libsortDistribSortPairsU64U32: the single-process multi-GPU stable
    sort of (uint64 key, uint32 payload) pairs (configs[4]).  Returns rank
    r's (keys, payloads) shard of the sorted whole on shard r's device."""
    R = len(key_shards)
    if len(val_shards) != R:
        raise ValueError("one payload shard per key shard")
    devs = []
    for i, (k, v) in enumerate(zip(key_shards, val_shards)):
        _need(k, _U64, "key_shards[%d]" % i)
        _need(v, _U32, "val_shards[%d]" % i)
        if k.numel() != v.numel() or k.device != v.device:
            raise ValueError("shard %d: keys and payloads differ in length or device" % i)
        devs.append(k.device.index)
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)
    N = sum(t.numel() for t in key_shards)
    S = -(-N // R) if R else 0
    ko = [torch.empty(max(S, 1), dtype=torch.int64, device=t.device) for t in key_shards]
    vo = [torch.empty(max(S, 1), dtype=torch.int32, device=t.device) for t in key_shards]
    P = ctypes.c_void_p * R
    arr_nout = (ctypes.c_size_t * R)()
    _check(_lib().libsortDistribSortPairsU64U32(R, (ctypes.c_int * R)(*devs), P(*[t.data_ptr() for t in key_shards]),
                                                P(*[t.data_ptr() for t in val_shards]),
                                                (ctypes.c_size_t * R)(*[t.numel() for t in key_shards]),
                                                P(*[t.data_ptr() for t in ko]), P(*[t.data_ptr() for t in vo]),
                                                arr_nout, flags), "libsortDistribSortPairsU64U32")
    return [k[:int(arr_nout[r])] for r, k in enumerate(ko)], [v[:int(arr_nout[r])] for r, v in enumerate(vo)]


def populate_u32(n, first=0, device=None, out=None):
    """Elements [first, first+n) of the reference populateInput stream (fresh
    process), generated on the device."""
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=device or torch.device("cuda"))
    _need(out, _U32, "out")
    _check(_lib().libsortPopulateDevice(_ptr(out), n, first, _stream()), "libsortPopulateDevice")
    return out


def timing_enable(on=True):
    _lib().libsortTimingEnable(bool(on))


def timing_reset():
    _lib().libsortTimingReset()


def timing_filter(kernels=None):
    """Record only the named kernels (a list or comma-separated string); None = all."""
    if kernels is not None and not isinstance(kernels, str):
        kernels = ",".join(kernels)
    _lib().libsortTimingFilter(kernels.encode() if kernels else None)


def timing_sample(every=1):
    """Record only every `every`-th filtered launch (libsortTimingSample)."""
    _lib().libsortTimingSample(int(every))


def timing_query(kernel):
    """(launches, total_ms, total_keys) of the recorded launches of `kernel`."""
    n = ctypes.c_uint64()
    ms = ctypes.c_double()
    k = ctypes.c_uint64()
    _check(_lib().libsortTimingQuery(kernel.encode(), ctypes.byref(n), ctypes.byref(ms),
                                     ctypes.byref(k)), "libsortTimingQuery")
    return n.value, ms.value, k.value


def as_u32_numpy(t):
    """Host numpy uint32 view of a uint32-carrying tensor."""
    return t.detach().cpu().numpy().view(np.uint32)
