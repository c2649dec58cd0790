"""GPU parity: libsort's HIP path (through the C ABI) against the oracle.

Sizes where the oracle finishes in seconds are compared element-wise; the
reference-size runs (2^28) are checked through the reference's own sha256 of
the sorted PCG stream plus size-independent properties.
"""
import hashlib
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SIZES = [0, 1, 2, 63, 64, 127, 129, 1021, 1111, 4095, 4096, 4097, 4099, 65539, 1 << 20, (1 << 22) + 5]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pylibsort
    import pylibsort.device as D
    assert pylibsort.gpu_ready(), pylibsort.last_error()
    return D


@pytest.fixture(params=[(4, "tiles"), (8, "tiles")], ids=["digit4", "digit8"])
def digit_bits(request, dev):
    """Every parity case runs under both digit widths of the product path (the
    tile-offset algorithm, which `auto` always picks); the non-default pass
    algorithms are covered by test_non_default_algorithms."""
    import pylibsort
    bits, algo = request.param
    prev = pylibsort.setDigitBits(bits)
    prev_algo = pylibsort.setAlgorithm(algo)
    yield bits
    assert pylibsort.lib().libsortDeviceErrors() == 0, "look-back spin bound hit"
    pylibsort.setDigitBits(prev)
    pylibsort.setAlgorithm(prev_algo)


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def _tensor(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda()


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u4").tobytes()).hexdigest()[:16]


def test_populate_device_matches_oracle(dev, oracle_mod, golden):
    g, _ = golden
    t = dev.populate_u32(1 << 20)
    got = _u32(t)
    assert [format(x, "08x") for x in got[:8]] == g["fresh_process_first_words"]
    assert sha16(got) == g["sha256_prefix"]["1048576"]["input"]
    # skip-ahead from an arbitrary offset
    first = 123457
    t2 = dev.populate_u32(4099, first=first)
    np.testing.assert_array_equal(_u32(t2), oracle_mod.pcg(4099, first=first))


@pytest.mark.ab  # (A/B pass algorithms the product path never picks: LIBSORT_TEST_AB=1 runs them)
@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("algo", ["onesweep", "rts"])
def test_non_default_algorithms(dev, oracle_mod, bits, algo):
    """The A/B pass algorithms (LIBSORT_ALGO=onesweep: decoupled look-back;
    rts: reduce-then-scan with the Blelloch-style scan) stay exact: full
    sorts over ragged sizes, partial sorts with boundaries, duplicate-heavy
    and presorted inputs, against the oracle."""
    import pylibsort
    prev_b, prev_a = pylibsort.setDigitBits(bits), pylibsort.setAlgorithm(algo)
    try:
        for n in (0, 1, 127, 4097, 65539, (1 << 20) + 3):
            x = oracle_mod.pcg(n, first=3 * n + bits)
            np.testing.assert_array_equal(_u32(dev.sort_keys_u32(_tensor(x))), oracle_mod.sort_u32(x))
        for n, off, w in ((1021, 0, 8), (4099, 4, 8), (100003, 3, 5), (65539, 0, 16)):
            x = oracle_mod.pcg(n, first=n + off)
            b = torch.empty(1 << w, dtype=torch.int32, device="cuda")
            out = dev.sort_keys_u32(_tensor(x), offset=off, width=w, boundaries=b)
            d, bb = oracle_mod.partial_u32(x, off, w)
            np.testing.assert_array_equal(_u32(out), d)
            np.testing.assert_array_equal(_u32(b), bb)
        rng = np.random.default_rng(bits)
        for x in (rng.integers(0, 4, 300007, dtype=np.uint64).astype(np.uint32),
                  np.sort(oracle_mod.pcg(70001))[::-1].copy(), np.full(5000, 9, dtype=np.uint32)):
            np.testing.assert_array_equal(_u32(dev.sort_keys_u32(_tensor(x))), oracle_mod.sort_u32(x))
        assert pylibsort.lib().libsortDeviceErrors() == 0, "look-back spin bound hit"
    finally:
        pylibsort.setDigitBits(prev_b)
        pylibsort.setAlgorithm(prev_a)


@pytest.mark.parametrize("n", SIZES)
def test_full_sort_matches_oracle(dev, oracle_mod, digit_bits, n):
    x = oracle_mod.pcg(n, first=7 * n)
    out = dev.sort_keys_u32(_tensor(x))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


@pytest.mark.parametrize("n", [1021, 1111, 4099, 100003])
@pytest.mark.parametrize("offset,width", [(0, 8), (4, 8), (0, 4), (6, 4), (0, 16), (3, 5), (0, 1),
                                          (8, 13), (24, 8), (31, 1), (0, 31), (1, 31)])
def test_partial_sort_and_boundaries(dev, oracle_mod, digit_bits, n, offset, width):
    x = oracle_mod.pcg(n, first=n + offset)
    b = torch.empty(1 << width, dtype=torch.int32, device="cuda") if width <= 20 else None
    out = dev.sort_keys_u32(_tensor(x), offset=offset, width=width, boundaries=b)
    torch.cuda.synchronize()
    ref_data, ref_bounds = oracle_mod.partial_u32(x, offset, width) if width <= 20 else (None, None)
    if ref_data is None:
        # wide groups: the stable partition equals a stable sort by the group
        key = (x.astype(np.uint64) >> np.uint64(offset)) & np.uint64((1 << width) - 1)
        ref_data = x[np.argsort(key, kind="stable")]
    np.testing.assert_array_equal(_u32(out), ref_data)
    if b is not None:
        np.testing.assert_array_equal(_u32(b), ref_bounds)


@pytest.mark.parametrize("n,width,offset", [(3, 31, 0), (1000, 31, 1), (5, 24, 8), (100003, 24, 0), (1, 20, 12)])
def test_wide_group_boundaries(dev, oracle_mod, n, width, offset):
    """Boundaries of wide groups (up to 2^31 of them) from few keys: every
    empty group takes the next non-empty group's start, in parallel (the
    first version filled the gap after the last key in one thread: ~2^31
    serial stores for n = 3).  Complete check without copying 8 GiB: the
    bounds are non-decreasing and exact at g = 0, the last group, and every
    present group value v and v + 1 -- a non-decreasing sequence pinned there
    is pinned everywhere."""
    import time
    x = oracle_mod.pcg(n, first=width * 7 + n)
    ng = 1 << width
    b = torch.empty(ng, dtype=torch.int32, device="cuda")
    t = _tensor(x)
    out = dev.sort_keys_u32(t, offset=offset, width=width, boundaries=b)   # warm-up (allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = dev.sort_keys_u32(t, offset=offset, width=width, boundaries=b)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    grp = (x.astype(np.uint64) >> np.uint64(offset)) & np.uint64(ng - 1)
    o = np.argsort(grp, kind="stable")
    np.testing.assert_array_equal(_u32(out), x[o])
    sg = np.sort(grp)
    bb = (b.to(torch.int64) & 0xFFFFFFFF)
    chunk = 1 << 26
    for i in range(0, ng, chunk):
        seg = bb[i:i + chunk + 1]
        assert bool((seg[1:] >= seg[:-1]).all())
    probes = np.unique(np.concatenate([[0, ng - 1], sg, np.minimum(sg + 1, ng - 1)]).astype(np.int64))
    got = bb[torch.from_numpy(probes).cuda()].cpu().numpy()
    np.testing.assert_array_equal(got, np.searchsorted(sg, probes.astype(np.uint64), side="left"))
    if width <= 24:
        np.testing.assert_array_equal(bb.cpu().numpy(), np.searchsorted(sg, np.arange(ng, dtype=np.uint64)))
    assert elapsed < 0.5, elapsed
    del b, bb
    torch.cuda.empty_cache()


def test_partial_matches_reference_kernel_emulation(dev, oracle_mod, digit_bits):
    # exact emulation of the reference's 2-bit kernels == our stable partition
    for n, off, w in ((1111, 0, 8), (1021, 4, 8), (300, 6, 4), (4099, 0, 32)):
        x = oracle_mod.pcg(n, first=3 * n)
        out = dev.sort_keys_u32(_tensor(x), offset=off, width=w)
        np.testing.assert_array_equal(_u32(out), oracle_mod.ref_step_u32(x, off, w))


@pytest.mark.parametrize("kind", ["equal", "four", "sorted", "reverse", "bucket1_empty", "low_entropy"])
def test_edge_distributions(dev, oracle_mod, digit_bits, kind):
    n = 50021
    rng = np.random.default_rng(5)
    if kind == "equal":
        x = np.full(n, 0xdeadbeef, dtype=np.uint32)
    elif kind == "four":
        x = rng.choice(np.array([0, 7, 1 << 31, 0xffffffff], dtype=np.uint32), n)
    elif kind == "sorted":
        x = np.sort(rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
    elif kind == "reverse":
        x = np.sort(rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))[::-1].copy()
    elif kind == "bucket1_empty":
        x = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        x[(x & 0xff) == 1] = 2
    else:
        x = (rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) & 0x0f0f0f0f)
    out = dev.sort_keys_u32(_tensor(x))
    np.testing.assert_array_equal(_u32(out), np.sort(x))
    b = torch.empty(256, dtype=torch.int32, device="cuda")
    out = dev.sort_keys_u32(_tensor(x), offset=0, width=8, boundaries=b)
    d, bb = oracle_mod.partial_u32(x, 0, 8)
    np.testing.assert_array_equal(_u32(out), d)
    np.testing.assert_array_equal(_u32(b), bb)


@pytest.mark.parametrize("lo,hi", [(0, 1 << 32), (0, 1 << 27), (0x12300000, 0x12300000 + (1 << 27)),
                                   (0xF0000000, 1 << 32), (0x80000001, 0x80000001 + 3000), (777, 778)])
@pytest.mark.parametrize("n", [1, 4097, 300001])
def test_sort_keys_range(dev, oracle_mod, digit_bits, lo, hi, n):
    """libsortSortKeysRangeU32 (digits of key - lo, ceil(log2(hi - lo) / bits)
    passes) == a full sort, for keys inside [lo, hi)."""
    x = oracle_mod.pcg(n, first=lo % 1000 + n)
    x = (np.uint64(lo) + x.astype(np.uint64) % np.uint64(hi - lo)).astype(np.uint32)
    got = dev.sort_keys_range_u32(_tensor(x), lo, hi)
    np.testing.assert_array_equal(_u32(got), np.sort(x))


def test_in_place_device_sort(dev, oracle_mod, digit_bits):
    x = oracle_mod.pcg(77777, first=5)
    t = _tensor(x)
    for w in (8, 16, 24, 32):  # odd and even pass counts
        t = _tensor(x)
        dev.sort_keys_u32(t, out=t, offset=0, width=w)
        d, _ = oracle_mod.partial_u32(x, 0, w) if w <= 24 else (np.sort(x), None)
        np.testing.assert_array_equal(_u32(t), d)


@pytest.mark.parametrize("n", [1, 2049, 300007])
def test_pairs_u64_u32_stable(dev, oracle_mod, digit_bits, n):
    rng = np.random.default_rng(n)
    k = rng.integers(0, 1 << 20, n, dtype=np.uint64) * np.uint64(0x100000001)  # many duplicates
    v = np.arange(n, dtype=np.uint32)
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    ok_, ov = dev.sort_pairs_u64_u32(kt, vt)
    rk, rv = oracle_mod.stable_sort_kv64(k, v)
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint32), rv)


@pytest.mark.parametrize("n", [1, 2049, 300007])
@pytest.mark.parametrize("offset,width", [(0, 64), (0, 40), (17, 31), (32, 32)])
def test_keys_u64(dev, oracle_mod, digit_bits, n, offset, width):
    rng = np.random.default_rng(n + offset)
    k = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    k[: n // 3] &= np.uint64(0xFFFF0000FFFF)  # duplicates and zero digits
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    out = dev.sort_keys_u64(kt, offset=offset, width=width)
    if (offset, width) == (0, 64):
        ref = oracle_mod.sort_u64(k)
    else:  # stable by the digit field: the same permutation as a stable pair sort
        field = (k >> np.uint64(offset)) & np.uint64((1 << width) - 1)
        _, idx = oracle_mod.stable_sort_kv64v64(field, np.arange(n, dtype=np.uint64))
        ref = k[idx.astype(np.int64)]
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), ref)


@pytest.mark.parametrize("n", [1, 2049, 300007])
def test_pairs_u64_u64_stable(dev, oracle_mod, digit_bits, n):
    rng = np.random.default_rng(n)
    k = rng.integers(0, 1 << 20, n, dtype=np.uint64) * np.uint64(0x100000001)  # many duplicates
    v = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (np.arange(n, dtype=np.uint64) << np.uint64(40))
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int64)).cuda()
    ok_, ov = dev.sort_pairs_u64_u64(kt, vt)
    rk, rv = oracle_mod.stable_sort_kv64v64(k, v)
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint64), rv)


def test_pairs_u32_u32_stable(dev, oracle_mod, digit_bits):
    n = 123457
    rng = np.random.default_rng(1)
    k = rng.integers(0, 1000, n, dtype=np.uint64).astype(np.uint32)
    v = np.arange(n, dtype=np.uint32)
    ok_, ov = dev.sort_pairs_u32_u32(_tensor(k), _tensor(v))
    rk, rv = oracle_mod.stable_sort_kv32(k, v)
    np.testing.assert_array_equal(_u32(ok_), rk)
    np.testing.assert_array_equal(_u32(ov), rv)


def test_histogram_and_partition(dev, oracle_mod):
    x = oracle_mod.pcg(200003, first=11)
    for shift, bits in ((0, 8), (20, 12), (16, 16), (28, 4)):
        h = dev.histogram_u32(_tensor(x), shift, bits)
        ref = np.bincount((x >> shift) & ((1 << bits) - 1), minlength=1 << bits)
        np.testing.assert_array_equal(h.cpu().numpy(), ref)
    for sp in ([1 << 31], [1 << 29, 1 << 30, 3 << 30], sorted(int(v) for v in x[:200])):
        out, cnt = dev.partition_u32(_tensor(x), sp)
        bucket = np.searchsorted(np.array(sp, dtype=np.uint64), x.astype(np.uint64), side="right")
        ref = x[np.argsort(bucket, kind="stable")]
        np.testing.assert_array_equal(_u32(out), ref)
        np.testing.assert_array_equal(cnt.cpu().numpy(), np.bincount(bucket, minlength=len(sp) + 1))


@pytest.mark.parametrize("n", [0, 1, 4095, 4097, 200003, 1 << 20])
@pytest.mark.parametrize("shift,nbuckets", [(20, 2), (20, 16), (24, 17), (20, 32), (28, 16), (30, 4), (20, 256)])
def test_partition_lut(dev, oracle_mod, n, shift, nbuckets):
    """libsortPartitionLutU32 (the multi-GPU schedule's partition) against a
    stable numpy partition; 4-bit (<= 16 buckets) and 8-bit tile paths,
    partial last tiles, buckets left empty."""
    x = oracle_mod.pcg(n, first=n + shift)
    rng = np.random.default_rng(shift * 1000 + nbuckets)
    lut = np.sort(rng.integers(0, nbuckets, 1 << (32 - shift))).astype(np.uint8)  # contiguous ranges
    if nbuckets == 32:
        lut = rng.integers(0, nbuckets, 1 << (32 - shift)).astype(np.uint8)        # arbitrary table
    out, b = dev.partition_lut_u32(_tensor(x), torch.from_numpy(lut).cuda(), shift, nbuckets)
    bucket = lut[x >> np.uint32(shift)].astype(np.int64)
    np.testing.assert_array_equal(_u32(out), x[np.argsort(bucket, kind="stable")])
    starts = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nbuckets))[:-1]])
    np.testing.assert_array_equal(b.cpu().numpy().astype(np.int64), starts)


@pytest.mark.parametrize("n", [0, 4097, 1 << 20])
@pytest.mark.parametrize("nbuckets", [16, 32, 200])
def test_partition_lut_split(dev, oracle_mod, n, nbuckets):
    """The two-call partition (count + scan, then scatter) gives the one-call
    result, for keys and for (u64, u32) pairs; a scatter without its count
    call, or after another sort used the workspace, fails loudly."""
    x = oracle_mod.pcg(n, first=7 * n + nbuckets)
    rng = np.random.default_rng(nbuckets)
    lut = torch.from_numpy(np.sort(rng.integers(0, nbuckets, 4096)).astype(np.uint8)).cuda()
    t = _tensor(x)
    ref, rb = dev.partition_lut_u32(t, lut, 20, nbuckets)
    b = dev.partition_lut_count_u32(t, lut, 20, nbuckets)
    out = dev.partition_lut_scatter_u32(t, lut, 20, nbuckets)
    torch.cuda.synchronize()
    assert torch.equal(b, rb) and torch.equal(out, ref)
    if n == 0:
        return
    with pytest.raises(RuntimeError):
        dev.partition_lut_scatter_u32(t, lut, 20, nbuckets)       # already consumed
    dev.partition_lut_count_u32(t, lut, 20, nbuckets)
    dev.sort_keys_u32(t)                                           # uses the workspace in between
    with pytest.raises(RuntimeError):
        dev.partition_lut_scatter_u32(t, lut, 20, nbuckets)
    k = torch.from_numpy((x.astype(np.uint64) << np.uint64(32) | np.uint64(5)).view(np.int64)).cuda()
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    rk, rv, rb2 = dev.partition_lut_pairs_u64_u32(k, v, lut, 20, nbuckets)
    b2 = dev.partition_lut_pairs_count_u64_u32(k, v, lut, 20, nbuckets)
    k2, v2 = dev.partition_lut_pairs_scatter_u64_u32(k, v, lut, 20, nbuckets)
    torch.cuda.synchronize()
    assert torch.equal(b2, rb2) and torch.equal(k2, rk) and torch.equal(v2, rv)


@pytest.mark.parametrize("n", [0, 3, 2049, 300007])
@pytest.mark.parametrize("nbuckets", [8, 16, 64])
def test_partition_lut_pairs(dev, n, nbuckets):
    """libsortPartitionLutU64U32 (the C5 multi-GPU partition): stable, pairs
    move together, bucket = lut[(key >> 32) >> 20]."""
    rng = np.random.default_rng(n + nbuckets)
    k = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    k[: n // 3] = k[0] if n else 0  # equal keys: stability visible in the payloads
    v = np.arange(n, dtype=np.uint32)
    lut = np.sort(rng.integers(0, nbuckets, 4096)).astype(np.uint8)
    ok_, ov, b = dev.partition_lut_pairs_u64_u32(torch.from_numpy(k.view(np.int64)).cuda(),
                                                 torch.from_numpy(v.view(np.int32)).cuda(),
                                                 torch.from_numpy(lut).cuda(), 20, nbuckets)
    bucket = lut[(k >> np.uint64(52)).astype(np.int64)].astype(np.int64)
    o = np.argsort(bucket, kind="stable")
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), k[o])
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint32), v[o])
    starts = np.concatenate([[0], np.cumsum(np.bincount(bucket, minlength=nbuckets))[:-1]])
    np.testing.assert_array_equal(b.cpu().numpy().astype(np.int64), starts)


def test_segment_copy(dev):
    src = torch.arange(1000, dtype=torch.int32, device="cuda")
    dst = torch.zeros(1000, dtype=torch.int32, device="cuda")
    so = np.array([0, 500, 100], dtype=np.uint64)
    do = np.array([900, 0, 400], dtype=np.uint64)
    ln = np.array([100, 400, 300], dtype=np.uint64)
    dev.segment_copy_u32(src, dst, so, do, ln)
    ref = np.zeros(1000, dtype=np.int32)
    for a, b, c in zip(so, do, ln):
        ref[int(b):int(b + c)] = np.arange(int(a), int(a + c))
    np.testing.assert_array_equal(dst.cpu().numpy(), ref)


# ---- host-pointer ABI (the drop-in boundary) --------------------------------

def test_host_abi_matches_golden(dev, golden):
    import pylibsort
    g, v = golden
    for n in (1021, 1111, 4099):
        buf = bytearray(v["in_%d" % n].astype("<u4").tobytes())
        pylibsort.sortFull(buf)
        got = np.frombuffer(buf, dtype=np.uint32)
        assert sha16(got) == g["sha256_prefix"][str(n)]["sorted"]
        for off, w in ((0, 8), (0, 4), (4, 8), (6, 4)):
            buf = bytearray(v["in_%d" % n].astype("<u4").tobytes())
            b = pylibsort.sortPartial(buf, off, w)
            np.testing.assert_array_equal(np.frombuffer(buf, dtype=np.uint32),
                                          v["partial_%d_%d_%d" % (n, off, w)])
            np.testing.assert_array_equal(np.array(b, dtype=np.uint32), v["bounds_%d_%d_%d" % (n, off, w)])
            pylibsort.checkPartial(v["in_%d" % n].tobytes(), bytes(buf), b, off, w)


def test_reference_boundaries_mode(dev, oracle_mod, golden):
    """libsortSetBoundaryMode(1): gpuPartial returns the reference
    GetBoundaries output bit for bit, quirk included (sort.cu:367-394; the
    oracle's restatement), on the survey's quirk cases and on inputs with
    group 1 empty; mode 0 (default) keeps the exclusive prefix."""
    import pylibsort
    g, _ = golden
    L = pylibsort.lib()
    rng = np.random.default_rng(9)
    cases = [(np.array(c["input"], dtype=np.uint32), c["offset"], c["width"]) for c in g["boundary_quirk_cases"]]
    for n, w in ((1021, 8), (5000, 4), (77, 6)):
        x = rng.integers(0, 1 << w, n, dtype=np.uint64).astype(np.uint32)
        x[(x & ((1 << w) - 1)) <= 1] |= 2                            # groups 0 and 1 empty
        cases.append((x, 0, w))
    cases.append((oracle_mod.pcg(1111), 0, 8))                       # group 1 non-empty: modes agree
    prev = L.libsortSetBoundaryMode(1)
    try:
        for x, off, w in cases:
            buf = bytearray(x.tobytes())
            b = pylibsort.sortPartial(buf, off, w)
            d, _ = oracle_mod.partial_u32(x, off, w)
            np.testing.assert_array_equal(np.frombuffer(buf, dtype=np.uint32), d)
            np.testing.assert_array_equal(np.array(b, dtype=np.uint32), oracle_mod.ref_boundaries(d, off, w))
    finally:
        L.libsortSetBoundaryMode(prev)
    x, off, w = cases[0]
    b = pylibsort.sortPartial(bytearray(x.tobytes()), off, w)
    assert b == g["boundary_quirk_cases"][0]["exclusive_prefix"]


def test_host_abi_edge_cases(dev):
    import pylibsort
    L = pylibsort.lib()
    buf = bytearray()
    pylibsort.sortFull(buf)  # len 0 is a no-op
    assert pylibsort.sortPartial(bytearray(), 0, 4) == [0] * 16
    x = (np.arange(10, dtype=np.uint32) * 7)[::-1].copy()
    import ctypes
    bnd = (ctypes.c_uint32 * 1)()
    assert L.gpuPartial(x.ctypes.data, ctypes.addressof(bnd), 10, 0, 32) == 0  # width 32 rejected
    assert L.gpuPartial(x.ctypes.data, ctypes.addressof(bnd), 10, 30, 4) == 0  # offset+width > 32
    assert L.providedGpu(x.ctypes.data, (1 << 32) + 1) == 0  # len > UINT32_MAX (checked first)
    assert L.initLibSort() == 0  # second init fails, as in the reference
    assert L.gpuFullSort(x.ctypes.data, 10) == 1
    np.testing.assert_array_equal(x, np.sort(np.arange(10, dtype=np.uint32) * 7))


def test_host_abi_concurrent_callers(dev, oracle_mod):
    # 16 concurrent full + 16 partial sorts through the device pool
    # (benchmark/pkg/sort/libsort_test.go:35-87 TestParallel)
    import concurrent.futures as cf
    import pylibsort
    inputs = [oracle_mod.pcg(4099 + i, first=i * 5000) for i in range(32)]

    def work(i):
        buf = bytearray(inputs[i].tobytes())
        if i % 2 == 0:
            pylibsort.sortFull(buf)
            return np.array_equal(np.frombuffer(buf, dtype=np.uint32), np.sort(inputs[i]))
        b = pylibsort.sortPartial(buf, 0, 8)
        d, bb = oracle_mod.partial_u32(inputs[i], 0, 8)
        return np.array_equal(np.frombuffer(buf, dtype=np.uint32), d) and np.array_equal(b, bb)

    with cf.ThreadPoolExecutor(16) as ex:
        assert all(ex.map(work, range(32)))


@pytest.mark.parametrize("kind", ["pcg", "ragged", "equal", "narrow", "heavy_bucket", "sorted", "reverse"])
def test_host_full_sort_pipelined(dev, oracle_mod, kind):
    """providedGpu at >= 2^22 keys takes the pipelined path (chunked H2D with
    per-chunk range partition, per-range gather + sort + D2H): bit-identical
    to std::sort for every distribution, including one where all keys fall
    in one range (no overlap possible) and ragged sizes."""
    import pylibsort
    rng = np.random.default_rng(len(kind))
    n = (1 << 22) + (12345 if kind == "ragged" else 0)
    if kind in ("pcg", "ragged", "sorted", "reverse"):
        x = oracle_mod.pcg(n, first=17)
        if kind == "sorted":
            x = np.sort(x)
        elif kind == "reverse":
            x = np.sort(x)[::-1].copy()
    elif kind == "equal":
        x = np.full(n, 0xDEADBEEF, dtype=np.uint32)
    elif kind == "narrow":
        x = (0x7FF00000 + rng.integers(0, 1 << 19, n)).astype(np.uint32)
    else:  # half the keys in one 12-bit top bucket, the rest uniform
        x = oracle_mod.pcg(n, first=99)
        x[: n // 2] = (0x12300000 + rng.integers(0, 1 << 20, n // 2)).astype(np.uint32)
    buf = bytearray(x.tobytes())
    pylibsort.sortFull(buf)
    np.testing.assert_array_equal(np.frombuffer(buf, dtype=np.uint32), oracle_mod.sort_u32(x))


def test_host_full_sort_pipelined_concurrent(dev, oracle_mod):
    """Concurrent large providedGpu callers share the device's workspace."""
    import concurrent.futures as cf
    import pylibsort
    xs = [oracle_mod.pcg((1 << 22) + 1000 * i, first=i << 24) for i in range(4)]

    def work(i):
        buf = bytearray(xs[i].tobytes())
        pylibsort.sortFull(buf)
        return np.array_equal(np.frombuffer(buf, dtype=np.uint32), oracle_mod.sort_u32(xs[i]))

    with cf.ThreadPoolExecutor(4) as ex:
        assert all(ex.map(work, range(4)))


def test_reference_localtest_harness(dev):
    # The reference's own localTest runTests (tests.cpp:88-161: gpuPartial,
    # providedGpu, providedCpu, distribSort with two concurrent gpuPartial
    # callers, cross-checks), compiled from the reference sources against
    # this libsort.so (oracle/Makefile).
    import pathlib
    exe = pathlib.Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "localtest_conformance"
    if not exe.exists():
        pytest.skip("oracle/_ref/localtest_conformance was not built (reference absent at build time)")
    r = subprocess.run([str(exe), "1111", "1021", "4099", "65536", "1000003"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Success!") == 5


@pytest.mark.slow
def test_reference_size_full_sort_sha(dev, golden, digit_bits):
    # C2 input: 2^28 PCG keys; the reference's own sha256 of the sorted array
    g, _ = golden
    n = 1 << 28
    x = dev.populate_u32(n)
    s_in = hashlib.sha256(x.cpu().numpy().view("<u4").tobytes()).hexdigest()[:16]
    assert s_in == g["sha256_prefix"][str(n)]["input"]
    out = dev.sort_keys_u32(x)
    torch.cuda.synchronize()
    host = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(host.tobytes()).hexdigest()[:16] == g["sha256_prefix"][str(n)]["sorted"]
    assert int(np.count_nonzero(host[1:] == host[:-1])) == g["sha256_prefix"][str(n)]["duplicate_keys"]


def _big_golden():
    import json
    import pathlib
    return json.loads((pathlib.Path(__file__).resolve().parent / "golden" / "big_golden.json").read_text())


def _device_sha256(t, np_dtype, chunk=1 << 27):
    """sha256 of a device tensor's little-endian bytes, copied in chunks."""
    h = hashlib.sha256()
    for i in range(0, t.numel(), chunk):
        h.update(t[i:i + chunk].cpu().numpy().view(np_dtype).astype(np_dtype.newbyteorder("<")).tobytes())
    return h.hexdigest()


def _device_sorted_and_checksums(x, out):
    """Size-independent parity at configs too large for the host oracle:
    out is non-decreasing as uint32 and holds the same multiset as x
    (sum and sum of squares of the keys, mod 2^64)."""
    flip = torch.tensor(-(1 << 31), dtype=torch.int32, device=out.device)
    s = torch.bitwise_xor(out, flip)              # uint32 order -> int32 order
    ok = True
    chunk = 1 << 26
    for i in range(0, out.numel() - 1, chunk):
        a = s[i:i + chunk + 1]
        ok &= bool((a[1:] >= a[:-1]).all())
    def sums(t):
        tot, sq = 0, 0
        for i in range(0, t.numel(), chunk):
            v = t[i:i + chunk].to(torch.int64) & 0xFFFFFFFF
            tot += int(v.sum())
            sq += int((v * v).sum())                  # int64 wrap = mod 2^64
        return tot % (1 << 64), sq % (1 << 64)
    return ok, sums(x) == sums(out)


@pytest.mark.parametrize("digit", [8, 4])
@pytest.mark.parametrize("width", [8, 16])
def test_partial_reference_size(dev, width, digit):
    """The reference's own benchmark workload (localTest/benchmarks.cpp:38-51,
    212-215 -> gpuPartialProfile(first 2^28 PCG keys, offset 0, width 16);
    analysis/libsort8b.csv is the same call at width 8), through both forms:
    the device-resident libsortSortKeysU32(..., d_boundaries) and the host
    ABI gpuPartial on a pageable buffer.  Parity: sha256 of the data and of
    the 2^width boundaries equal to the oracle's stable counting partition of
    the same keys (tests/golden/big_golden.json "partial_u32", which
    make_big_golden.py also checked against the exact emulation of the
    reference's Step kernels and GetBoundaries)."""
    import ctypes
    import pylibsort
    n = 1 << 28
    g = _big_golden()["partial_u32"]["%d/0/%d" % (n, width)]
    prev = pylibsort.setDigitBits(digit)
    try:
        x = dev.populate_u32(n)
        b = torch.empty(1 << width, dtype=torch.int32, device="cuda")
        out = dev.sort_keys_u32(x, offset=0, width=width, boundaries=b)
        torch.cuda.synchronize()
        assert pylibsort.lib().libsortDeviceErrors() == 0
        assert _device_sha256(out, np.dtype(np.uint32)) == g["data"]
        hb = _u32(b)
        assert list(hb[:4]) == g["boundaries_head"] and list(hb[-4:]) == g["boundaries_tail"]
        assert hashlib.sha256(hb.astype("<u4").tobytes()).hexdigest() == g["boundaries"]
        del out
        host = x.cpu().numpy().view(np.uint32).copy()
        del x
        bnd = (ctypes.c_uint32 * (1 << width))()
        assert pylibsort.lib().gpuPartial(host.ctypes.data, ctypes.addressof(bnd), n, 0, width) == 1, \
            pylibsort.last_error()
        assert hashlib.sha256(host.astype("<u4").tobytes()).hexdigest() == g["data"]
        assert hashlib.sha256(np.frombuffer(bnd, dtype=np.uint32).astype("<u4").tobytes()).hexdigest() == \
            g["boundaries"]
    finally:
        pylibsort.setDigitBits(prev)
        torch.cuda.empty_cache()


@pytest.mark.parametrize("bits", [8, 4])
def test_config3_2pow30(dev, bits):
    # C3: 2^30 keys of the PCG stream (device skip-ahead), full sort on one GPU
    import pylibsort
    prev = pylibsort.setDigitBits(bits)
    try:
        n = 1 << 30
        x = dev.populate_u32(n)
        out = dev.sort_keys_u32(x)
        torch.cuda.synchronize()
        assert pylibsort.lib().libsortDeviceErrors() == 0
        ok, same = _device_sorted_and_checksums(x, out)
        assert ok and same
        # bit-exact: the oracle's std::sort of the same stream (big_golden.json)
        assert _device_sha256(out, np.dtype(np.uint32)) == _big_golden()["sorted_u32"][str(n)]
    finally:
        pylibsort.setDigitBits(prev)


@pytest.mark.parametrize("bits", [8, 4])
def test_maximum_size(dev, bits):
    """n = 2^32 - 1 keys, the largest the ABI accepts: 32-bit run offsets up to
    the last tile (whose next-tile index wraps), 2^19 / 2^20 tiles.  The keys
    are the PCG stream; parity: sha256 of the output equal to the oracle's
    std::sort of the same stream (tests/golden/big_golden.json)."""
    import pylibsort
    if torch.cuda.get_device_properties(0).total_memory < (80 << 30):
        pytest.skip("needs ~64 GiB of device memory")
    prev = pylibsort.setDigitBits(bits)
    try:
        n = (1 << 32) - 1
        x = dev.populate_u32(n)
        out = dev.sort_keys_u32(x)
        torch.cuda.synchronize()
        assert pylibsort.lib().libsortDeviceErrors() == 0
        del x
        assert _device_sha256(out, np.dtype(np.uint32)) == _big_golden()["sorted_u32"][str(n)]
    finally:
        pylibsort.setDigitBits(prev)
        torch.cuda.empty_cache()


@pytest.mark.parametrize("bits", [8, 4])
def test_config5_pairs_size(dev, bits):
    """C5's per-GPU share as one sort: 2^28 (u64 key, u32 payload) pairs with
    the bench's keys (two consecutive PCG draws) and payload = index.  Parity:
    sha256 of keys and payloads equal to std::stable_sort of the same pairs
    (tests/golden/big_golden.json), plus the properties (keys non-decreasing,
    payloads increasing inside runs of equal keys)."""
    import pylibsort
    prev = pylibsort.setDigitBits(bits)
    try:
        n = 1 << 28
        w = dev.populate_u32(2 * n).view(n, 2).to(torch.int64)
        keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
        del w
        keys[: n // 64] = keys[: n // 64] & 0x7FF                  # many equal keys (stability matters)
        vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32)
        ok_, ov = dev.sort_pairs_u64_u32(keys, vals)
        torch.cuda.synchronize()
        assert pylibsort.lib().libsortDeviceErrors() == 0
        flip = torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")
        s = torch.bitwise_xor(ok_, flip)
        v = ov.to(torch.int64) & 0xFFFFFFFF
        chunk = 1 << 25
        for i in range(0, n - 1, chunk):
            a, b = s[i:i + chunk + 1], v[i:i + chunk + 1]
            assert bool((a[1:] >= a[:-1]).all())
            eq = a[1:] == a[:-1]
            assert bool((b[1:][eq] > b[:-1][eq]).all())

        def mix(k, p):
            return (((k & 0xFFFFFF) * 1000003 + (k >> 40) * 7 + p) % 1000000007).sum()
        assert int(mix(keys, vals.to(torch.int64) & 0xFFFFFFFF)) == int(mix(ok_, v))
        # bit-exact: std::stable_sort of the same pairs (big_golden.json)
        g = _big_golden()["c5_pairs"][str(n)]
        assert _device_sha256(ok_, np.dtype(np.uint64)) == g["keys"]
        assert _device_sha256(ov, np.dtype(np.uint32)) == g["payloads"]
    finally:
        pylibsort.setDigitBits(prev)
        torch.cuda.empty_cache()


def _delta_pack_ref(x):
    """numpy/Python restatement of the delta-coded run format (libsort.h):
    per 64-key group the first key, then 64 gaps of w bits packed little-endian
    at bit lane * w (lane 0's gap is 0)."""
    n = x.size
    ng = -(-n // 64)
    gaps = [0]
    for g in range(ng):
        seg = x[g * 64:(g + 1) * 64].astype(np.int64)
        gaps.append(int(np.diff(seg).max()) if seg.size > 1 else 0)
    w = max(gaps).bit_length()
    words = [int(x[g * 64]) for g in range(ng)]
    for g in range(ng):
        seg = x[g * 64:(g + 1) * 64].astype(np.int64)
        d = np.concatenate([[0], np.diff(seg)]) if seg.size else np.zeros(0, np.int64)
        acc = 0
        for lane, v in enumerate(d):
            acc |= int(v) << (lane * w)
        words += [(acc >> (32 * q)) & 0xFFFFFFFF for q in range(2 * w)]
    return max(gaps), w, np.array(words, dtype=np.uint32)


@pytest.mark.parametrize("kind,n", [("uniform", 1), ("uniform", 63), ("uniform", 64), ("uniform", 65),
                                    ("uniform", 100003), ("equal", 5000), ("wide", 4097), ("clustered", 70001),
                                    ("dups", 20000)])
def test_delta_code_roundtrip(dev, kind, n):
    """Delta-coded runs (the msdz exchange): the largest gap, the coded words
    (pinned to a Python restatement of the format) and the decode round trip."""
    import pylibsort.device as D
    rng = np.random.default_rng(n)
    if kind == "uniform":
        x = np.sort(rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
    elif kind == "equal":
        x = np.full(n, 0xDEADBEEF, dtype=np.uint32)
    elif kind == "wide":
        x = np.sort(np.concatenate([[0, 0xFFFFFFFF], rng.integers(0, 1 << 32, n - 2, dtype=np.uint64)])
                    .astype(np.uint32))
    elif kind == "clustered":
        x = np.sort((rng.integers(0, 8, n, dtype=np.uint64) << np.uint64(29)
                     | rng.integers(0, 1000, n, dtype=np.uint64)).astype(np.uint32))
    else:
        x = np.sort(rng.integers(0, 300, n, dtype=np.uint64).astype(np.uint32))
    t = torch.from_numpy(x.view(np.int32)).cuda()
    mg = D.delta_maxgap_u32(t)
    maxgap, w, ref = _delta_pack_ref(x)
    assert int(mg.item()) & 0xFFFFFFFF == maxgap
    assert D.delta_bits(maxgap) == w and D.delta_words(n, w) == ref.size
    coded = D.delta_pack_u32(t, mg, out=torch.empty(ref.size, dtype=torch.int32, device="cuda"))
    np.testing.assert_array_equal(coded.cpu().numpy().view(np.uint32), ref)
    back = D.delta_unpack_u32(coded, n, w)
    np.testing.assert_array_equal(back.cpu().numpy().view(np.uint32), x)
    # into a destination 1..3 words past 16-byte alignment (the rounds decode
    # at arbitrary key offsets; the aligned case takes 16-byte stores)
    for off in (1, 2, 3):
        buf = torch.full((n + off,), -1, dtype=torch.int32, device="cuda")
        D.delta_unpack_u32(coded, n, w, out=buf[off:])
        got = buf.cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(got[off:], x)
        assert (got[:off] == 0xFFFFFFFF).all()


@pytest.mark.parametrize("na,nb", [(0, 0), (0, 5), (7, 0), (1, 1), (2048, 2048), (100003, 77777), (5, 300000),
                                   (1 << 20, (1 << 20) + 13)])
def test_merge_u32(dev, na, nb):
    import pylibsort.device as D
    rng = np.random.default_rng(na * 7 + nb)
    hi = 1000 if na == 2048 else 1 << 32                      # ties across the runs
    a = np.sort(rng.integers(0, hi, na, dtype=np.uint64).astype(np.uint32))
    b = np.sort(rng.integers(0, hi, nb, dtype=np.uint64).astype(np.uint32))
    ta = torch.from_numpy(a.view(np.int32)).cuda()
    tb = torch.from_numpy(b.view(np.int32)).cuda()
    out = D.merge_u32(ta, tb)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), np.sort(np.concatenate([a, b])))


def test_host_word_wait_fallback(oracle_mod):
    """The hybrid's host waits (wait_host_word, radix_kernels.hip) poll a
    pinned word a kernel raises; past LIBSORT_HOST_WAIT_MS they synchronise
    the stream and re-check instead.  With the limit at 0 every
    wait longer than a few hundred polls takes that branch; a full sort (the
    hybrid: sampler + bucket-stat words) and a piece sort (the multi-GPU
    rounds' entry point) are queued behind a 2^28-key sort so their words
    arrive late.  Fresh process; exact against the oracle."""
    import os
    import pathlib
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = pathlib.Path(__file__).resolve().parents[1]
    code = r"""
import sys, numpy as np, torch
sys.path[:0] = [%r, %r]
import pylibsort.device as D
from oracle import oracle
big = D.populate_u32(1 << 28)
x = oracle.pcg((1 << 27) + 4097, first=11)
t = torch.from_numpy(x.view(np.int32)).cuda()
o1 = D.sort_keys_u32(big)      # queued ahead: the next sorts' words arrive late
o2 = D.sort_keys_u32(t)
xs = x[np.argsort(x >> np.uint32(24), kind="stable")]  # pieces: the keys grouped by top digit
cnt = np.bincount(x >> np.uint32(24), minlength=256).astype(np.uint64)
off = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
o3 = D.sort_pieces_u32(torch.from_numpy(xs.view(np.int32)).cuda(), off, cnt, np.arange(256, dtype=np.uint32), 256, 24)
torch.cuda.synchronize()
want = oracle.sort_u32(x)
assert np.array_equal(o2.cpu().numpy().view(np.uint32), want), "full sort"
assert np.array_equal(o3.cpu().numpy().view(np.uint32), want), "piece sort"
print("OK")
""" % (str(root), str(root / "gpu-radix-sort_amd"))
    env = dict(os.environ, LIBSORT_HOST_WAIT_MS="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
