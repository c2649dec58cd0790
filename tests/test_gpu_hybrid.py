"""GPU parity of the MSD hybrid (sort_hybrid_u32: digit passes from the top
digit down over segment-aligned tiles, then every bucket of keys sharing the
top 16 bits sorted on chip), through the C ABI, against the oracle.

The hybrid serves full 32-bit sorts of 2^27 .. 2^28 + 2^24 keys; "force"
mode (libsortSetHybrid(2)) runs it for every full sort of >= 1024 keys, so
ragged sizes, skewed and duplicate-heavy inputs are checked at sizes the
oracle sorts in a moment.  Both fallbacks are covered: a skewed top digit
abandons the hybrid after the first column scan (LSD sort of the untouched
input), and buckets larger than a block are finished by an LSD sort of the
output in place.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pylibsort
    import pylibsort.device as D
    assert pylibsort.gpu_ready(), pylibsort.last_error()
    return D


@pytest.fixture(params=[4, 8], ids=["digit4", "digit8"])
def bits(request, dev):
    import pylibsort
    prev = pylibsort.setDigitBits(request.param)
    yield request.param
    pylibsort.setDigitBits(prev)


@pytest.fixture
def force(dev):
    import pylibsort
    prev = pylibsort.setHybrid("force")
    yield
    pylibsort.setHybrid(prev)


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def _tensor(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda()


def _sort_counting_buckets(dev, *args, **kw):
    """dev.sort_keys_u32 with the per-kernel timing registry on: returns the
    output and how many bucket-sort launches (the hybrid's last step) ran."""
    out, nbs, _ = _sort_counting(dev, *args, **kw)
    return out, nbs


def _sort_counting(dev, *args, **kw):
    """... and how many digit passes ran (16 / bits when the hybrid needed no
    fallback)."""
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        out = dev.sort_keys_u32(*args, **kw)
        torch.cuda.synchronize()
        return out, dev.timing_query("bucketsort")[0], dev.timing_query("tilepass")[0]
    finally:
        dev.timing_enable(False)


def _inputs(kind, n, seed):
    import oracle.oracle as o
    x = o.pcg(n, first=seed)
    rng = np.random.default_rng(seed)
    if kind == "pcg":
        return x
    if kind == "top_skew":        # keys < 2^30: 4 of 16 top digits -> hybrid abandoned
        return x >> 2
    if kind == "deep_skew":       # top digit uniform, bits 16-27 zero -> buckets overflow
        return x & np.uint32(0xF000FFFF)
    if kind == "equal":
        return np.full(n, 0x9E3779B9, dtype=np.uint32)
    if kind == "four":
        return rng.integers(0, 4, n, dtype=np.uint64).astype(np.uint32) * np.uint32(0x40000001)
    if kind == "sorted":
        return np.sort(x)
    if kind == "reverse":
        return np.sort(x)[::-1].copy()
    if kind == "low16_const":     # every bucket all-equal keys
        return x & np.uint32(0xFFFF0000)
    if kind == "top16_dense":     # ~16 keys per bucket at 2^20
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("n", [1024, 1025, 4097, 65539, (1 << 20) + 3, (1 << 22) + 5])
def test_hybrid_forced_sizes(dev, oracle_mod, bits, force, n):
    x = oracle_mod.pcg(n, first=5 * n + bits)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 1


@pytest.mark.parametrize("kind", ["top_skew", "deep_skew", "equal", "four", "sorted", "reverse", "low16_const"])
def test_hybrid_forced_distributions(dev, oracle_mod, bits, force, kind):
    n = (1 << 22) + 17
    x = _inputs(kind, n, 11 + bits)
    out = dev.sort_keys_u32(_tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


def test_hybrid_forced_in_place(dev, oracle_mod, bits, force):
    x = oracle_mod.pcg((1 << 21) + 9, first=77)
    t = _tensor(x)
    tmp = torch.empty_like(t)
    dev.sort_keys_u32(t, out=t, tmp=tmp)
    np.testing.assert_array_equal(_u32(t), oracle_mod.sort_u32(x))


def test_hybrid_forced_host_abi(dev, oracle_mod, bits, force):
    import pylibsort
    x = oracle_mod.pcg(300007, first=91)
    buf = bytearray(x.tobytes())
    pylibsort.sortFull(buf)
    np.testing.assert_array_equal(np.frombuffer(buf, dtype=np.uint32), oracle_mod.sort_u32(x))


@pytest.mark.parametrize("n", [1 << 27, (1 << 27) + 12345, (1 << 28) + (1 << 24) - 3])
def test_hybrid_auto_large(dev, oracle_mod, bits, n):
    """The sizes the auto mode serves (the 2^28 reference hash is in
    test_gpu_parity.test_reference_size_full_sort_sha): PCG keys sorted on
    the device, sha256 against the oracle's counting-sort restatement."""
    import hashlib
    x = dev.populate_u32(n, first=n % 1000)
    out, nbs, npass = _sort_counting(dev, x)
    assert nbs == 1
    assert npass == 16 // bits, "uniform keys must not need the LSD fallback"
    h = hashlib.sha256()
    for i in range(0, n, 1 << 26):
        h.update(out[i:i + (1 << 26)].cpu().numpy().view("<u4").tobytes())
    assert h.hexdigest() == oracle_mod.sorted_pcg_sha256(n, first=n % 1000)


def test_hybrid_auto_skewed_large(dev, oracle_mod, bits):
    """2^27 keys that overflow the buckets (the bits below the top digit
    down to bit 16 zero): the planning of the last depth sees the bucket
    sizes, the bucket sort is not launched and the LSD sort of the output
    finishes; and a skewed top digit (keys < 2^30) abandons the hybrid after
    its first pass (which wrote only tmp)."""
    n = 1 << 27
    x = dev.populate_u32(n, first=3)
    for mask_kind in ("deep", "top"):
        if mask_kind == "deep":
            # the top digit uniform, the bits below it down to bit 16 zero
            mask = 0xF000FFFF if bits == 4 else 0xFF00FFFF
            y = torch.bitwise_and(x, torch.tensor(mask - (1 << 32), dtype=torch.int32, device=x.device))
        else:
            y = torch.bitwise_and(torch.bitwise_right_shift(x, 2), 0x3FFFFFFF)
        out, nbs, npass = _sort_counting(dev, y)
        assert nbs == 0
        assert npass == (16 // bits if mask_kind == "deep" else 1) + 32 // bits
        host = y.cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(host))


@pytest.mark.parametrize("lo,width", [(0x12300000, 27), (0, 24), (0xFFF00000, 20), (7, 31)])
@pytest.mark.parametrize("n", [4099, (1 << 21) + 11])
def test_hybrid_forced_range_sorts(dev, oracle_mod, bits, force, lo, width, n):
    """Range-restricted sorts (libsortSortKeysRangeU32: keys in [lo, lo +
    2^width), the multi-GPU round sorts) take the hybrid over the width bits
    of key - lo: digit passes over the top 16 of them, buckets sorted on the
    rest (pads lo - 1)."""
    hi = lo + (1 << width)
    x = (oracle_mod.pcg(n, first=n + width).astype(np.uint64) % (hi - lo) + lo).astype(np.uint32)
    x[:5] = [lo, hi - 1, lo, hi - 1, lo + 1]
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        out = dev.sort_keys_range_u32(_tensor(x), lo, hi)
        torch.cuda.synchronize()
        nbs = dev.timing_query("bucketsort")[0]
    finally:
        dev.timing_enable(False)
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 1


def test_hybrid_auto_range_large(dev, oracle_mod, bits):
    """The size of a multi-GPU round sort at 8 GPUs (2^27 keys spanning
    2^27 values): the auto mode takes the hybrid."""
    import hashlib
    n, lo = 1 << 27, 0x40000000
    x = dev.populate_u32(n, first=5)
    y = torch.bitwise_or(torch.bitwise_and(x, (1 << 27) - 1), lo)
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        out = dev.sort_keys_range_u32(y, lo, lo + (1 << 27))
        torch.cuda.synchronize()
        nbs = dev.timing_query("bucketsort")[0]
    finally:
        dev.timing_enable(False)
    assert nbs == 1
    host = y.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(host))


@pytest.mark.parametrize("frac", [0.55, 0.9])
def test_hybrid_auto_range_partial_span(dev, oracle_mod, bits, frac):
    """A round of the 8-GPU sort: 2^27 + 2^23 keys spanning frac * 2^27 values
    (the round's share of the key space is no power of two, so W = 27 bits
    of key - lo are sorted but only frac of their top digits and 16-bit
    prefixes occur).  The hybrid must size its skew check and buckets by the
    span and run without a fallback (it used to take the populated top
    digits for skew, run the LSD sort after its first pass and waste it)."""
    n, lo = (1 << 27) + (1 << 23), 0x20000000
    span = int(frac * (1 << 27))
    x = dev.populate_u32(n, first=9)
    y = (((x.to(torch.int64) & 0xFFFFFFFF) * span >> 32) + lo).to(torch.int32)
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        out = dev.sort_keys_range_u32(y, lo, lo + span)
        torch.cuda.synchronize()
        nbs, npass = dev.timing_query("bucketsort")[0], dev.timing_query("tilepass")[0]
    finally:
        dev.timing_enable(False)
    assert nbs == 1
    assert npass == 16 // bits, "a partial span must not look skewed"
    host = y.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(host))


def _pairs_counting(dev, kt, vt):
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        ok_, ov = dev.sort_pairs_u64_u32(kt, vt)
        torch.cuda.synchronize()
        return ok_, ov, dev.timing_query("bucketsort")[0], dev.timing_query("tilepass")[0]
    finally:
        dev.timing_enable(False)


@pytest.fixture
def bits8(dev):
    import pylibsort
    prev = pylibsort.setDigitBits(8)
    yield 8
    pylibsort.setDigitBits(prev)


KINDS64 = ["uniform", "dups", "top_skew", "deep_skew", "equal", "runs", "long_runs"]


def _keys64(kind, n):
    """64-bit key sets for the hybrid: uniform; few distinct values; skewed
    top digit (abandons); skewed second byte (oversized buckets); all equal;
    runs of keys sharing their top 32 bits (the bucket sort's tie fix-up:
    insertion-sorted runs, and past 64 keys the reload with every step)."""
    rng = np.random.default_rng(n + len(kind))
    k = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    if kind == "dups":
        k = rng.integers(0, 1 << 10, n, dtype=np.uint64) * np.uint64(0x0040000100000001)
    elif kind == "top_skew":
        k >>= np.uint64(4)
    elif kind == "deep_skew":
        k &= np.uint64(0xFF00FFFFFFFFFFFF)
    elif kind == "equal":
        k[:] = np.uint64(0x123456789ABCDEF0)
    elif kind == "runs":          # bits 32-47 from 4 values: runs of a quarter bucket
        k = (k & np.uint64(0xFFFF0000FFFFFFFF)) | (rng.integers(0, 4, n, dtype=np.uint64) << np.uint64(32))
    elif kind == "long_runs":     # 4096 buckets, bits 32-47 zero: a run is the whole bucket
        top = rng.integers(0, 4096, n, dtype=np.uint64) * np.uint64(16)
        k = (top << np.uint64(48)) | (k & np.uint64(0xFFFFFFFF))
    return k


@pytest.mark.parametrize("kind", KINDS64)
@pytest.mark.parametrize("n", [1024, 65539, (1 << 21) + 7])
def test_hybrid_forced_pairs_u64_u32(dev, oracle_mod, bits, force, kind, n):
    """(u64 key, u32 payload) pairs (configs[4]'s record) through the hybrid:
    two digit passes over the top 16 key bits, buckets sorted on chip on the
    low 48 bits; stable (payload = input index, ties keep it increasing)."""
    k = _keys64(kind, n)
    v = np.arange(n, dtype=np.uint32)
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    ok_, ov, nbs, _ = _pairs_counting(dev, kt, vt)
    rk, rv = oracle_mod.stable_sort_kv64(k, v)
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint32), rv)
    if kind in ("uniform", "dups", "runs", "long_runs") or (kind == "deep_skew" and n < 1 << 20):
        assert nbs == 1  # (deep_skew at 2^21: buckets of 8192 -> the LSD sort, no bucket sort)


@pytest.mark.parametrize("kind", KINDS64)
@pytest.mark.parametrize("n", [4097, (1 << 21) + 7])
def test_hybrid_forced_pairs_u64_u64(dev, oracle_mod, bits, force, kind, n):
    """(u64 key, u64 payload) pairs through the hybrid, stable."""
    k = _keys64(kind, n)
    v = np.arange(n, dtype=np.uint64) * np.uint64(0x100000001)
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int64)).cuda()
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        ok_, ov = dev.sort_pairs_u64_u64(kt, vt)
        torch.cuda.synchronize()
        nbs = dev.timing_query("bucketsort")[0]
    finally:
        dev.timing_enable(False)
    rk, rv = oracle_mod.stable_sort_kv64v64(k, v)
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint64), rv)
    if kind in ("uniform", "dups", "runs", "long_runs") or (kind == "deep_skew" and n < 1 << 20):
        assert nbs == 1  # (deep_skew at 2^21: buckets of 8192 -> the LSD sort, no bucket sort)


def test_hybrid_auto_pairs_u64_u64_large(dev, oracle_mod, bits8):
    """2^27 (u64, u64) pairs (uniform keys, 1/64 of them repeated) through
    the auto mode: no fallback, equal to the oracle's stable sort."""
    n = 1 << 27
    d = dev.populate_u32(2 * n, first=17).to(torch.int64) & 0xFFFFFFFF
    kt = (d[0::2] << 32) | d[1::2]
    del d
    kt[n // 64: n // 32] = kt[: n // 64]
    vt = torch.arange(n, dtype=torch.int64, device="cuda")
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        ok_, ov = dev.sort_pairs_u64_u64(kt, vt)
        torch.cuda.synchronize()
        nbs, npass = dev.timing_query("bucketsort")[0], dev.timing_query("tilepass")[0]
    finally:
        dev.timing_enable(False)
    assert nbs == 1 and npass == 2, "uniform keys must not need the LSD fallback"
    k = kt.cpu().numpy().view(np.uint64)
    rk, rv = oracle_mod.stable_sort_kv64v64(k, np.arange(n, dtype=np.uint64))
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint64), rv)


@pytest.mark.parametrize("n", [4097, (1 << 21) + 7])
def test_hybrid_forced_keys_u64(dev, oracle_mod, bits, force, n):
    rng = np.random.default_rng(n)
    k = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    k[: n // 5] &= np.uint64(0xFFFF0000FFFF)
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    out = dev.sort_keys_u64(kt)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), oracle_mod.sort_u64(k))


def test_hybrid_auto_pairs_large(dev, oracle_mod, bits):
    """configs[4]'s per-GPU record at 2^27 pairs (key = two consecutive PCG
    draws, payload = index) through the auto mode: no fallback, and equal to
    the oracle's stable sort."""
    n = 1 << 27
    d = dev.populate_u32(2 * n, first=11).to(torch.int64) & 0xFFFFFFFF
    kt = (d[0::2] << 32) | d[1::2]
    vt = torch.arange(n, dtype=torch.int32, device="cuda")
    ok_, ov, nbs, npass = _pairs_counting(dev, kt, vt)
    assert nbs == 1 and npass == 16 // bits
    k = kt.cpu().numpy().view(np.uint64)
    rk, rv = oracle_mod.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint32), rv)



def test_hybrid_forced_second_block(dev, oracle_mod, bits, force):
    """One bucket of 3000 keys (above the first block's slots, within the
    second's): sorted by the second bucket-sort launch, no LSD fallback."""
    n = 1 << 22
    rng = np.random.default_rng(5)
    x = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    x[:3000] = np.uint32(0x12340000) | rng.integers(0, 1 << 16, 3000, dtype=np.uint64).astype(np.uint32)
    out, nbs, npass = _sort_counting(dev, _tensor(x))
    assert nbs == 1
    assert npass == 16 // bits, "a bucket within the second block must not need the LSD fallback"
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


def test_hybrid_forced_second_block_pairs(dev, oracle_mod, bits8, force):
    """The same for stable (u64, u32) pairs (512-thread blocks)."""
    n = 1 << 22
    rng = np.random.default_rng(6)
    k = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2)
    k[:3000] = np.uint64(0x1234 << 48) | (k[:3000] & np.uint64((1 << 48) - 1))
    k[3000:3100] = k[:100]  # equal keys: the payload order must hold
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.arange(n, dtype=torch.int32, device="cuda")
    ok_, ov, nbs, npass = _pairs_counting(dev, kt, vt)
    assert nbs == 1 and npass == 2, "a bucket within the second block must not need the LSD fallback"
    rk, rv = oracle_mod.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(ok_.cpu().numpy().view(np.uint64), rk)
    np.testing.assert_array_equal(ov.cpu().numpy().view(np.uint32), rv)


@pytest.mark.parametrize("n", [1 << 28])
def test_hybrid_auto_bench_size(dev, bits, n):
    """The bench's size (2^28 keys, where ~2 buckets outgrow the first block):
    no LSD fallback, output sorted (checked on the device)."""
    x = dev.populate_u32(n)
    out, nbs, npass = _sort_counting(dev, x)
    assert nbs == 1
    assert npass == 16 // bits, "uniform keys must not need the LSD fallback"
    o = out.view(torch.int32) ^ torch.iinfo(torch.int32).min  # unsigned order as signed
    assert bool((o[1:] >= o[:-1]).all())


def test_hybrid_auto_pairs_bench_size(dev, bits8):
    """configs[4]'s per-GPU share (2^28 pairs, random 64-bit keys, payload =
    index): no LSD fallback; keys sorted and the payloads a permutation that
    follows them (checked on the device)."""
    n = 1 << 28
    d = dev.populate_u32(2 * n, first=3).to(torch.int64) & 0xFFFFFFFF
    kt = (d[0::2] << 32) | d[1::2]
    del d
    vt = torch.arange(n, dtype=torch.int32, device="cuda")
    ok_, ov, nbs, npass = _pairs_counting(dev, kt, vt)
    assert nbs == 1 and npass == 2, "uniform keys must not need the LSD fallback"
    o = ok_ ^ torch.iinfo(torch.int64).min
    assert bool((o[1:] >= o[:-1]).all())
    assert bool((kt[ov.to(torch.int64)] == ok_).all())
    assert bool((torch.sort(ov)[0] == vt).all())


@pytest.mark.parametrize("kind", ["pcg", "low16_const", "four", "top_skew", "deep_skew", "equal"])
@pytest.mark.parametrize("n", [1024, 65539, (1 << 21) + 7])
def test_hybrid_forced_pairs_u32_u32(dev, oracle_mod, bits, force, kind, n):
    """(u32 key, u32 payload) pairs through the hybrid, stable."""
    k = _inputs(kind, n, n + len(kind))
    v = np.arange(n, dtype=np.uint32)
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        ok_, ov = dev.sort_pairs_u32_u32(_tensor(k), _tensor(v))
        torch.cuda.synchronize()
        nbs = dev.timing_query("bucketsort")[0]
    finally:
        dev.timing_enable(False)
    rk, rv = oracle_mod.stable_sort_kv32(k, v)
    np.testing.assert_array_equal(_u32(ok_), rk)
    np.testing.assert_array_equal(_u32(ov), rv)
    if kind in ("pcg", "low16_const"):
        assert nbs == 1


def test_hybrid_auto_pairs_u32_u32_large(dev, oracle_mod, bits):
    """2^27 PCG keys with index payloads through the auto mode: no fallback,
    equal to the oracle's stable sort."""
    n = 1 << 27
    kt = dev.populate_u32(n, first=29)
    vt = torch.arange(n, dtype=torch.int32, device="cuda")
    dev.timing_enable(True)
    dev.timing_reset()
    try:
        ok_, ov = dev.sort_pairs_u32_u32(kt, vt)
        torch.cuda.synchronize()
        nbs, npass = dev.timing_query("bucketsort")[0], dev.timing_query("tilepass")[0]
    finally:
        dev.timing_enable(False)
    assert nbs == 1 and npass == 16 // bits, "uniform keys must not need the LSD fallback"
    rk, rv = oracle_mod.stable_sort_kv32(_u32(kt), np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(_u32(ok_), rk)
    np.testing.assert_array_equal(_u32(ov), rv)


def test_graph_capture_skips_the_host_waits(dev, oracle_mod):
    """Under HIP stream capture a full sort never takes the hybrid (whose two
    host read-backs cannot happen inside a graph): a forced-hybrid
    size captured into a graph by torch.cuda.graph replays to the oracle's
    result."""
    import pylibsort
    x = oracle_mod.pcg((1 << 20) + 77, first=3)
    keys = _tensor(x)
    out = torch.empty_like(keys)
    tmp = torch.empty_like(keys)
    s = torch.cuda.Stream()
    prev = pylibsort.setHybrid("off")
    try:
        with torch.cuda.stream(s):  # warm-up on the capture stream: workspace allocated, same stream
            dev.sort_keys_u32(keys, out=out, tmp=tmp)
        s.synchronize()
        pylibsort.setHybrid("force")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            dev.sort_keys_u32(keys, out=out, tmp=tmp)
        out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    finally:
        pylibsort.setHybrid(prev)


@pytest.mark.parametrize("n", [(1 << 29) + 12345, 400000007])
def test_hybrid_auto_2pow29_class(dev, bits, n):
    """Full sorts of 2^28 + 2^24 .. 2^29 + 2^23 keys take the hybrid with
    the 512-thread bucket blocks (buckets of ~6-8K keys; configs[3]'s 2^29
    keys per GPU): the sha256 of the sorted keys equals the oracle's
    (tests/golden/big_golden.json "sorted_u32_first", made by
    make_big_golden.py from the counting-sort restatement pinned on the
    reference's own hashes), and one bucket-sort launch pair ran."""
    import hashlib
    import json
    import pathlib
    big = json.loads((pathlib.Path(__file__).with_name("golden") / "big_golden.json").read_text())
    x = dev.populate_u32(n, first=n)
    out = torch.empty_like(x)
    tmp = torch.empty_like(x)
    got, nbs, npass = _sort_counting(dev, x, out=out, tmp=tmp)
    assert nbs == 1 and npass == 16 // bits, (nbs, npass)  # 16 / bits digit passes + the bucket sort, no fallback
    h = hashlib.sha256()
    for i in range(0, n, 1 << 26):
        h.update(got[i:i + (1 << 26)].cpu().numpy().view("<u4").tobytes())
    assert h.hexdigest() == big["sorted_u32_first"]["%d@%d" % (n, n)]
    del x, out, tmp
    torch.cuda.empty_cache()


# ---- Reserved depth 0 (keys-only 4-bit sorts: no count pass; the depth-0
# pass reserves its runs in sampled slices) ----

@pytest.fixture
def digit4(dev):
    import pylibsort
    prev = pylibsort.setDigitBits(4)
    yield
    pylibsort.setDigitBits(prev)


@pytest.fixture
def digit8(dev):
    import pylibsort
    prev = pylibsort.setDigitBits(8)
    yield
    pylibsort.setDigitBits(prev)


@pytest.mark.parametrize("reserve", ["0", "1"])
@pytest.mark.parametrize("kind", ["pcg", "sorted", "four", "deep_skew", "low16_const", "reverse"])
@pytest.mark.parametrize("n", [1024, 4097, (1 << 18) + 7, (1 << 22) + 5])
def test_reserved_depth0(dev, oracle_mod, digit4, force, monkeypatch, reserve, kind, n):
    """Ranges of <= 32768 keys are counted exactly (n <= 2^18 here, and the
    empty ranges of a 2-tile input), larger ones sampled; both depth-0 forms
    give the oracle's output."""
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", reserve)
    x = _inputs(kind, n, 11 * n + 3)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


@pytest.mark.parametrize("n", [(1 << 22) + 5, (1 << 23) + 1])
def test_reserved_depth0_overflow_falls_back(dev, oracle_mod, digit4, force, monkeypatch, n):
    """Slices at half their sampled capacity (LIBSORT_HYB_RESERVE=short; sampled
    ranges, > 32768 keys each, since capacities are whole tiles): the
    depth-0 tiles that find their slice full write nothing and raise the
    flag, the later depths do nothing, and the LSD sort of the untouched input
    runs instead (no bucket sort)."""
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "short")
    x = oracle_mod.pcg(n, first=n + 99)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 0
    # the next sort on the same workspace is unaffected
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "1")
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 1


@pytest.mark.parametrize("reserve", ["0", "1"])
@pytest.mark.parametrize("kind", ["pcg", "sorted", "four", "low16_const"])
@pytest.mark.parametrize("n", [1024, 8193, (1 << 20) + 7, (1 << 23) + 5])
def test_reserved_depth0_digit8(dev, oracle_mod, digit8, force, monkeypatch, reserve, kind, n):
    """8-bit digits: 2048 slices (256 digits x 8 ranges), 131072 samples per
    range (ranges of <= 131072 keys counted exactly); the next depth's counts
    are read from its (compacted) tile table."""
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", reserve)
    x = _inputs(kind, n, 13 * n + 1)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


def test_reserved_depth0_digit8_overflow_falls_back(dev, oracle_mod, digit8, force, monkeypatch):
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "short")
    n = (1 << 26) + 1  # slices of ~32K keys: half of it, in whole 8192-key tiles, is short
    x = oracle_mod.pcg(n, first=n + 7)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 0


def test_reserved_depth0_range_sort(dev, oracle_mod, digit4, force, monkeypatch):
    """Range sorts (keys in [lo, lo + span)) take the reserved depth 0 too."""
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "1")
    n = (1 << 21) + 9
    lo = 0x12345678
    x = (oracle_mod.pcg(n, first=77) % np.uint32(0x5000000)) + np.uint32(lo)
    out = dev.sort_keys_range_u32(_tensor(x), lo, lo + 0x5000000)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))


def test_reserved_depth0_nomem_falls_back(dev, oracle_mod, digit4, force, monkeypatch):
    """The slices cannot be allocated (LIBSORT_HYB_RESERVE=nomem acts as a
    failed allocation): depth 0 takes the count pass and the hybrid still
    runs to its bucket sort (the sort must not fail)."""
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "nomem")
    n = (1 << 22) + 5
    x = oracle_mod.pcg(n, first=n + 3)
    out, nbs = _sort_counting_buckets(dev, _tensor(x))
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
    assert nbs == 1


@pytest.mark.parametrize("four", [False, True], ids=["low16_const", "low16_four"])
def test_counting_bucket_duplicates_full_size(dev, oracle_mod, bits, four):
    """Duplicate-heavy keys at the bench size (2^28, auto mode): every 16-bit
    bucket holds ~4096 keys of one (or four) values, so the counting
    placement's counts overflow in every bucket and the bucket is sorted by
    the LSD steps instead (no per-cell search, whose cost grew
    with the square of the cell).  Exact: f(x) = high 16 bits of x, plus (four)
    its bits 14-15 as the low bits, is monotone, so sort(f(x)) == f(sort(x)),
    and sort(x) is pinned by the oracle's hash.  Timed against the uniform
    sort: within 3x (the quadratic search was ~100x)."""
    import hashlib
    import time
    n = 1 << 28
    x = dev.populate_u32(n, first=0)
    ref = dev.sort_keys_u32(x)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for i in range(0, n, 1 << 26):
        h.update(ref[i:i + (1 << 26)].cpu().numpy().view("<u4").tobytes())
    assert h.hexdigest() == oracle_mod.sorted_pcg_sha256(n, first=0)
    def f(t):
        y = t & -65536  # the high 16 bits
        return (y | ((t & 0xC000) >> 14)) if four else y
    xm = f(x)
    out = torch.empty_like(x)
    tmp = torch.empty_like(x)

    def timed(t):
        dev.sort_keys_u32(t, out=out, tmp=tmp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            dev.sort_keys_u32(t, out=out, tmp=tmp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3

    t_dup = timed(xm)
    assert torch.equal(out, f(ref))
    t_uni = timed(x)
    assert t_dup < 3.0 * t_uni, (t_dup, t_uni)
    del x, xm, ref, out, tmp
    torch.cuda.empty_cache()


def test_counting_bucket_overflow_classes(dev, oracle_mod, bits):
    """One 2^27-key sort whose buckets take every route of the counting
    placement at once: uniform buckets (2-bit cells; the ~4% with a value of
    4+ keys retry with 3-bit cells), buckets given one value of 6 keys (a
    light overflow: the 3-bit retry), buckets made of 2 values (heavy: straight
    to the LSD-step list), and buckets over the first block (~3.2K keys where
    the mean is 2048: they join the retry list at the second size).  Exact
    against the oracle."""
    n = (1 << 27) + 77
    rng = np.random.default_rng(27)
    import oracle.oracle as o
    x = o.pcg(n, first=27)
    nb = 1 << 16
    pos = rng.permutation(n)
    cur = 0

    def take(k):
        nonlocal cur
        p = pos[cur:cur + k]
        cur += k
        return p
    pref = rng.permutation(nb).astype(np.uint32)
    # light: 6 keys of one value in each of 1500 buckets
    for b in pref[:1500]:
        x[take(6)] = (b << 16) | np.uint32(rng.integers(0, 1 << 16))
    # heavy: 2000 keys of 2 values in each of 40 buckets (their own keys
    # spread over random buckets)
    for b in pref[1500:1540]:
        own = np.nonzero((x >> 16) == b)[0]
        x[own] = (x[own] & np.uint32(0xFFFF)) | (rng.integers(0, nb, own.size).astype(np.uint32) << 16)
        v = (b << 16) | np.uint32(rng.integers(0, 1 << 16))
        x[take(2000)] = np.where(rng.random(2000) < 0.5, v, v ^ np.uint32(1)).astype(np.uint32)
    # over the first block (2304 keys at this size; the second holds 3840):
    # 1200 more keys in each of 3 buckets
    for b in pref[1540:1543]:
        x[take(1200)] = (b << 16) | rng.integers(0, 1 << 16, 1200).astype(np.uint32)
    t = _tensor(x)
    out, nbs, npass = _sort_counting(dev, t)
    assert nbs == 1 and npass == 16 // bits
    np.testing.assert_array_equal(_u32(out), oracle_mod.sort_u32(x))
