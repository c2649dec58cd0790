"""The multi-GPU sort behind the C ABI (libsort.h gpuDistribSort /
libsortDistribSortU32, csrc/distrib.cpp) on the one-GPU test box:

- one rank over a real single-process RCCL communicator (ncclCommInitAll of
  one device) with every piece sent through RCCL (LIBSORT_DISTRIB_SELF_RCCL),
  both schedules;
- 2, 3, 5 and 8 ranks sharing the GPU (8 = configs[3]'s world size: 32 (round,
  rank) buckets, 8-way re-cut and LSD segment gathers on the HIP kernels) (device-copy exchanges: RCCL refuses two ranks
  on one GPU), both schedules, ragged and empty shards, duplicate-heavy and
  skewed inputs (the range schedule falls back to the LSD rounds);
- the host-pointer entry point gpuDistribSort against the reference's golden
  sorted hashes.

Parity: the concatenated shards equal std::sort (oracle) bit for bit and
each shard holds ceil(N/R) keys (the reference's re-cut, distrib.go:113);
the LSD schedule's shards equal the reference BSP driver's output shard for
shard (oracle_distrib_bsp_u32)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LSD, COPY, SELF_RCCL, WIRE32, CODED = 1, 2, 4, 8, 16


@pytest.fixture(scope="module")
def D():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pylibsort
    import pylibsort.device as D
    assert pylibsort.gpu_ready(), pylibsort.last_error()
    return D


@pytest.fixture(params=[4, 8], ids=["digit4", "digit8"])
def bits(request):
    import pylibsort
    prev = pylibsort.setDigitBits(request.param)
    yield request.param
    pylibsort.setDigitBits(prev)


def _cut(x, R, ragged=False):
    """R input shards of x (equal, or deliberately ragged with an empty one)."""
    if not ragged:
        S = -(-x.size // R)
        return [x[r * S:(r + 1) * S] for r in range(R)]
    w = np.array([3, 0, 1, 5, 2, 4, 0, 2][:R], dtype=np.float64) + 1e-9
    cuts = np.concatenate([[0], np.round(np.cumsum(w) / w.sum() * x.size).astype(np.int64)])
    cuts[-1] = x.size
    return [x[cuts[r]:cuts[r + 1]] for r in range(R)]


def _run(D, x, R, flags, ragged=False):
    shards = [torch.from_numpy(np.ascontiguousarray(s).view(np.int32)).cuda() for s in _cut(x, R, ragged)]
    outs = D.distrib_sort_u32(shards, flags)
    return [o.cpu().numpy().view(np.uint32) for o in outs]


def _check(oracle, x, outs, R, lsd):
    want = oracle.sort_u32(x)
    S = -(-x.size // R)
    assert [o.size for o in outs] == [max(0, min(x.size, (r + 1) * S) - r * S) for r in range(R)]
    np.testing.assert_array_equal(np.concatenate(outs) if outs else np.empty(0, np.uint32), want)
    if lsd and x.size:
        ref, _ = oracle.distrib_bsp_u32(x, R, 8)
        for r, o in enumerate(outs):
            np.testing.assert_array_equal(o, ref[r * S:(r + 1) * S])


@pytest.mark.parametrize("flags", [SELF_RCCL, SELF_RCCL | LSD, 0, LSD], ids=["rccl-range", "rccl-lsd", "range", "lsd"])
def test_one_rank_over_rccl(D, oracle_mod, bits, flags):
    x = oracle_mod.pcg((1 << 22) + 12345, first=5)
    _check(oracle_mod, x, _run(D, x, 1, flags), 1, flags & LSD)


def _cases(oracle):
    rng = np.random.default_rng(5)
    return {
        "pcg": oracle.pcg((1 << 20) + 4321, first=17),
        "dups": rng.integers(0, 50, 300007, dtype=np.uint64).astype(np.uint32),
        "skewtop": rng.integers(0, 1 << 20, 200003, dtype=np.uint64).astype(np.uint32),  # one top bucket
        "allequal": np.full(100001, 7, dtype=np.uint32),
        "small": oracle.pcg(1111),
        "tiny": oracle.pcg(3, first=2),
    }


@pytest.mark.parametrize("R", [2, 3, 5, 8])
@pytest.mark.parametrize("lsd", [False, True], ids=["range", "lsd"])
@pytest.mark.parametrize("case", ["pcg", "dups", "skewtop", "allequal", "small", "tiny"])
def test_ranks_sharing_the_gpu(D, oracle_mod, R, lsd, case):
    x = _cases(oracle_mod)[case]
    outs = _run(D, x, R, COPY | (LSD if lsd else 0), ragged=(case == "pcg"))
    _check(oracle_mod, x, outs, R, lsd)


def _timed_names(D, fn, *names):
    """Runs fn with the per-kernel timing registry on; returns fn's result and
    the launch count of each named timer."""
    D.timing_enable(True)
    D.timing_reset()
    try:
        out = fn()
        torch.cuda.synchronize()
        return out, [D.timing_query(nm)[0] for nm in names]
    finally:
        D.timing_enable(False)


@pytest.mark.parametrize("R", [3, 8])
@pytest.mark.parametrize("case", ["below2pow26", "offset_narrow", "one_digit_dups"])
def test_range_digit_rounds(D, oracle_mod, R, case):
    """Keys whose top 8 bits take fewer values than there are ranks (below
    2^26 at 8 ranks; a 2^25-wide range at 2^31; 40 values inside one top
    digit): the top-digit plan is too skewed, so the rounds re-partition by
    the 8-bit digit of key - min over the populated range instead of falling
    back to the 4-exchange LSD rounds.  Exact against the oracle;
    the LSD rounds did not run (no "lsdround" launches); at 8 ranks (and for
    the one-digit input at any R) the min/max kernel ran once per rank (at 3
    ranks, 2-4 populated top digits can still give a balanced plan)."""
    rng = np.random.default_rng(R)
    n = (1 << 21) + 77
    if case == "below2pow26":
        x = rng.integers(0, 1 << 26, n, dtype=np.uint64).astype(np.uint32)
    elif case == "offset_narrow":
        x = (rng.integers(0, 1 << 25, n, dtype=np.uint64) + (1 << 31)).astype(np.uint32)
    else:  # 40 distinct values a few apart: shift 0, one value per digit
        x = (rng.integers(0, 40, n, dtype=np.uint64) * 3 + 0x7F000000).astype(np.uint32)
    outs, (nlsd, nmm) = _timed_names(D, lambda: _run(D, x, R, COPY), "lsdround", "minmax")
    _check(oracle_mod, x, outs, R, False)
    assert nlsd == 0 and nmm in (0, R), (nlsd, nmm)
    if R == 8 or case == "one_digit_dups":
        assert nmm == R, nmm


def test_range_digit_all_equal_takes_lsd(D, oracle_mod):
    """One distinct key: no digit splits it, so the LSD rounds run (exact)."""
    x = np.full(300001, 0xDEADBEEF, dtype=np.uint32)
    outs, (nlsd,) = _timed_names(D, lambda: _run(D, x, 4, COPY), "lsdround")
    _check(oracle_mod, x, outs, 4, False)
    assert nlsd > 0


def test_repeated_calls_reuse_the_context(D, oracle_mod):
    """Same ranks, different sizes and inputs back to back (grow-only
    buffers, cached communicator, stream ordering of the workspaces)."""
    for i, n in enumerate([1 << 21, 5000, (1 << 21) + 777, 0, 1 << 16]):
        x = oracle_mod.pcg(n, first=i * 1000)
        _check(oracle_mod, x, _run(D, x, 3, COPY), 3, False)
        _check(oracle_mod, x, _run(D, x, 1, SELF_RCCL), 1, False)


def test_host_entry_point_golden(D, golden):
    import pylibsort
    g, _ = golden
    for n in (1021, 1111, 4099):
        x = pylibsort.lib()
        buf = np.empty(n, dtype=np.uint32)
        # a fresh stream: elements [0, n) by skip-ahead on the device
        buf[:] = D.populate_u32(n).cpu().numpy().view(np.uint32)
        assert hashlib.sha256(buf.tobytes()).hexdigest()[:16] == g["sha256_prefix"][str(n)]["input"]
        assert x.gpuDistribSort(buf.ctypes.data, n, 1) == 1, pylibsort.last_error()
        assert hashlib.sha256(buf.tobytes()).hexdigest()[:16] == g["sha256_prefix"][str(n)]["sorted"]
    # ngpu beyond the pool fails loudly
    buf = np.arange(10, dtype=np.uint32)
    assert pylibsort.lib().gpuDistribSort(buf.ctypes.data, buf.size, 64) == 0
    assert "ngpu" in pylibsort.last_error()


@pytest.mark.slow
def test_reference_size_over_rccl(D, golden, bits):
    """configs[1]'s 2^28 keys through the distributed path (one RCCL rank,
    every piece through RCCL): the reference's sorted sha256.  At 4-bit digits
    the keys cross RCCL as 24-bit planes (the default wire format), at 8-bit
    as 32-bit words."""
    import pylibsort
    g, _ = golden
    n = 1 << 28
    x = D.populate_u32(n)
    out = D.distrib_sort_u32([x], SELF_RCCL)[0]
    h = hashlib.sha256(out.cpu().numpy().view(np.uint32).tobytes()).hexdigest()[:16]
    assert h == g["sha256_prefix"][str(n)]["sorted"]
    assert pylibsort.lib().libsortDeviceErrors() == 0


@pytest.mark.parametrize("R", [1, 3, 8])
@pytest.mark.parametrize("n", [(1 << 21) + 333, (1 << 23) + 77])
def test_wire24(D, oracle_mod, R, n):
    """24-bit keys on the wire: the partition scatter
    writes each key's low 16 bits and bits 16..23 as two planes, the rounds
    move 3 bytes per key, and the round sorts' reserved depth 0 (or, for
    rounds below 2^20 keys, the unpacking gather) rebuilds the key with the
    piece's digit as its top byte.  Exact against the oracle at both wire
    formats; every rank's exchange bytes are exactly 3/4 of the 32-bit
    format's (R = 1: every piece through one RCCL rank, nothing counted)."""
    import pylibsort
    prev = pylibsort.setDigitBits(4)
    try:
        x = oracle_mod.pcg(n, first=9)
        flags = SELF_RCCL if R == 1 else COPY
        o24 = _run(D, x, R, flags)
        b24 = D.distrib_last_bytes(R)
        o32 = _run(D, x, R, flags | WIRE32)
        b32 = D.distrib_last_bytes(R)
        _check(oracle_mod, x, o24, R, False)
        _check(oracle_mod, x, o32, R, False)
        if R > 1:
            assert sum(b32) > 0 and all(4 * a == 3 * b for a, b in zip(b24, b32)), (b24, b32)
        assert pylibsort.lib().libsortDeviceErrors() == 0
    finally:
        pylibsort.setDigitBits(prev)


@pytest.mark.parametrize("R", [1, 2, 3, 8])
@pytest.mark.parametrize("case", ["pcg", "dups", "skewtop", "allequal", "small", "tiny"])
def test_coded_rounds(D, oracle_mod, bits, R, case):
    """The gap-coded rounds (LIBSORT_DISTRIB_CODED; VERDICT r05 item 2: the
    torch engine's msdz in the C engine): every sender sorts its outgoing
    pieces, codes them as gaps, the receiver decodes and merges R runs.  R = 1
    sends every coded piece through a one-rank RCCL communicator; R > 1 shares
    the GPU (device copies).  Exact against the oracle, shards of ceil(N/R);
    skewed inputs take the range digit or the LSD rounds as without coding."""
    x = _cases(oracle_mod)[case]
    flags = (SELF_RCCL if R == 1 else COPY) | CODED
    _check(oracle_mod, x, _run(D, x, R, flags, ragged=(case == "pcg")), R, False)


@pytest.mark.parametrize("R", [2, 4])
def test_coded_rounds_bytes(D, oracle_mod, R):
    """The coded exchange's bytes (libsortDistribLastBytes counts the coded
    words): for 2^23 uniform keys well under half the 32-bit format's -- the
    gap width is ~log2(2^32 R K / n) + 2 bits -- and exact against the oracle
    with and without the stage trace."""
    import pylibsort
    x = oracle_mod.pcg((1 << 23) + 3, first=21)
    o32 = _run(D, x, R, COPY | WIRE32)
    b32 = D.distrib_last_bytes(R)
    oz = _run(D, x, R, COPY | CODED)
    bz = D.distrib_last_bytes(R)
    _check(oracle_mod, x, o32, R, False)
    _check(oracle_mod, x, oz, R, False)
    assert all(0 < z < 0.5 * w for z, w in zip(bz, b32)), (bz, b32)
    L = pylibsort.lib()
    prev = L.libsortSetDistribTrace(1)
    try:
        _check(oracle_mod, x, _run(D, x, R, COPY | CODED), R, False)
    finally:
        L.libsortSetDistribTrace(prev)
    assert pylibsort.lib().libsortDeviceErrors() == 0


@pytest.mark.parametrize("reserve", ["on", "nomem"])
def test_wire24_reserved_depth0_odd_offsets(D, oracle_mod, reserve):
    """Three ranks, 2^26 + 77 keys: rounds of 4-7M keys over <= 32 segments
    (two digit depths below the top digit), so the round sorts read the 24-bit
    planes through the reserved depth 0's
    planar loader, at round offsets (and 8-bit plane starts 2 n_recv + a) that
    are not multiples of 4 (the loader aligns on the absolute
    address).  reserve=nomem: the reserved depth 0 is unavailable, so the
    rounds take the unpacking gather and then the range sort of their span
    (not a 32-bit LSD sort).  Exact against the oracle."""
    import os
    import pylibsort
    prev = pylibsort.setDigitBits(4)
    old = os.environ.get("LIBSORT_HYB_RESERVE")
    if reserve == "nomem":
        os.environ["LIBSORT_HYB_RESERVE"] = "nomem"
    try:
        x = oracle_mod.pcg((1 << 26) + 77, first=11)
        outs, (nrsv, nseg) = _timed_names(D, lambda: _run(D, x, 3, COPY), "rsvsample", "segcopy")
        _check(oracle_mod, x, outs, 3, False)
        if reserve == "on":
            assert nrsv > 0, nrsv
        else:
            assert nrsv == 0 and nseg > 0, (nrsv, nseg)
        assert pylibsort.lib().libsortDeviceErrors() == 0
    finally:
        if old is None:
            os.environ.pop("LIBSORT_HYB_RESERVE", None)
        else:
            os.environ["LIBSORT_HYB_RESERVE"] = old
        pylibsort.setDigitBits(prev)


@pytest.mark.slow
def test_shape8_2pow29(D):
    """configs[3]'s per-rank size in the 8-GPU shape (2^29 keys of the stream
    >> 3: the keys of 32 top digits, as one of 8 ranks receives them; round
    sorts of 8 segments of ~2^24 keys, the reserved depth 0 of the piece sort)
    through one RCCL rank with every piece through RCCL: the oracle's sha256
    (big_golden.json "sorted_u32_shift", monotone map of the pinned sorted
    stream).  Reference: localTest/tests.cpp:137-143 (GPU == CPU)."""
    import json
    import pathlib
    big = json.loads((pathlib.Path(__file__).with_name("golden") / "big_golden.json").read_text())
    n = 1 << 29
    x = D.populate_u32(n)
    x >>= 3
    x &= 0x1FFFFFFF  # (a logical shift: the tensor is int32)
    out = D.distrib_sort_u32([x], SELF_RCCL)[0]
    del x
    h = hashlib.sha256()
    for i in range(0, n, 1 << 26):
        h.update(out[i:i + (1 << 26)].cpu().numpy().view("<u4").tobytes())
    assert h.hexdigest() == big["sorted_u32_shift"]["%d>>3" % n]
    del out
    torch.cuda.empty_cache()


def _pair_case(oracle, case):
    rng = np.random.default_rng(len(case))
    if case == "c5":            # configs[4]'s pairs: key = draw 2i << 32 | draw 2i+1
        w = oracle.pcg(2 * ((1 << 20) + 333), first=3).astype(np.uint64)
        return (w[0::2] << np.uint64(32)) | w[1::2]
    if case == "ties":          # equal keys spread over every rank (stability across ranks)
        return rng.integers(0, 1 << 12, 300007, dtype=np.uint64) * np.uint64(0x0010000100000001)
    if case == "onekey":
        return np.full(100003, 0x123456789ABCDEF0, dtype=np.uint64)
    if case == "below2pow40":   # IDs: every key in top digit 0 (range partition)
        return rng.integers(0, 1 << 40, 400009, dtype=np.uint64)
    if case == "stamps":        # ns timestamps of one day: one shared top byte, ties included
        return np.uint64(0x17A0000000000000) + rng.integers(0, 86400 * 10**9, 400009, dtype=np.uint64) // np.uint64(1000)
    return rng.integers(0, 1 << 63, 5, dtype=np.uint64)  # tiny: empty shards at 8 ranks


@pytest.mark.parametrize("R", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("case", ["c5", "ties", "onekey", "tiny", "below2pow40", "stamps"])
def test_pairs_engine(D, oracle_mod, bits, R, case):
    """configs[4] behind the C ABI (libsortDistribSortPairsU64U32): one RCCL
    rank with every piece through RCCL, or R ranks sharing the GPU; the
    concatenated shards equal std::stable_sort by key of (key, input index)
    -- payloads of equal keys in input order across ranks -- and each shard
    holds ceil(N/R) pairs."""
    k = _pair_case(oracle_mod, case)
    n = k.size
    v = np.arange(n, dtype=np.uint32)
    S = -(-n // R)
    ks = [torch.from_numpy(k[r * S:(r + 1) * S].view(np.int64).copy()).cuda() for r in range(R)]
    vs = [torch.from_numpy(v[r * S:(r + 1) * S].view(np.int32).copy()).cuda() for r in range(R)]
    ko, vo = D.distrib_sort_pairs_u64_u32(ks, vs, SELF_RCCL if R == 1 else COPY)
    rk, rv = oracle_mod.stable_sort_kv64(k, v)
    assert [t.numel() for t in ko] == [max(0, min(n, (r + 1) * S) - r * S) for r in range(R)]
    np.testing.assert_array_equal(np.concatenate([t.cpu().numpy().view(np.uint64) for t in ko]), rk)
    np.testing.assert_array_equal(np.concatenate([t.cpu().numpy().view(np.uint32) for t in vo]), rv)


@pytest.mark.parametrize("case", ["below2pow40", "stamps"])
def test_pairs_range_digit(D, oracle_mod, case):
    """Pair keys below 2^56 or sharing their top byte: the top-digit plan
    would send every pair to one rank, so the engine re-partitions by the
    8-bit digit over the populated key range (the min/max kernel runs once
    per rank); exact and stable against the oracle.  (The balance itself is
    host arithmetic, checked in tests/cpp/distrib_sim.cpp.)"""
    R = 4
    k = _pair_case(oracle_mod, case)
    n = k.size
    v = np.arange(n, dtype=np.uint32)
    S = -(-n // R)
    ks = [torch.from_numpy(k[r * S:(r + 1) * S].view(np.int64).copy()).cuda() for r in range(R)]
    vs = [torch.from_numpy(v[r * S:(r + 1) * S].view(np.int32).copy()).cuda() for r in range(R)]
    (ko, vo), (nmm,) = _timed_names(D, lambda: D.distrib_sort_pairs_u64_u32(ks, vs, COPY), "minmax")
    rk, rv = oracle_mod.stable_sort_kv64(k, v)
    np.testing.assert_array_equal(np.concatenate([t.cpu().numpy().view(np.uint64) for t in ko]), rk)
    np.testing.assert_array_equal(np.concatenate([t.cpu().numpy().view(np.uint32) for t in vo]), rv)
    assert nmm == R


def test_pairs_engine_rejects_lsd(D):
    import pylibsort
    k = [torch.zeros(10, dtype=torch.int64, device="cuda")]
    v = [torch.zeros(10, dtype=torch.int32, device="cuda")]
    with pytest.raises(RuntimeError):
        D.distrib_sort_pairs_u64_u32(k, v, LSD)
    assert "keys only" in pylibsort.last_error()


@pytest.mark.slow
def test_config5_share_over_rccl(D):
    """configs[4]'s per-GPU share (2^28 pairs) through the C-ABI pair engine
    over one RCCL rank (every piece through RCCL): the oracle's sha256 of the
    stably sorted keys and payloads (tests/golden/big_golden.json)."""
    import hashlib
    import json
    import pathlib
    big = json.loads((pathlib.Path(__file__).with_name("golden") / "big_golden.json").read_text())
    n = 1 << 28
    want = big["c5_pairs"][str(n)]
    w = D.populate_u32(2 * n).view(n, 2).to(torch.int64)
    keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
    del w
    keys[: n // 64] = keys[: n // 64] & 0x7FF  # the pinned input (test_gpu_parity.test_config5_pairs_size)
    vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32)
    ko, vo = D.distrib_sort_pairs_u64_u32([keys], [vals], SELF_RCCL)
    del keys, vals

    def sha(t, dt):
        h = hashlib.sha256()
        for i in range(0, t.numel(), 1 << 26):
            h.update(t[i:i + (1 << 26)].cpu().numpy().view(dt).tobytes())
        return h.hexdigest()
    assert sha(ko[0], np.uint64) == want["keys"]
    assert sha(vo[0], np.uint32) == want["payloads"]


@pytest.mark.parametrize("parts", ["2", "1"], ids=["two-parts", "one-part"])
def test_threaded_round_issue(oracle_mod, parts):
    """The multi-device issue path of the C engine (one host thread per
    device sorting round i as soon as round i's exchange is issued) on the
    one-GPU box, forced by LIBSORT_DISTRIB_THREADS=1 in a fresh process: one
    RCCL rank, 3 ranks sharing the GPU, keys and pairs, against the oracle.
    parts: the ranks' partition in two parts (the default with R > 1: the
    first part's pieces of rounds 0 and 1 go before the second part is
    written) or, LIBSORT_DISTRIB_PARTS=1, in one."""
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
x = oracle.pcg((1 << 22) + 999, first=4)
for R, flags in ((1, 4), (3, 2), (2, 2 | 16), (3, 2 | 16)):
    S = -(-x.size // R)
    sh = [torch.from_numpy(x[r * S:(r + 1) * S].view(np.int32).copy()).cuda() for r in range(R)]
    outs = D.distrib_sort_u32(sh, flags)
    got = np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs])
    assert np.array_equal(got, oracle.sort_u32(x)), R
    if flags & 16:
        continue  # (the coded rounds are for keys only)
    k = (x.astype(np.uint64) << np.uint64(32)) | x.astype(np.uint64)[::-1]
    v = np.arange(x.size, dtype=np.uint32)
    ks = [torch.from_numpy(k[r * S:(r + 1) * S].view(np.int64).copy()).cuda() for r in range(R)]
    vs = [torch.from_numpy(v[r * S:(r + 1) * S].view(np.int32).copy()).cuda() for r in range(R)]
    ko, vo = D.distrib_sort_pairs_u64_u32(ks, vs, flags)
    rk, rv = oracle.stable_sort_kv64(k, v)
    assert np.array_equal(np.concatenate([t.cpu().numpy().view(np.uint64) for t in ko]), rk), R
    assert np.array_equal(np.concatenate([t.cpu().numpy().view(np.uint32) for t in vo]), rv), R
print("OK")
""" % (str(root), str(root / "gpu-radix-sort_amd"))
    env = dict(os.environ, LIBSORT_DISTRIB_THREADS="1", LIBSORT_DISTRIB_PARTS=parts)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("lsd", [False, True], ids=["rounds", "lsd"])
def test_stage_trace(D, oracle_mod, capfd, lsd):
    """libsortSetDistribTrace(1) (LIBSORT_DISTRIB_TRACE=1): the engine names
    every stage on stderr -- the partition, the plan, each round's exchange
    issue, its arrival and sort on every rank, the re-cut, the end -- so a
    multi-GPU run that hangs shows where.  The traced sort
    is still exact."""
    import re
    import pylibsort
    L = pylibsort.lib()
    prev = L.libsortSetDistribTrace(1)
    try:
        x = oracle_mod.pcg((1 << 21) + 5, first=3)
        capfd.readouterr()
        outs = _run(D, x, 4, COPY | (LSD if lsd else 0))
        err = capfd.readouterr().err
    finally:
        L.libsortSetDistribTrace(prev)
    _check(oracle_mod, x, outs, 4, lsd)
    lines = [ln for ln in err.splitlines() if ln.startswith("libsort distrib [")]
    text = "\n".join(lines)
    assert re.search(r"sort u32: 4 ranks on 1 devices, exchanges by device/peer copies", text), text
    assert "done: ok" in text, text
    if lsd:
        for step in range(4):
            assert "lsd step %d: exchange issued" % step in text, text
    else:
        assert "partition (top digit, 24-bit planes, 1 part)" in text or "partition (top digit, 1 part)" in text, text
        assert "plan: 4 rounds per rank" in text, text
        for i in range(4):
            assert "round %d: exchange issued" % i in text, text
            for r in range(4):
                assert re.search(r"round %d rank %d: arrived" % (i, r), text), text
        assert "re-cut" in text, text
    # stamps non-decreasing
    ms = [float(re.match(r"libsort distrib \[\s*([0-9.]+) ms\]", ln).group(1)) for ln in lines]
    assert ms == sorted(ms)
    # tracing off: silent
    capfd.readouterr()
    _run(D, x, 4, COPY)
    assert "libsort distrib [" not in capfd.readouterr().err


def test_engine_streams_overlap(D, oracle_mod):
    """in the C engine's driving process -- torch's
    streams in use, libsort's workspace streams, the engine's compute (st) and
    communication (cs) streams and RCCL's communicator (a one-rank RCCL sort
    first) -- a spinning kernel on st and one on cs run at the same time, so
    with the box's GPU_MAX_HW_QUEUES = 4 the two streams are not multiplexed
    onto one in-order hardware queue (where an RCCL kernel waiting for its
    peer on cs would hold the round sorts on st)."""
    import ctypes
    import os
    import pylibsort
    x = D.populate_u32(1 << 22)                       # torch's stream
    D.sort_keys_u32(x)                                # libsort's workspace stream
    torch.cuda.synchronize()
    xs = oracle_mod.pcg((1 << 20) + 7, first=2)
    _check(oracle_mod, xs, _run(D, xs, 1, SELF_RCCL), 1, False)  # the engine's streams + RCCL's
    ms = (ctypes.c_double * 4)()
    devs = (ctypes.c_int * 1)(0)
    assert pylibsort.lib().libsortDistribOverlapProbe(1, devs, 20000, ms) == 1, pylibsort.last_error()
    st0, st1, cs0, cs1 = list(ms)
    print("GPU_MAX_HW_QUEUES=%s st [%.3f, %.3f] ms, cs [%.3f, %.3f] ms" % (
        os.environ.get("GPU_MAX_HW_QUEUES"), st0, st1, cs0, cs1))
    assert st1 - st0 > 15.0 and cs1 - cs0 > 15.0, list(ms)   # both spun ~20 ms
    assert cs0 < st1 - 10.0 and st0 < cs1 - 10.0, list(ms)   # the windows overlap
