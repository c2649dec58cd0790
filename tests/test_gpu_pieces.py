"""GPU parity of the pre-partitioned sort (libsortSortPiecesU32, the
receive side of the multi-GPU top-digit rounds): the keys of one round arrive
as pieces (source rank r, top digit g), laid out source-major in the receive
buffer, and are sorted straight from those pieces (the MSD hybrid's depth-0
tiles come from the piece table; no gather copy).  Checked bit-exact against
the oracle's std::sort on rounds cut the way distrib.py cuts them, on skewed
inputs (both fallbacks: the gather + LSD sort after depth 0, the LSD sort of
the output when buckets overflow), with empty pieces and empty segments, at
both digit widths and in auto mode."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def D():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pylibsort
    import pylibsort.device as D
    assert pylibsort.gpu_ready(), pylibsort.last_error()
    return D


@pytest.fixture(params=[4, 8], ids=["digit4", "digit8"])
def bits(request, D):
    import pylibsort
    prev = pylibsort.setDigitBits(request.param)
    yield request.param
    pylibsort.setDigitBits(prev)


@pytest.fixture(params=["force", "auto"])
def mode(request, D):
    import pylibsort
    prev = pylibsort.setHybrid(request.param)
    yield request.param
    pylibsort.setHybrid(prev)


def _round(x, R, a, b, shift=24, seed=0):
    """The receive buffer of one round: keys of x whose top digit (x >> shift)
    lies in [a, b), dealt to R sources, each source's keys partitioned by
    digit (stable) and the sources laid out one after another.  Returns
    (buffer, off, len, seg) with the pieces listed segment-major,
    source-minor."""
    rng = np.random.default_rng(seed)
    d = (x >> np.uint32(shift)).astype(np.int64)
    keep = x[(d >= a) & (d < b)]
    src = rng.integers(0, R, keep.size)
    parts, pieces = [], {}
    pos = 0
    for s in range(R):
        ks = keep[src == s]
        ds = (ks >> np.uint32(shift)).astype(np.int64)
        order = np.argsort(ds, kind="stable")
        ks, ds = ks[order], ds[order]
        for g in range(a, b):
            m = int((ds == g).sum())
            pieces[(g, s)] = (pos, m)
            pos += m
        parts.append(ks)
    buf = np.concatenate(parts) if parts else np.empty(0, np.uint32)
    off, ln, sg = [], [], []
    for g in range(a, b):
        for s in range(R):
            o, m = pieces[(g, s)]
            off.append(o)
            ln.append(m)
            sg.append(g - a)
    return buf, np.array(off, np.uint64), np.array(ln, np.uint64), np.array(sg, np.uint32)


def _sort(D, buf, off, ln, sg, nseg, b):
    t = torch.from_numpy(np.ascontiguousarray(buf).view(np.int32)).cuda()
    out = D.sort_pieces_u32(t, off, ln, sg, nseg, b)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,R,a,b", [(1 << 20, 8, 40, 48), ((1 << 22) + 17, 8, 0, 9), ((1 << 21) + 5, 3, 250, 256),
                                     (5000, 2, 3, 5), (1 << 22, 1, 100, 101), ((1 << 20) + 1, 4, 0, 256)])
def test_round_pieces(D, oracle_mod, bits, mode, n, R, a, b):
    x = oracle_mod.pcg(n, first=n + a)
    buf, off, ln, sg = _round(x, R, a, b, seed=R)
    got = _sort(D, buf, off, ln, sg, b - a, 24)
    np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))


@pytest.mark.parametrize("kind", ["low_skew", "equal", "dups", "one_digit", "empty_segments"])
def test_skewed_rounds(D, oracle_mod, bits, kind):
    """Inputs the hybrid must hand to a fallback (or survive): all keys of a
    digit in one 12-bit prefix (buckets overflow), all-equal keys, few
    distinct keys, one populated digit of many, empty segments between."""
    import pylibsort
    prev = pylibsort.setHybrid("force")
    try:
        n = (1 << 21) + 3
        x = oracle_mod.pcg(n, first=7)
        a, b = 16, 24
        if kind == "low_skew":
            x = (x & np.uint32(0xFFF00FFF)) | np.uint32(0x00055000)
        elif kind == "equal":
            x = np.full(n, 0x12345678, dtype=np.uint32)
            a, b = 0x12, 0x13
        elif kind == "dups":
            x = (np.random.default_rng(1).integers(0, 7, n, dtype=np.uint64).astype(np.uint32) << np.uint32(20)) | \
                np.uint32(0x10000000)
        elif kind == "one_digit":
            x = (x & np.uint32(0x00FFFFFF)) | np.uint32(20 << 24)
        else:
            x = x & np.uint32(0xF7FFFFFF)  # bit 27 clear: of digits 16..31 only 16..23 populated
            a, b = 16, 32
        buf, off, ln, sg = _round(x, 5, a, b, seed=3)
        got = _sort(D, buf, off, ln, sg, b - a, 24)
        np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))
    finally:
        pylibsort.setHybrid(prev)


def test_segments_of_other_widths(D, oracle_mod, bits, mode):
    """Segments fixed by the top 12 bits (bits = 20) and by the top 4 bits
    (bits = 28); pieces in arbitrary offsets of the buffer."""
    n = (1 << 21) + 99
    x = oracle_mod.pcg(n, first=11)
    for shift, a, b in ((20, 1000, 1040), (28, 3, 9)):
        buf, off, ln, sg = _round(x, 6, a, b, shift=shift, seed=shift)
        got = _sort(D, buf, off, ln, sg, b - a, shift)
        np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))


def test_bad_tables_fail_loudly(D):
    import pylibsort
    t = torch.zeros(100, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError):  # segments out of order
        D.sort_pieces_u32(t, [0, 50], [50, 50], [1, 0], 2, 24)
    with pytest.raises(RuntimeError):  # segment >= nseg
        D.sort_pieces_u32(t, [0], [100], [2], 2, 24)
    assert "libsortSortPiecesU32" in pylibsort.last_error()
    out = D.sort_pieces_u32(t, [], [], [], 1, 24)  # nothing to sort
    assert out.numel() == 0


def _digits_round(oracle_mod, n, R, a, b, seed):
    """A round whose every key lies in the top digits [a, b), uniform below:
    segments large enough for two or more digit passes."""
    rng = np.random.default_rng(seed)
    x = (oracle_mod.pcg(n, first=seed) & np.uint32(0x00FFFFFF)) | \
        (rng.integers(a, b, n, dtype=np.uint64).astype(np.uint32) << np.uint32(24))
    return _round(x, R, a, b, seed=seed)


def _sort_timed(D, buf, off, ln, sg, nseg, b):
    D.timing_enable(True)
    D.timing_reset()
    try:
        got = _sort(D, buf, off, ln, sg, nseg, b)
        return got, D.timing_query("rsvsample")[0], D.timing_query("bucketsort")[0]
    finally:
        D.timing_enable(False)


@pytest.mark.parametrize("reserve", ["0", "1"])
@pytest.mark.parametrize("nseg,n", [(1, (1 << 21) + 5), (5, (1 << 22) + 3), (8, (1 << 23) + 1), (16, (1 << 23) + 5),
                                    (31, (1 << 23) + 7),
                                    (40, (1 << 23) + 9)])
def test_reserved_depth0_pieces(D, oracle_mod, monkeypatch, reserve, nseg, n):
    """The piece sort's reserved depth 0 (4-bit digits; the round sorts of the
    multi-GPU schedule): no count pass, the depth-0 pass reserves each run in
    a slice per (segment, digit, range) sized by 32768 (<= 8 segments),
    65536 (16) or 131072 (31) samples per range, taken by global key rank
    through the piece table.  Up to 4096 slices (31 segments); 40 segments
    keep the count pass.  Exact; which depth 0
    ran is read from the timing registry."""
    import pylibsort
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", reserve)
    prev = pylibsort.setDigitBits(4)
    try:
        buf, off, ln, sg = _digits_round(oracle_mod, n, 8, 100, 100 + nseg, seed=nseg)
        got, nsample, nbs = _sort_timed(D, buf, off, ln, sg, nseg, 24)
        np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))
        assert nbs == 1
        assert nsample == (1 if reserve == "1" and nseg * 16 * 8 <= 4096 else 0), nsample
    finally:
        pylibsort.setDigitBits(prev)


def test_reserved_depth0_pieces_digit8(D, oracle_mod, monkeypatch):
    """8-bit digits: 2 segments x 256 digits x 8 ranges = 4096 slices."""
    import pylibsort
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", "1")
    prev = pylibsort.setDigitBits(8)
    try:
        buf, off, ln, sg = _digits_round(oracle_mod, (1 << 23) + 3, 4, 7, 9, seed=2)
        got, nsample, nbs = _sort_timed(D, buf, off, ln, sg, 2, 24)
        np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))
        assert nsample == 1 and nbs == 1
    finally:
        pylibsort.setDigitBits(prev)


@pytest.mark.parametrize("reserve", ["short", "nomem"])
def test_reserved_depth0_pieces_fallbacks(D, oracle_mod, monkeypatch, reserve):
    """Slices at half their sampled capacity (a depth-0 tile finds its slice
    full: the piece sort gathers and LSD-sorts from the untouched pieces), and
    an allocation that fails (the count pass instead)."""
    import pylibsort
    monkeypatch.setenv("LIBSORT_HYB_RESERVE", reserve)
    prev = pylibsort.setDigitBits(4)
    try:
        buf, off, ln, sg = _digits_round(oracle_mod, (1 << 23) + 1, 8, 40, 48, seed=9)
        got, nsample, nbs = _sort_timed(D, buf, off, ln, sg, 8, 24)
        np.testing.assert_array_equal(got, oracle_mod.sort_u32(buf))
        assert (nsample, nbs) == ((1, 0) if reserve == "short" else (0, 1)), (nsample, nbs)
    finally:
        pylibsort.setDigitBits(prev)
