"""The oracle (CPU restatement) pinned against the reference's own outputs
(tests/golden/pcg_golden.json, recorded from the reference utils.cu /
std::sort) and against an exact emulation of the reference kernels."""
import hashlib

import numpy as np
import pytest


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u4").tobytes()).hexdigest()[:16]


def test_pcg_first_words_and_persistence(oracle_mod, golden):
    g, _ = golden
    p = oracle_mod.Pcg()
    first = p.take(8)
    assert [format(int(v), "08x") for v in first] == g["fresh_process_first_words"]
    nxt = p.take(4)  # the state persists across populateInput calls (utils.cu:67)
    assert [format(int(v), "08x") for v in nxt] == g["next_call_words_after_8"]


@pytest.mark.parametrize("n", ["1021", "1111", "4099", "1048576"])
def test_pcg_and_sort_sha_match_reference(oracle_mod, golden, n):
    g, _ = golden
    x = oracle_mod.pcg(int(n))
    assert sha16(x) == g["sha256_prefix"][n]["input"]
    s = oracle_mod.sort_u32(x)
    assert sha16(s) == g["sha256_prefix"][n]["sorted"]
    if "duplicate_keys" in g["sha256_prefix"][n]:
        assert int(np.count_nonzero(s[1:] == s[:-1])) == g["sha256_prefix"][n]["duplicate_keys"]


def test_pcg_reference_size_input_sha(oracle_mod, golden):
    g, _ = golden
    x = oracle_mod.pcg(1 << 28)
    assert sha16(x) == g["sha256_prefix"]["268435456"]["input"]


def test_bucket_facts_from_survey(oracle_mod, golden):
    g, _ = golden
    for n in ("1021", "1111"):
        x = oracle_mod.pcg(int(n))
        c = np.bincount(x & 0xFF, minlength=256)
        assert int((c == 0).sum()) == g["sha256_prefix"][n]["empty_8bit_buckets"]
        assert int(c[1]) == g["sha256_prefix"][n]["bucket1_count"]


def test_golden_vectors_consistent(oracle_mod, golden):
    _, v = golden
    for n in (1021, 1111, 4099):
        x = v["in_%d" % n]
        np.testing.assert_array_equal(x, oracle_mod.pcg(n))
        np.testing.assert_array_equal(v["sorted_%d" % n], np.sort(x))
        for off, w in ((0, 8), (0, 4), (4, 8), (6, 4)):
            d, b = oracle_mod.partial_u32(x, off, w)
            np.testing.assert_array_equal(v["partial_%d_%d_%d" % (n, off, w)], d)
            np.testing.assert_array_equal(v["bounds_%d_%d_%d" % (n, off, w)], b)


def test_boundary_quirk_cases(oracle_mod, golden):
    g, _ = golden
    for c in g["boundary_quirk_cases"]:
        x = np.array(c["input"], dtype=np.uint32)
        d, b = oracle_mod.partial_u32(x, c["offset"], c["width"])
        assert b.tolist() == c["exclusive_prefix"]
        assert oracle_mod.ref_boundaries(d, c["offset"], c["width"]).tolist() == c["reference"]


def test_reference_boundaries_agree_when_group1_nonempty(oracle_mod):
    # The reference GetBoundaries (sort.cu:367-394) equals the exclusive
    # prefix whenever group 1 is non-empty (always true for the reference's
    # own test inputs).
    for n in (1021, 1111, 4099):
        x = oracle_mod.pcg(n)
        d, b = oracle_mod.partial_u32(x, 0, 8)
        np.testing.assert_array_equal(oracle_mod.ref_boundaries(d, 0, 8), b)


@pytest.mark.parametrize("n,off,w", [(1111, 0, 8), (1021, 4, 8), (300, 6, 4), (4099, 0, 32), (128, 0, 2),
                                     (129, 2, 6), (5000, 10, 12)])
def test_reference_kernel_emulation_is_stable_partition(oracle_mod, n, off, w):
    # exact emulation of the reference 2-bit kernels == stable partition
    x = oracle_mod.pcg(n, first=n)
    ref = oracle_mod.ref_step_u32(x, off, w)
    if w == 32:
        np.testing.assert_array_equal(ref, np.sort(x))
    else:
        np.testing.assert_array_equal(ref, oracle_mod.partial_u32(x, off, w)[0])


def test_reference_odd_width_sorts_an_extra_bit(oracle_mod):
    # sort.cu:323 steps 2 bits at a time: an odd width sorts width+1 bits
    x = oracle_mod.pcg(3001, first=9)
    np.testing.assert_array_equal(oracle_mod.ref_step_u32(x, 0, 5), oracle_mod.partial_u32(x, 0, 6)[0])


def test_distrib_oracles_are_sorts(oracle_mod):
    for n in (1111, 1021, 4099):
        x = oracle_mod.pcg(n)
        np.testing.assert_array_equal(oracle_mod.distrib_local_u32(x, 8), np.sort(x))
        for nw in (1, 2, 3, 5):
            got, lens = oracle_mod.distrib_bsp_u32(x, nw, 8)
            np.testing.assert_array_equal(got, np.sort(x))
            per = -(-n // nw)
            assert lens.tolist() == [min(n, (w + 1) * per) - min(n, w * per) for w in range(nw)]


def test_kv_oracles_are_stable(oracle_mod):
    rng = np.random.default_rng(0)
    k = rng.integers(0, 10, 1000, dtype=np.uint64)
    v = np.arange(1000, dtype=np.uint32)
    kk, vv = oracle_mod.stable_sort_kv64(k, v)
    order = np.lexsort((v, k))
    np.testing.assert_array_equal(kk, k[order])
    np.testing.assert_array_equal(vv, v[order])


def test_u64_oracles_match_numpy(oracle_mod):
    rng = np.random.default_rng(7)
    k = rng.integers(0, 1 << 12, 5000, dtype=np.uint64) << np.uint64(40)
    v = rng.integers(0, 1 << 63, 5000, dtype=np.uint64)
    np.testing.assert_array_equal(oracle_mod.sort_u64(k), np.sort(k))
    idx = np.argsort(k, kind="stable")
    rk, rv = oracle_mod.stable_sort_kv64v64(k, v)
    np.testing.assert_array_equal(rk, k[idx])
    np.testing.assert_array_equal(rv, v[idx])


def test_counting_sort_restatement_pinned(oracle_mod, golden):
    """oracle.sorted_pcg_sha256 (the counting-sort restatement that produced
    tests/golden/big_golden.json for 2^30, 2^32-1 and 2^32 keys) reproduces the
    reference's own sorted hash (pcg_golden.json, recorded from utils.cu +
    std::sort) at 2^20, and agrees with std::sort at an offset."""
    import hashlib
    import json
    import pathlib
    g, _ = golden
    assert oracle_mod.sorted_pcg_sha256(1 << 20)[:16] == g["sha256_prefix"][str(1 << 20)]["sorted"]
    x = oracle_mod.pcg(70001, first=123)
    want = hashlib.sha256(oracle_mod.sort_u32(x).astype("<u4").tobytes()).hexdigest()
    assert oracle_mod.sorted_pcg_sha256(70001, first=123) == want
    big = json.loads((pathlib.Path(__file__).resolve().parent / "golden" / "big_golden.json").read_text())
    # 2^30 (configs[2]), 2^32 - 1 (the ABI maximum), 2^32 (configs[3]'s global input, round 5)
    assert set(big["sorted_u32"]) == {str(1 << 30), str((1 << 32) - 1), str(1 << 32)}
    assert set(big["c5_pairs"][str(1 << 28)]) == {"keys", "payloads"}


def test_partial_reference_workload_golden(oracle_mod, golden):
    """big_golden.json "partial_u32" (the reference's own benchmark call,
    localTest/benchmarks.cpp:38-51,212-215: first 2^28 keys, offset 0) is
    reproduced by the oracle at width 8 from the pinned input stream."""
    import json
    import pathlib
    g, _ = golden
    n = 1 << 28
    x = oracle_mod.pcg(n)
    assert sha16(x) == g["sha256_prefix"][str(n)]["input"]
    big = json.loads((pathlib.Path(__file__).resolve().parent / "golden" / "big_golden.json").read_text())
    assert set(big["partial_u32"]) == {"%d/0/8" % n, "%d/0/16" % n}
    d, b = oracle_mod.partial_u32(x, 0, 8)
    want = big["partial_u32"]["%d/0/8" % n]
    assert hashlib.sha256(d.astype("<u4").tobytes()).hexdigest() == want["data"]
    assert hashlib.sha256(b.astype("<u4").tobytes()).hexdigest() == want["boundaries"]
    assert b[:4].tolist() == want["boundaries_head"]
