"""Multi-rank path on the CPU: world_size 2 and 3 with gloo, local operations
from the oracle backend (tests/distrib_helpers.OracleOps).  Checks the
exchange arithmetic (bucket-major / rank-minor re-cut, alltoallv splits,
segment tables, rebalancing) against the reference's distributed-sort
semantics (benchmark/pkg/sort/distrib.go:90-179; oracle_distrib_bsp_u32)."""
import numpy as np
import pytest

from distrib_helpers import run_ranks, shard_inputs


def _cases():
    from oracle import oracle
    rng = np.random.default_rng(7)
    return {
        "pcg1111": oracle.pcg(1111),
        "pcg40001": oracle.pcg(40001, first=5),
        "dups": rng.integers(0, 50, 30011, dtype=np.uint64).astype(np.uint32),
        "allequal": np.full(9001, 12345, dtype=np.uint32),
        "skewtop": (rng.integers(0, 1 << 20, 20000, dtype=np.uint64).astype(np.uint32)),  # one top bucket
        "tiny": oracle.pcg(2, first=9),                                                    # an empty shard at 3 ranks
    }


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("schedule", ["lsd", "msd", "msdz"])
@pytest.mark.parametrize("case", ["pcg1111", "pcg40001", "dups", "allequal", "skewtop", "tiny"])
def test_distributed_sort_gloo(tmp_path, world, schedule, case):
    from oracle import oracle
    x = _cases()[case]
    port = 29600 + world * 30 + ["lsd", "msd", "msdz"].index(schedule) + 3 * list(_cases()).index(case)
    shards = run_ranks(x, world, schedule, tmp_path, port=port)
    got = np.concatenate(shards)
    np.testing.assert_array_equal(got, oracle.sort_u32(x))
    # shard sizes: the reference's equal re-cut, ceil(N / R) per rank
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]
    if schedule == "lsd":
        # rank r's final shard = the reference BSP driver's STRIDED re-read cut
        ref, _ = oracle.distrib_bsp_u32(x, world, 8)
        for s, r in zip(shards, shard_inputs(ref, world)):
            np.testing.assert_array_equal(s, r)


@pytest.mark.parametrize("world,rounds", [(2, 1), (2, 3), (3, 8), (2, 128)])
def test_msd_rounds_gloo(tmp_path, world, rounds):
    """Range-split rounds: every round count (including rounds with no keys
    and R*K capped at 256 buckets) gives the sorted array and equal shards."""
    from oracle import oracle
    x = oracle.pcg(50021, first=rounds)
    shards = run_ranks(x, world, "msd", tmp_path, port=29700 + 7 * world + rounds % 50, kw={"rounds": rounds})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


def test_msd_larger_input_gloo(tmp_path):
    """600K keys over 2 ranks: every digit populated, 4 rounds of ~16 digits."""
    from oracle import oracle
    x = oracle.pcg(2 * 300007, first=11)
    shards = run_ranks(x, 2, "msd", tmp_path, port=29790, kw={"rounds": 4})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, 2)]


def test_msd_sparse_key_ranges_gloo(tmp_path):
    """Keys in a few narrow ranges: most (rank, round) groups are empty."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.integers(0, 1 << 22, 7000), rng.integers(0xF0000000, 0xF0400000, 9000),
                        rng.integers(0x80000000, 0x80000100, 5000)]).astype(np.uint32)
    rng.shuffle(x)
    shards = run_ranks(x, 3, "msd", tmp_path, port=29795, kw={"rounds": 5, "max_imbalance": 10.0})
    np.testing.assert_array_equal(np.concatenate(shards), np.sort(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, 3)]


@pytest.mark.parametrize("world,rounds,case", [(2, 4, "dups"), (3, 3, "wide"), (2, 1, "wide"), (3, 5, "onekey")])
def test_distrib_pairs_stable_gloo(tmp_path, world, rounds, case):
    """C5 semantics: stable (u64 key, u32 payload) sort across ranks -- payload
    = original global index, so equal keys must keep increasing payloads."""
    from distrib_helpers import run_pair_ranks
    from oracle import oracle
    rng = np.random.default_rng(world * 100 + rounds)
    n = 40013
    if case == "dups":
        k = rng.integers(0, 1 << 10, n, dtype=np.uint64) * np.uint64(0x0040000000100001)  # many equal keys
    elif case == "wide":
        k = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    else:
        k = np.full(n, 0x123456789ABCDEF0, dtype=np.uint64)
    ks, vs = run_pair_ranks(k, world, tmp_path, port=29870 + 10 * world + rounds, kw={"rounds": rounds})
    rk, rv = oracle.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(np.concatenate(ks), rk)
    np.testing.assert_array_equal(np.concatenate(vs), rv)
    S = -(-n // world)
    assert [x.size for x in ks] == [min(n, (r + 1) * S) - min(n, r * S) for r in range(world)]


def _plan_digits_restated(C, R, K, growth):
    """numpy restatement of csrc/distrib_plan.h plan_rounds over the 256 top
    digits (the checker of the one host plan both engines run): digit g's
    middle in rank coordinates x = (cum(g) - G(g)/2) / N * R gives rank
    floor(x); its round is the first i with x - rank < cw[i]; rank * K +
    round made monotone by a cumulative max."""
    G = C.sum(axis=0).astype(np.float64)
    T = max(G.sum(), 1.0)
    x = (np.cumsum(G) - G / 2.0) / T * R
    rank = np.clip(np.floor(x), 0, R - 1).astype(np.int64)
    w, p = [], 1.0
    for _ in range(K):
        w.append(p)
        p *= growth
    cw = np.cumsum(w) / np.sum(w)
    rnd = np.minimum(np.searchsorted(cw, x - rank, side="right"), K - 1)
    grp = np.maximum.accumulate(rank * K + rnd)
    lut = ((grp % K) * R + grp // K).astype(np.uint8)
    est = np.bincount(grp // K, weights=C.sum(axis=0), minlength=R).astype(np.int64)
    return lut, est


@pytest.mark.parametrize("R,K", [(1, 1), (2, 4), (3, 5), (8, 4), (16, 16), (4, 64)])
@pytest.mark.parametrize("kind", ["uniform", "skew", "zero", "sparse"])
def test_digit_plan_c_matches_restatement(R, K, kind):
    """libsortDistribPlanDigits (the host plan sort_msd, sort_msdz, the pair
    rounds and the single-process engine all run) equals the numpy
    restatement; groups are contiguous, monotone and cover every digit."""
    from pylibsort.distrib import plan_digits
    rng = np.random.default_rng(R * 100 + K)
    if kind == "uniform":
        C = rng.integers(0, 100000, (R, 256))
    elif kind == "skew":
        C = rng.integers(0, 3, (R, 256))
        C[:, 77] = 10 ** 9
    elif kind == "zero":
        C = np.zeros((R, 256), dtype=np.int64)
    else:
        C = np.zeros((R, 256), dtype=np.int64)
        C[:, rng.integers(0, 256, 5)] = rng.integers(1, 5000, (R, 5))
    for growth in (1.2, 0.6):
        lut, est = plan_digits(C, R, K, growth)
        lut_ref, est_ref = _plan_digits_restated(C, R, K, growth)
        np.testing.assert_array_equal(lut, lut_ref)
        np.testing.assert_array_equal(est, est_ref)
        grp = (lut.astype(np.int64) % R) * K + lut // R
        assert np.all(np.diff(grp) >= 0) and est.sum() == C.sum()


def test_digit_plan_balanced_rounds_grow():
    from pylibsort.distrib import plan_digits, shard_cut
    rng = np.random.default_rng(4)
    R, K = 8, 4
    C = np.stack([np.bincount(rng.integers(0, 256, 2000000), minlength=256) for _ in range(R)])
    lut, est = plan_digits(C, R, K, 1.2)
    S, _ = shard_cut(int(C.sum()), R)
    assert np.abs(est - S).max() <= C.sum(axis=0).max()        # within one digit of the equal share
    grp = (lut.astype(np.int64) % R) * K + lut // R
    g = np.bincount(grp, weights=C.sum(axis=0), minlength=R * K).reshape(R, K)
    w = 1.2 ** np.arange(K)
    np.testing.assert_allclose(g / g.sum(axis=1, keepdims=True), np.tile(w / w.sum(), (R, 1)), atol=0.04)
    skew = np.zeros((R, 256), dtype=np.int64)
    skew[:, 17] = 1000
    _, est2 = plan_digits(skew, R, K)
    assert est2.max() == skew.sum()  # one digit holds everything -> sort_msd falls back to lsd


def test_shard_cut_matches_reference():
    from pylibsort.distrib import shard_cut
    # distrib.go:113: maxPerWorker = ceil(N / nworker)
    assert shard_cut(1111, 2) == (556, [(0, 556), (556, 1111)])
    assert shard_cut(10, 4)[1] == [(0, 3), (3, 6), (6, 9), (9, 10)]


@pytest.mark.parametrize("world,schedule", [(4, "msd"), (8, "msd"), (4, "lsd")])
def test_msd_bench_world_sizes_gloo(tmp_path, world, schedule):
    """The world sizes of the driver's scaling job (4 and 8 ranks) with the
    bench's default schedule (msd, 4 rounds -> 16 / 32 partition buckets), and
    the reference-semantics lsd schedule (the skew fallback) at 4 ranks."""
    from oracle import oracle
    x = oracle.pcg(8 * 20011, first=world)
    shards = run_ranks(x, world, schedule, tmp_path, port=29900 + world + 20 * (schedule == "lsd"))
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


def test_distrib_pairs_eight_ranks_gloo(tmp_path):
    """C5 at the world size it is quoted on (8 ranks, 4 rounds)."""
    from distrib_helpers import run_pair_ranks
    from oracle import oracle
    rng = np.random.default_rng(88)
    n = 8 * 5003
    k = rng.integers(0, 1 << 12, n, dtype=np.uint64) * np.uint64(0x0010000100000001)
    ks, vs = run_pair_ranks(k, 8, tmp_path, port=29920, kw={"rounds": 4})
    rk, rv = oracle.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(np.concatenate(ks), rk)
    np.testing.assert_array_equal(np.concatenate(vs), rv)


@pytest.mark.parametrize("world,rounds,case", [(2, 4, "pcg"), (2, 1, "dups"), (3, 3, "pcg"), (2, 5, "clustered"),
                                               (4, 2, "pcg")])
def test_msdz_delta_coded_exchange_gloo(tmp_path, world, rounds, case):
    """The delta-coded schedule (sender-side round sorts, coded pieces,
    receiver-side merges): shard for shard equal to the oracle, including
    duplicate-heavy input (zero gaps) and clustered keys (wide gaps)."""
    from oracle import oracle
    rng = np.random.default_rng(world * 10 + rounds)
    if case == "pcg":
        x = oracle.pcg(40009, first=world + rounds)
    elif case == "dups":
        x = rng.integers(0, 1 << 20, 30011, dtype=np.uint64).astype(np.uint32) << np.uint32(12)
    else:
        x = (rng.integers(0, 16, 30011, dtype=np.uint64) << np.uint64(28)
             | rng.integers(0, 5000, 30011, dtype=np.uint64)).astype(np.uint32)
    shards = run_ranks(x, world, "msdz", tmp_path, port=30100 + 13 * world + rounds, kw={"rounds": rounds})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


def test_auto_schedule_gloo(tmp_path):
    """schedule="auto" (the bench default) picks the delta-coded schedule at 2 ranks."""
    from oracle import oracle
    x = oracle.pcg(20011, first=5)
    shards = run_ranks(x, 2, "auto", tmp_path, port=30190)
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))


def _narrow_case(case, n=60013, seed=3):
    rng = np.random.default_rng(seed)
    if case == "below2pow24":      # every key in top digit 0
        return rng.integers(0, 1 << 24, n, dtype=np.uint64).astype(np.uint32)
    if case == "offset_narrow":    # a 2^23-wide range at 2^31: one top digit
        return (rng.integers(0, 1 << 23, n, dtype=np.uint64) + (1 << 31)).astype(np.uint32)
    # 40 values a few apart inside one top digit: shift 0, one value per digit
    return (rng.integers(0, 40, n, dtype=np.uint64) * 3 + 0x7F000000).astype(np.uint32)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("schedule", ["msd", "msdz"])
@pytest.mark.parametrize("case", ["below2pow24", "offset_narrow", "one_digit_dups"])
def test_range_digit_gloo(tmp_path, world, schedule, case):
    """the torch engine re-partitions narrow key ranges
    by the range digit (key - min) >> shift (libsortDistribRangeDigit, the C
    engine's rule) instead of the 4-exchange LSD rounds: the LSD rounds must
    not run (partial_sort raises), the result equals the oracle's sort and the
    shards are the equal re-cut."""
    from oracle import oracle
    x = _narrow_case(case)
    port = 30100 + 40 * world + 10 * ["msd", "msdz"].index(schedule) + ["below2pow24", "offset_narrow",
                                                                        "one_digit_dups"].index(case)
    shards = run_ranks(x, world, schedule, tmp_path, port=port, kw={"no_lsd": True})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


@pytest.mark.parametrize("world,case", [(2, "below2pow40"), (3, "stamps")])
def test_pairs_range_digit_gloo(tmp_path, world, case):
    """Pair keys below 2^56 or sharing their top byte: the pair rounds
    re-partition by the range digit (it must run), stable and exact."""
    from distrib_helpers import run_pair_ranks
    from oracle import oracle
    rng = np.random.default_rng(world)
    n = 30011
    if case == "below2pow40":
        k = rng.integers(0, 1 << 40, n, dtype=np.uint64)
    else:
        k = np.uint64(0x17A0000000000000) + rng.integers(0, 86400 * 10**9, n, dtype=np.uint64) // np.uint64(1000)
        k[::7] = k[3]  # ties across ranks
    ks, vs = run_pair_ranks(k, world, tmp_path, port=30300 + 10 * world, kw={"expect_range": True})
    rk, rv = oracle.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(np.concatenate(ks), rk)
    np.testing.assert_array_equal(np.concatenate(vs), rv)
