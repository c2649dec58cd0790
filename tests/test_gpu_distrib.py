"""Multi-rank driver with the HIP backend: 2 and 3 ranks sharing the one GPU
of the test box (exchanges over gloo, staged through host memory; on an
8-GPU node bench.py runs the same driver over RCCL).  Results are checked
against the oracle and the reference's re-cut semantics."""
import numpy as np
import pytest

from distrib_helpers import run_ranks, shard_inputs

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("schedule", ["msd", "lsd"])
def test_distributed_sort_hip_backend(tmp_path, world, schedule):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle
    x = oracle.pcg((1 << 20) + 12345, first=77)
    shards = run_ranks(x, world, schedule, tmp_path, use_gpu=True,
                       port=29700 + world * 2 + (schedule == "lsd"))
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


def test_distributed_skew_falls_back(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle
    rng = np.random.default_rng(11)
    x = rng.integers(0, 300, 200003, dtype=np.uint64).astype(np.uint32)  # one top bucket
    shards = run_ranks(x, 2, "msd", tmp_path, use_gpu=True, port=29790)
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))


@pytest.mark.parametrize("rounds", [1, 4, 16])
def test_msd_rounds_hip_backend(tmp_path, rounds):
    """Range-split rounds with libsort's table partition and sorts on the GPU
    (2 ranks sharing the GPU, gloo host-staged exchanges)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle
    x = oracle.pcg((1 << 20) + 777, first=rounds)
    shards = run_ranks(x, 2, "msd", tmp_path, use_gpu=True, port=29820 + rounds, kw={"rounds": rounds})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, 2)]


@pytest.mark.parametrize("world,rounds", [(2, 4), (2, 1), (3, 3)])
def test_msdz_hip_backend(tmp_path, world, rounds):
    """The delta-coded schedule with libsort's kernels (range sorts, gap
    coding, merges) on the GPU; ranks share the GPU, exchanges over gloo."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle
    x = oracle.pcg((1 << 20) + 4321, first=world * 10 + rounds)
    shards = run_ranks(x, world, "msdz", tmp_path, use_gpu=True, port=30300 + 10 * world + rounds,
                       kw={"rounds": rounds})
    np.testing.assert_array_equal(np.concatenate(shards), oracle.sort_u32(x))
    assert [s.size for s in shards] == [s.size for s in shard_inputs(x, world)]


def test_distrib_pairs_hip_backend(tmp_path):
    """C5 path on the GPU: stable (u64 key, u32 payload) sort over 2 ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distrib_helpers import run_pair_ranks
    from oracle import oracle
    rng = np.random.default_rng(9)
    n = (1 << 19) + 333
    k = rng.integers(0, 1 << 12, n, dtype=np.uint64) * np.uint64(0x0010000000000001)  # ties across ranks
    ks, vs = run_pair_ranks(k, 2, tmp_path, use_gpu=True, port=29960, kw={"rounds": 4})
    rk, rv = oracle.stable_sort_kv64(k, np.arange(n, dtype=np.uint32))
    np.testing.assert_array_equal(np.concatenate(ks), rk)
    np.testing.assert_array_equal(np.concatenate(vs), rv)


def test_round_schedules_over_rccl_single_rank():
    """The exchange path of the 8-GPU job on a real RCCL communicator (one
    rank: RCCL refuses two ranks on one GPU): async all_to_all_single per
    round, stream-level waits, per-round range sorts, pair rounds."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    import pathlib
    import subprocess
    import sys
    worker = pathlib.Path(__file__).with_name("rccl_single_rank_worker.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29993")
    r = subprocess.run([sys.executable, str(worker)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


def test_bench_self_launch_rehearsal():
    """bench.py's N>1 path end to end as the driver's 8-GPU job starts it
    (`python bench.py --gpus N`, no launcher: the bench starts
    torch.distributed.run itself as a child) with 2 ranks on the one GPU of
    the test box over gloo: timed distributed sorts, max-over-ranks timing,
    the collective verification and the 8-bit variant all complete, and the
    parent relays exactly one line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_REHEARSAL"] = "1"
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--keys-log2", "20"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified"] is True and line["rehearsal"]
    assert line["config"]["global_keys"] == 2 << 20 and line["variants"]["digit8"]["value"] > 0


def test_bench_self_launch_rehearsal_world8():
    """configs[3]'s world size on the HIP kernels: `bench.py --gpus 8` with
    eight gloo ranks sharing the one GPU (BENCH_REHEARSAL), 2^20 keys per
    rank: the 8-rank plan, partition, exchange, round sorts, re-cut and the
    collective verification all run on the GPU, and rank 0's line is relayed."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_REHEARSAL"] = "1"
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1", "--keys-log2", "20",
           "--no-variants"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["verified"] is True and line["rehearsal"]
    assert line["config"]["global_keys"] == 8 << 20


@pytest.mark.parametrize("world,pairs,sched", [(2, False, "auto"), (8, False, "auto"), (3, True, "auto"),
                                               (2, False, "msdz")])
def test_bench_cabi_engine_rehearsal(world, pairs, sched):
    """`bench.py --gpus N --engine cabi`: rank 0 drives all N ranks through
    the C ABI (libsortDistribSortU32 / libsortDistribSortPairsU64U32; here
    all on the one GPU, device-copy exchanges) while the other ranks keep the
    barriers; the result is verified on rank 0 and relayed."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_REHEARSAL"] = "1"
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--keys-log2", "20", "--engine", "cabi", "--no-variants", "--schedule", sched] + \
        (["--workload", "c5"] if pairs else [])
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["verified"] is True
    assert "C-ABI engine" in line["config"]["workload"]
    assert "engine_note" not in line and line["engine"].startswith("cabi")
    assert line["cabi_first_step"] == "verified"
    sent = line["exchange_bytes_per_rank"]
    assert len(sent) == world and all(b > 0 for b in sent), sent
    if sched == "msdz":  # the gap-coded rounds (LIBSORT_DISTRIB_CODED): ~16.5 bits per sent key at 2^20 per rank
        assert "delta-coded" in line["config"]["workload"]
        assert all(b < 0.6 * 4 * (1 << 20) * (world - 1) / world for b in sent), sent
    # the stage trace of the verified first step is in the stderr tail
    assert "libsort distrib [" in r.stderr and "done: ok" in r.stderr, r.stderr[-3000:]
    assert "bench.py [rank 0" in r.stderr


def test_bench_cabi_bad_first_step_falls_back_to_torch():
    """The C engine's first step is verified before it is timed (its
    distinct-device paths only run on a multi-GPU node): a wrong result
    (BENCH_CABI_FAULT=1 corrupts one key of it) hands the measurement to the
    torch engine on every rank, and the line says so."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_REHEARSAL"] = "1"
    env["BENCH_CABI_FAULT"] = "1"
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--keys-log2", "20", "--engine", "cabi", "--no-variants"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["verified"] is True
    assert "failed verification" in line["engine_note"] and not line["engine"].startswith("cabi")
    assert line["cabi_first_step"].startswith("FAILED")


@pytest.mark.parametrize("fault", [None, "fail", "hang"])
def test_bench_cabi_probe(fault):
    """On a multi-GPU node rank 0 first runs one verified C-engine step in a
    child process (`bench.py ... --cabi-probe`, its stage trace passed
    through): a child that fails or hangs (killed at BENCH_CABI_PROBE_S)
    hands the measurement to the torch engine instead of ending the run.
    Here forced on (BENCH_CABI_PROBE=1) with the ranks sharing the GPU; the
    faults are injected in the child (BENCH_CABI_PROBE_FAULT)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import os
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(BENCH_REHEARSAL="1", BENCH_CABI_PROBE="1", BENCH_CABI_PROBE_S="30")
    if fault:
        env["BENCH_CABI_PROBE_FAULT"] = fault
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--keys-log2", "20", "--engine", "cabi", "--no-variants"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["verified"] is True
    if fault is None:
        assert line["cabi_probe"].startswith("verified in a child process"), line["cabi_probe"]
        assert line["engine"].startswith("cabi") and line["cabi_first_step"] == "verified"
        assert "bench.py [cabi probe]: libsort distrib [" in r.stderr, r.stderr[-3000:]
    else:
        want = "timed out after 30 s" if fault == "hang" else "exited with 1"
        assert want in line["cabi_probe"] and want in line["engine_note"], line
        assert not line["engine"].startswith("cabi") and line["cabi_first_step"].startswith("FAILED")


def test_bench_single_gpu_line_contract():
    """bench.py at N=1 (small steps): one JSON line with the driver's keys,
    the roofline object (live per-launch pass time), a verified sort, the
    8-bit variant and the PCIe-inclusive host-ABI leg checked against the
    device sort."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    cmd = [sys.executable, str(root / "bench.py"), "--steps", "3", "--warmup", "1", "--keys-log2", "24",
           "--cpu-sample-log2", "18"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=str(root))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["verified"] is True and d["value"] > 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0 and 0 < rf["frac"] < 1
    assert abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 1e-3
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] == 1
    assert d["cpu_baseline"]["nproc"] >= 1 and d["cpu_baseline"]["host_cpu"]
    assert d["host_abi"]["value"] > 0 and d["variants"]["digit8"]["value"] > 0
    assert d["settle"]["steps"] >= 2 and d["settle"]["seconds"] > 0  # untimed clock-settle steps, reported
