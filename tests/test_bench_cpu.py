"""bench.py's launcher contract on the CPU (no GPU touched): `python bench.py
--gpus N` with no launcher starts torch.distributed.run with N ranks as a
child process, relays rank 0's single JSON line and exits non-zero when any
rank fails; a WORLD_SIZE / --gpus mismatch is rejected.  The ranks run the
BENCH_LAUNCH_PROBE body (join a gloo group, rank 0 prints one line); the
full N>1 bench body is rehearsed on the GPU box
(tests/test_gpu_distrib.py::test_bench_self_launch_rehearsal)."""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=str(ROOT))


def test_bench_starts_its_ranks_without_a_launcher():
    r = _run(["--gpus", "2"], _env(BENCH_LAUNCH_PROBE="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == {"probe": True, "world": 2}


def test_bench_launcher_fails_when_a_rank_fails():
    r = _run(["--gpus", "2"], _env(BENCH_LAUNCH_PROBE="fail"))
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_rejects_world_size_mismatch():
    r = _run(["--gpus", "4"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", BENCH_LAUNCH_PROBE="1"), timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_n_gt_1_defaults_to_configs3_share():
    """configs[3] = 2^32 keys over 8 GPUs: 2^29 keys per GPU at N>1, 2^28
    (configs[1]) at N=1."""
    sys.path.insert(0, str(ROOT))
    import bench
    old = sys.argv
    try:
        sys.argv = ["bench.py", "--gpus", "8"]
        a = bench.parse()
        assert a.keys_log2 == 29 and a.digit_bits == 4
        sys.argv = ["bench.py"]
        a = bench.parse()
        assert a.keys_log2 == 28 and a.digit_bits == 4
        sys.argv = ["bench.py", "--gpus", "8", "--workload", "c5"]
        assert bench.parse().keys_log2 == 28                       # 2^31 pairs over 8 GPUs
    finally:
        sys.argv = old
