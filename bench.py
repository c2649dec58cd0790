#!/usr/bin/env python3
"""Benchmark: uint32 full sort, keys resident in HBM (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c5]

c2 (default; the bench line): configs[1] = "256M uint32, 4-bit digits,
    gpuFullSort on 1 MI355X": 2^28 keys of the reference populateInput stream
    (generated on the GPU by skip-ahead), one step = one full 32-bit sort
    through the libsort C ABI (libsortSortKeysU32 = the device-resident form
    of providedGpu): the MSD hybrid, i.e. four 4-bit digit passes from the top
    digit down (the first with reserved runs, no count pass) and the on-chip
    sort of every 16-bit bucket; `variants.lsd` times
    the plain 8-pass LSD sort.
    N>1 = configs[3] ("2^32 uint32 sharded 8xMI355X"): 2^29 keys per GPU
    (2^32 at N=8); rank r holds keys [r*2^29, (r+1)*2^29) of the same stream
    (weak scaling); one step = one distributed sort ending with rank r holding
    keys [r*S, (r+1)*S) of the sorted array.  Engine (--engine auto): the C
    engine at every N -- rank 0 drives every GPU through the C ABI
    (libsortDistribSortU32, what C and Go callers bind: top-digit partition,
    K = 4 RCCL point-to-point rounds overlapped with the round sorts; at 2
    GPUs its gap-coded rounds, LIBSORT_DISTRIB_CODED: the same rounds sorted
    by the sender and exchanged gap-coded, since one xGMI link carries half
    of every shard), its first step verified (and stage-traced) before
    timing; --engine torch = one process per GPU (pylibsort.distrib, the
    same schedules over torch.distributed).  `python bench.py --gpus N` with no launcher starts its N ranks
    itself: torch.distributed.run as a CHILD process (no exec), rank 0's JSON
    line relayed, non-zero exit if any rank fails.
c3: configs[2], 2^30 keys, 8-bit digits, one GPU.
c5: configs[4], stable (u64 key, u32 payload) sort, 2^28 pairs per GPU (2^31
    on 8 GPUs); key = (draw 2i << 32) | draw 2i+1 of the stream, payload = the
    global index; N>1 runs the C pair engine (libsortDistribSortPairsU64U32)
    (the same engine choice as c2).

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
for p in (str(ROOT), str(ROOT / "gpu-radix-sort_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# N>1 engine when --engine auto: the C engine at every
# world size (the engine Go/C callers bind is the one
# measured).  It was the faster of the two on the one-GPU schedule
# measurement at 2^29 keys per rank (profiles/r03w_msd_schedule_2pow29_shape8.txt:
# 6.56 vs 6.71 ms in the 8-GPU per-rank shape); at N = 2 it runs the
# gap-coded rounds (~9.5 of 32 bits per key on the wire) that were the torch
# engine's reason to exist there -- two GPUs share ONE xGMI link, so the link,
# not the GPU work, bounds that step.
def default_engine(world):
    return "cabi"
PASS_KERNELS = "tilepass,onesweep,downsweep"  # the roofline kernel candidates (timed-region events)
EVENT_STRIDE = 5  # N=1 timed region: events around every 5th pass launch (libsortTimingSample)
# N=1 secondary legs: untimed calls for at least this long before each timed
# region.  The first ~30 ms of calls after the GPU idled (the CPU baseline,
# the host ABI leg's PCIe copies) run up to 25% slow: an 8-bit digit pass
# took 550 us falling to 420 us over 16 calls (profiles/r06i_clock_settle.txt)
SETTLE_S = 0.25


def settle(step, torch, seconds=SETTLE_S):
    """Untimed calls of `step` (each synchronised) until `seconds` have
    passed, at least 2; returns how many ran.  World size 1 only: the ranks
    of a multi-process step would disagree on the count."""
    calls, t_end = 0, time.perf_counter() + seconds
    while calls < 2 or time.perf_counter() < t_end:
        step()
        torch.cuda.synchronize()
        calls += 1
    return calls


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 20 (~45 ms at N=1): the clocks settle over the first ~30 ms of sorting
    # after the GPU idled (--warmup 3: 2.243 ms/step, 60: 2.203; r06i)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c5"])
    ap.add_argument("--keys-log2", type=int, default=None, help="keys (pairs) per GPU = 2^k")
    ap.add_argument("--digit-bits", type=int, default=None, help="configs[1] names 4-bit digits")
    ap.add_argument("--schedule", default="auto", choices=["auto", "msd", "msdz", "lsd"],
                    help="auto: msdz (gap-coded exchange) at 2 GPUs, msd otherwise")
    ap.add_argument("--rounds", type=int, default=4, help="msd exchange rounds (pylibsort.distrib.ROUNDS)")
    ap.add_argument("--engine", default="auto", choices=["auto", "torch", "cabi"],
                    help="N>1: torch = one process per GPU (pylibsort.distrib over torch.distributed); cabi = rank "
                         "0 drives every GPU through the C ABI (libsortDistribSortU32 / ...PairsU64U32, the "
                         "single-process RCCL engine C and Go callers bind; gap-coded rounds at 2 GPUs); auto = cabi")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log2", type=int, default=28,
                    help="keys of the providedCpu baseline sample (BASELINE.md section 3: 2^28)")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-host-abi", action="store_true", help="skip the PCIe-inclusive providedGpu leg")
    ap.add_argument("--no-legs", action="store_true", help="skip the configs[2] / configs[4] legs of the N=1 line")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--algo", default=None, choices=["auto", "tiles", "onesweep", "rts"],
                    help="force the pass algorithm (LIBSORT_ALGO)")
    ap.add_argument("--cabi-probe", action="store_true", help=argparse.SUPPRESS)  # (rank 0's child: cabi_probe)
    a = ap.parse_args()
    # c2 at N>1 is configs[3]: 2^29 keys per GPU, 2^32 over 8 GPUs
    defaults = {"c2": (28 if a.gpus == 1 else 29, 4), "c3": (30, 8), "c5": (28, 8)}[a.workload]
    a.keys_log2 = defaults[0] if a.keys_log2 is None else a.keys_log2
    a.digit_bits = defaults[1] if a.digit_bits is None else a.digit_bits
    return a


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nranks, argv):
    """`bench.py --gpus N` without a launcher: start torch.distributed.run
    with N ranks as a child process (never exec: nothing here has touched the
    GPU, and the ranks initialise it themselves), pass its stderr through,
    relay rank 0's JSON line and return the launcher's exit status (non-zero
    when any rank failed)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(pathlib.Path(__file__).resolve())]
    cmd += list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for ln in p.stdout:
        if ln.startswith("{"):
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = p.wait()
    if rc != 0:
        sys.stderr.write("bench.py: torch.distributed.run exited with %d\n" % rc)
        return rc if rc > 0 else 1
    if len(lines) != 1:
        sys.stderr.write("bench.py: expected one JSON line from rank 0, got %d\n" % len(lines))
        return 1
    print(lines[0], flush=True)
    return 0


def launch_probe(mode):
    """BENCH_LAUNCH_PROBE (CPU tests of the launcher): every rank joins a gloo
    group and rank 0 prints one JSON line; "fail" makes rank 1 exit 3.  No GPU
    is touched."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if mode == "fail" and rank == 1:
        sys.exit(3)
    dist.init_process_group("gloo")
    dist.barrier()
    if rank == 0:
        print(json.dumps({"probe": True, "world": world}), flush=True)
    dist.destroy_process_group()


def stage(rank, world, what):
    """One stderr line per bench phase at N > 1 (the driver's record keeps the
    stderr tail: a run that hangs names its phase; with the C engine's own
    stage trace on for its first step, libsortSetDistribTrace)."""
    if world > 1:
        sys.stderr.write("bench.py [rank %d, %.1f s]: %s\n" % (rank, time.perf_counter() - _T0, what))
        sys.stderr.flush()


_T0 = time.perf_counter()


def main():
    args = parse()
    if args.algo:
        os.environ["LIBSORT_ALGO"] = args.algo
    if args.schedule == "msd" and args.gpus == 2:
        os.environ["LIBSORT_DISTRIB_CODED"] = "0"  # (the C engine's default at 2 GPUs is the coded rounds)
    if args.cabi_probe:
        return cabi_probe(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    probe = os.environ.get("BENCH_LAUNCH_PROBE")
    if probe:
        return launch_probe(probe)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.workload == "c3" and world > 1:
        raise SystemExit("c3 is a single-GPU configuration")
    # BENCH_REHEARSAL=1: several ranks on ONE GPU over gloo (host-staged
    # exchanges) to exercise the N>1 code path on a 1-GPU box; never a result
    rehearsal = os.environ.get("BENCH_REHEARSAL") == "1"
    dev_index = 0 if rehearsal else local_rank
    torch.cuda.set_device(dev_index)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))

    import pylibsort
    import pylibsort.device as D
    from pylibsort import distrib

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    pylibsort.setDigitBits(args.digit_bits)
    pairs = args.workload == "c5"

    n = 1 << args.keys_log2
    vals = None
    if pairs:
        w = D.populate_u32(2 * n, first=rank * 2 * n).view(n, 2).to(torch.int64)
        keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
        vals = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64, device="cuda").to(torch.int32)
        del w
        out, outv = torch.empty_like(keys), torch.empty_like(vals)
        tmp, tmpv = torch.empty_like(keys), torch.empty_like(vals)
    else:
        keys = D.populate_u32(n, first=rank * n)
        out = torch.empty_like(keys)
        tmp = torch.empty_like(keys)
    torch.cuda.synchronize()
    ops = distrib.HipOps() if world > 1 else None
    engine = default_engine(world) if args.engine == "auto" else args.engine
    cabi = world > 1 and engine == "cabi"
    # host-side waits: barriers, the engine decision and the max-over-ranks
    # time go over gloo, so a rank that waits (every rank but 0 while the C
    # engine runs) holds no spinning RCCL kernel on its GPU
    cpu_pg = dist.new_group(backend="gloo") if world > 1 and not rehearsal else None
    engine_note = None
    probe_note = None  # the line's record of the C engine's probe (N > 1)
    if cabi and rank == 0 and cabi_probe_on(rehearsal):
        # one verified C-engine step in a child process first: a hang or a
        # fault there costs a timeout and the torch engine, not the run
        tmo = float(os.environ.get("BENCH_CABI_PROBE_S", "240"))
        stage(rank, world, "C-ABI engine probe: one verified step in a child process (timeout %.0f s)" % tmo)
        ok, probe_note = run_cabi_probe(tmo)
        if not ok:
            engine_note = "C-ABI engine probe %s; torch engine measured" % probe_note
    shards = vshards = None
    if cabi and rank == 0 and engine_note is None:
        # one process drives every GPU through the C ABI (what a C or Go
        # caller binds); the other ranks keep the barriers and the max-over-
        # ranks timing.  Shard r = the same keys rank r holds in torch mode.
        # (every rank keeps its own keys too: the torch engine takes over if
        # the C engine fails its first step)
        shards, vshards = make_shards(torch, D, [0] * world if rehearsal else list(range(world)), n, pairs)

    # C engine flags: the schedule asked for (auto: the engine's own choice --
    # gap-coded rounds at 2 GPUs, top-digit rounds otherwise)
    cabi_flags = cabi_flags_for(D, args.schedule)

    def step():
        if cabi:
            if rank != 0:
                return None
            if pairs:
                return D.distrib_sort_pairs_u64_u32(shards, vshards)
            return D.distrib_sort_u32(shards, cabi_flags)
        if pairs:
            if world == 1:
                return D.sort_pairs_u64_u32(keys, vals, out_keys=out, out_vals=outv, tmp_keys=tmp, tmp_vals=tmpv)
            return distrib.distrib_sort_pairs(keys, vals, ops=ops, rounds=args.rounds)
        if world == 1:
            return D.sort_keys_u32(keys, out=out, tmp=tmp)
        if args.schedule == "lsd":
            return distrib.distrib_sort(keys, ops=ops, schedule="lsd")
        return distrib.distrib_sort(keys, ops=ops, schedule=args.schedule, rounds=args.rounds)

    def barrier():
        if world > 1:
            dist.barrier(group=cpu_pg)

    cabi_first = None  # the line's record of the C engine's verified first step (N > 1)
    if cabi:
        # first step of the C engine, verified; if it fails or its output is
        # wrong on rank 0 (distinct-device paths run only on a multi-GPU
        # node), every rank switches to the torch engine (identical decision
        # via all_reduce)
        failed = 1 if engine_note else 0
        stage(rank, world, "C-ABI engine: first step (verified; stage trace on)")
        if rank == 0 and not failed:
            try:
                prev_trace = pylibsort.lib().libsortSetDistribTrace(1)
                try:
                    first = step()
                    torch.cuda.synchronize()
                finally:
                    pylibsort.lib().libsortSetDistribTrace(prev_trace)
                if os.environ.get("BENCH_CABI_FAULT") == "1":  # rehearsal of the fallback (tests only)
                    (first[0] if pairs else first)[0][:1] = 0 if pairs else -1
                if not args.no_verify and not verify_cabi(torch, shards, first, vshards if pairs else None):
                    failed, engine_note = 1, "C-ABI engine's first step failed verification; torch engine measured"
                else:
                    cabi_first = "verified" if not args.no_verify else "not verified (--no-verify)"
                del first
            except RuntimeError as e:
                failed, engine_note = 1, "C-ABI engine failed its first step (%s); torch engine measured" % e
        flag = torch.tensor([failed], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=cpu_pg)
        if int(flag.item()):
            cabi = False
            engine = "torch"
            if rank == 0:
                sys.stderr.write("bench.py: %s\n" % engine_note)
    stage(rank, world, "warmup (%d steps, %s engine)" % (args.warmup, engine))
    # N=1: untimed steps for SETTLE_S first, whatever W is (the clocks settle
    # over the first ~30 ms of sorting: W=3 2.243 ms/step, W=60 2.203; r06i);
    # reported in the line.  (N>1: the ranks' step counts must agree)
    settled = settle(step, torch) if world == 1 and os.environ.get("BENCH_SETTLE", "1") != "0" else 0
    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    barrier()
    stage(rank, world, "timed steps (%d)" % args.steps)

    # events in the timed region only around the pass kernel the roofline is
    # priced on (every kernel's events cost ~2.5% of the 2^28 sort); the full
    # per-kernel breakdown comes from two more steps after the timed region
    events = os.environ.get("BENCH_KERNEL_EVENTS", "1") != "0"  # "0": A/B of the events' own cost
    # every EVENT_STRIDE-th pass launch gets its two events: 5 is coprime to
    # the 4 digit passes of a configs[1] sort, so the sampled launches rotate
    # over all four (each event stalls the stream ~5 us: 8 per sort cost ~1.5%)
    stride = EVENT_STRIDE if world == 1 else 1
    D.timing_reset()
    D.timing_filter(PASS_KERNELS)
    D.timing_sample(stride)
    D.timing_enable(events)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    D.timing_enable(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cpu_pg)
        elapsed = float(t.item())

    # live per-kernel durations (hipEvents on libsort's launch stream): the
    # pass kernel from the timed steps, every kernel from two more steps
    def query(names):
        got = {}
        for name in names:
            launches, ms, kk = D.timing_query(name)
            if launches:
                got[name] = {"launches": launches, "avg_us": 1e3 * ms / launches, "keys_per_launch": kk / launches}
        return got

    stage(rank, world, "timed steps done: %.3f s; per-kernel event steps" % elapsed)
    timed_pass = query(PASS_KERNELS.split(","))
    D.timing_reset()
    D.timing_sample(1)
    D.timing_filter(None)
    D.timing_enable(events)
    for _ in range(2):
        res = step()
    torch.cuda.synchronize()
    barrier()
    D.timing_enable(False)
    kern = query(("whist", "onesweep", "upsweep", "scan", "downsweep", "tilecounts", "colscan", "tilepass",
                  "hybplan", "bucketsort", "partition", "histogram", "segcopy", "rsvsample"))
    for name in kern:
        kern[name]["from"] = "2 steps after the timed region"
    kern.update({name: dict(v, **{"from": "the timed steps"}) for name, v in timed_pass.items()})

    # verification outside the timed region: sorted + same multiset (checksums)
    stage(rank, world, "verification")
    verified = None
    if not args.no_verify and cabi:
        verified = verify_cabi(torch, shards, res, vshards if pairs else None) if rank == 0 else None
    elif not args.no_verify:
        verified = verify(torch, dist, world, keys, res, vals)

    # N>1: the same distributed sort with 8-bit local digits (all ranks take
    # part; max over ranks), reported beside the 4-bit line, never as `value`
    variant8 = None
    if world > 1 and not args.no_variants and not pairs:
        stage(rank, world, "8-bit digit variant")
        prev = pylibsort.setDigitBits(8)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        barrier()
        reps = max(5, args.steps // 2)
        v0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        barrier()
        tv = torch.tensor([time.perf_counter() - v0], dtype=torch.float64)
        dist.all_reduce(tv, op=dist.ReduceOp.MAX, group=cpu_pg)
        pylibsort.setDigitBits(prev)
        ms8 = 1e3 * float(tv.item()) / reps
        variant8 = {"ms_per_step": round(ms8, 4), "value": round(n * world / (ms8 * 1e-3) / 1e9, 3),
                    "note": "same distributed sort with 8-bit digits in the local round sorts (the reference's "
                            "distributed driver rounds are 8 bits wide); reported beside the 4-bit line"}

    total_keys = n * world
    ms_per_step = 1e3 * elapsed / args.steps
    value = total_keys / (elapsed / args.steps) / 1e9

    if rank == 0:
        ds_name = next((k for k in ("tilepass", "onesweep", "downsweep") if k in kern), "downsweep")
        ds = kern.get(ds_name)
        unit_bytes = 24.0 if pairs else 8.0  # read + write of one key (pair)
        roofline = None
        if ds:
            bytes_per_launch = unit_bytes * ds["keys_per_launch"]
            achieved = bytes_per_launch / (ds["avg_us"] * 1e-6) / 1e9
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                        "kernel": "k_%s (rank + scatter pass)" % ds_name, "algorithmic_bytes_per_launch": bytes_per_launch,
                        "avg_launch_us": round(ds["avg_us"], 2), "launches": ds["launches"],
                        "timing": "live hipEvents around every %s pass launch of the timed steps (and no other "
                                  "kernel), on libsort's stream" % ("%dth (rotating over a sort's passes)" % stride
                                                                    if stride > 1 else "")}
            # the committed profiles of THIS round's build and bench command
            # (tools/collect_profiles.sh): HBM bytes per launch from the PMC
            # passes, and the same kernel's average duration in rocprofv3's
            # kernel trace, so `frac` can be re-derived from profiles/
            if args.workload == "c2" and world == 1 and args.keys_log2 == 28 and ds_name == "tilepass":
                roofline.update(committed_profile(bytes_per_launch))
        if roofline is not None and world == 1 and not pairs:
            roofline["step"] = step_roofline(n, args.digit_bits, ms_per_step, kern)
        bs = kern.get("bucketsort")
        if bs:
            ach = 8.0 * bs["keys_per_launch"] / (bs["avg_us"] * 1e-6) / 1e9 if not pairs else None
            if ach:
                bs["achieved_gbps"] = round(ach, 1)
                bs["frac"] = round(ach / HBM_PEAK_GBPS, 4)
                bs["bytes_per_key"] = 8.0
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not pairs:
            cpu = cpu_baseline_leg(torch, pylibsort, keys, out, args.cpu_sample_log2)
        variants = {}
        if world > 1 and variant8 is not None:
            variants["digit8"] = variant8
        if world == 1 and not args.no_variants and args.workload == "c2":
            ref_out = out.clone()
            prev = pylibsort.setDigitBits(8)
            settle(lambda: D.sort_keys_u32(keys, out=out, tmp=tmp), torch)
            if not torch.equal(out, ref_out):
                raise RuntimeError("8-bit digit variant disagrees with the 4-bit sort")
            del ref_out
            v0 = time.perf_counter()
            for _ in range(max(5, args.steps // 2)):
                D.sort_keys_u32(keys, out=out, tmp=tmp)
            torch.cuda.synchronize()
            v1 = time.perf_counter()
            pylibsort.setDigitBits(prev)
            ms8 = 1e3 * (v1 - v0) / max(5, args.steps // 2)
            variants["digit8"] = {"ms_per_step": round(ms8, 4), "value": round(n / (ms8 * 1e-3) / 1e9, 3),
                                  "note": "same sort with 8-bit digits (4 passes, configs[2] digit width); output "
                                          "checked equal to the 4-bit sort"}
        if world == 1 and not args.no_variants and args.workload == "c2":
            variants["lsd"] = lsd_variant(torch, pylibsort, D, keys, out, tmp, max(5, args.steps // 2))
            variants["bucket_lsd_steps"] = bucket_steps_variant(torch, pylibsort, D, keys, out, tmp,
                                                                max(5, args.steps // 2))
        if world == 1 and not args.no_variants and not args.no_legs and args.workload == "c2" and args.keys_log2 == 28:
            # the other single-GPU configurations, each with its own live
            # per-kernel timings (never `value`)
            variants["c3"] = config_leg(torch, pylibsort, D, "c3", max(5, args.steps // 2))
            variants["c5"] = config_leg(torch, pylibsort, D, "c5", max(5, args.steps // 2))
        host_abi = None
        if world == 1 and not args.no_host_abi and args.workload == "c2":
            host_abi = host_abi_leg(torch, pylibsort, keys, out)
        if world == 1 and not args.no_variants and not args.no_legs and args.workload == "c2" and args.keys_log2 == 28:
            # gpuPartial at the reference's own benchmark workload (these
            # overwrite `out`: after every use of the line's sorted keys)
            for w in (8, 16):
                variants["partial%d" % w] = partial_leg(torch, pylibsort, D, keys, out, tmp, w,
                                                        max(5, args.steps // 2))
        sched = ""
        if world > 1:
            sname = args.schedule
            if sname == "auto":
                sname = "msdz" if world == 2 and not rehearsal else "msd"
            if pairs:
                sname = "msd"
            sched = (", %s schedule (top-digit rounds)%s, %d rounds, over %d GPUs (RCCL point-to-point)"
                     % (sname, " with delta-coded exchange" if sname == "msdz" else "", args.rounds, world)
                     if sname != "lsd" else ", lsd schedule over %d GPUs (RCCL alltoallv)" % world)
            sched += (", C-ABI engine (one process drives every GPU: libsortDistribSort%s)"
                      % ("PairsU64U32" if pairs else "U32") if cabi else
                      ", torch engine (one process per GPU, pylibsort.distrib)")
        if pairs:
            metric, unit, dtype = "Gpairs/sec (u64 key, u32 payload) stable sort", "Gpairs/s", "u64+u32"
            workload = "configs[4]: 2^%d (u64 key, u32 payload) pairs per GPU, %d-bit digits, stable sort%s" % (
                args.keys_log2, args.digit_bits, sched)
        else:
            metric, unit, dtype = "Gkeys/sec uint32 full sort", "Gkeys/s", "u32"
            if world > 1:
                workload = ("configs[3]: sharded full sort of 2^%d uint32 keys = 2^%d per GPU (configs[3] names "
                            "2^32 over 8 GPUs), %d-bit digits in the local sorts, weak scaling%s"
                            % (args.keys_log2 + (world - 1).bit_length(), args.keys_log2, args.digit_bits, sched)
                            if world & (world - 1) == 0 else
                            "configs[3]: sharded full sort, 2^%d uint32 keys per GPU over %d GPUs, %d-bit digits%s"
                            % (args.keys_log2, world, args.digit_bits, sched))
            else:
                workload = "configs[%d]: 2^%d uint32 keys per GPU, %d-bit digits, full sort%s" % (
                    1 if args.workload == "c2" else 2, args.keys_log2, args.digit_bits, sched)
        line = {
            "metric": metric,
            "value": round(value, 3),
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"steps": settled, "seconds": SETTLE_S if settled else 0,
                       "note": "untimed steps before the W warm-up steps (N=1): the GPU's clocks settle over the "
                               "first ~30 ms of sorting after idling (profiles/r06i_clock_settle.txt)"},
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic: reference populateInput PCG32 stream, generated on device",
            "config": {"workload": workload, "keys_per_gpu": n, "digit_bits": args.digit_bits,
                       "global_keys": total_keys, "parallelism": "shards%d" % world},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": kern,
            "verified": verified,
            "variants": variants or None,
            "host_abi": host_abi,
        }
        if world > 1:
            line["engine"] = ("cabi: rank 0 drives all %d GPUs through the C ABI" % world if cabi else
                              "torch: one process per GPU")
            # the C engine's first step, always stated: a failure there is
            # measured on the torch engine but shows in the line
            line["cabi_first_step"] = (engine_note and "FAILED: " + engine_note) or cabi_first or \
                "not run (torch engine chosen)"
            if probe_note is not None:
                line["cabi_probe"] = probe_note
            if engine_note:
                line["engine_note"] = engine_note
            if cabi:
                try:  # (bytes each rank sent in the last step's exchange rounds)
                    line["exchange_bytes_per_rank"] = D.distrib_last_bytes(world)
                except RuntimeError:
                    pass
        if rehearsal:
            line["rehearsal"] = "gloo, all ranks on one GPU: exercises the N>1 path, not a measurement"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier(group=cpu_pg)
        dist.destroy_process_group()


PROFILE_TAG = "r06y"  # profiles/<tag>_* of this round's build (tools/collect_profiles.sh)


def committed_profile(bytes_per_launch):
    """traffic + rocprof agreement fields from profiles/<PROFILE_TAG>_*.json."""
    out = {}
    pmc = ROOT / "profiles" / ("%s_pmc_tilepass.json" % PROFILE_TAG)
    rp = ROOT / "profiles" / ("%s_rocprof_tilepass.json" % PROFILE_TAG)
    try:
        d = json.loads(pmc.read_text())
        out["traffic"] = d["hbm_bytes_per_launch"]
        out["traffic_source"] = "profiles/%s (%s)" % (pmc.name, d.get("method", ""))
    except (OSError, ValueError, KeyError):
        pass
    try:
        d = json.loads(rp.read_text())
        us = float(d["avg_launch_us"])
        out["rocprof"] = {"avg_launch_us": round(us, 2), "launches": d.get("launches"),
                          "frac": round(bytes_per_launch / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                          "source": "profiles/%s" % rp.name, "cmd": d.get("cmd")}
    except (OSError, ValueError, KeyError):
        pass
    return out


def committed_leg(leg):
    """The committed rocprof average and PMC traffic of a leg's kernel
    (profiles/<PROFILE_TAG>_legs.json, tools/make_profile_summary.py), for the
    legs' live `frac` to be checked against (same command as the line)."""
    try:
        d = json.loads((ROOT / "profiles" / ("%s_legs.json" % PROFILE_TAG)).read_text())
        g = d["legs"][leg]
    except (OSError, ValueError, KeyError):
        return {}
    out = {"rocprof": {"avg_launch_us": round(g["avg_launch_us"], 2), "launches": g["launches"],
                       "frac": g["frac_rocprof"], "kernel": g["kernel"],
                       "source": "profiles/%s_legs.json" % PROFILE_TAG, "cmd": d.get("cmd")}}
    if "hbm_bytes_per_launch" in g:
        out["traffic"] = g["hbm_bytes_per_launch"]
        out["traffic_over_algorithmic"] = g["traffic_over_algorithmic"]
    return out


def step_roofline(n, digit_bits, ms_per_step, kern):
    """The whole N=1 step against HBM: the bytes the
    hybrid sort actually moves per step -- one count read (4 B/key; none with
    the reserved depth 0), 16 / digit_bits digit passes and the bucket sort
    (read + write, 8 B/key each) -- / ms_per_step.  (Round 4's LSD-equivalent
    figure priced passes the step does not run; dropped)"""
    passes = 16 // digit_bits if "bucketsort" in kern else 32 // digit_bits
    count = "tilecounts" in kern  # (4-bit keys-only hybrid: reserved depth 0, no count read)
    actual = n * ((4.0 if count else 0.0) + 8.0 * passes + (8.0 if "bucketsort" in kern else 0.0))
    t = ms_per_step * 1e-3
    return {"actual_bytes_per_key": actual / n, "actual_gbps": round(actual / t / 1e9, 1),
            "actual_frac": round(actual / t / 1e9 / HBM_PEAK_GBPS, 4),
            "note": "whole step (ms_per_step): %s%d digit passes%s" % ("count read + " if count else "", passes,
                                                                       " + bucket sort" if "bucketsort" in kern
                                                                       else "")}


def lsd_variant(torch, pylibsort, D, keys, out, tmp, reps):
    """The reference-shaped LSB sort (libsortSetHybrid(0): 32 / digit-bits
    LSD passes, what north_star names), timed beside the hybrid line and
    checked equal to its output."""
    ref = out.clone()
    prev = pylibsort.setHybrid("off")
    try:
        settle(lambda: D.sort_keys_u32(keys, out=out, tmp=tmp), torch)
        same = bool(torch.equal(out, ref))
        t0 = time.perf_counter()
        for _ in range(reps):
            D.sort_keys_u32(keys, out=out, tmp=tmp)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / reps
    finally:
        pylibsort.setHybrid(prev)
    if not same:
        raise RuntimeError("LSD variant disagrees with the hybrid sort")
    return {"ms_per_step": round(ms, 4), "value": round(keys.numel() / (ms * 1e-3) / 1e9, 3),
            "verified_equal_to_value_sort": same,
            "note": "libsortSetHybrid(0): the LSB radix sort of north_star (%d LSD passes at the line's digit width), "
                    "output checked equal to the hybrid sort's" % (32 // pylibsort.getDigitBits())}


def bucket_steps_variant(torch, pylibsort, D, keys, out, tmp, reps):
    """The same hybrid sort with the bucket sort's 4-bit LSD steps on chip
    (libsortSetBucketMode(0)) instead of the counting placement (12-bit cells
    with 4-bit residual counts), timed beside the line and checked equal."""
    ref = out.clone()
    lib = pylibsort.lib()
    prev = lib.libsortSetBucketMode(0)
    try:
        settle(lambda: D.sort_keys_u32(keys, out=out, tmp=tmp), torch)
        same = bool(torch.equal(out, ref))
        t0 = time.perf_counter()
        for _ in range(reps):
            D.sort_keys_u32(keys, out=out, tmp=tmp)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / reps
    finally:
        lib.libsortSetBucketMode(prev)
    if not same:
        raise RuntimeError("bucket-steps variant disagrees with the line's sort")
    return {"ms_per_step": round(ms, 4), "value": round(keys.numel() / (ms * 1e-3) / 1e9, 3),
            "verified_equal_to_value_sort": same,
            "note": "libsortSetBucketMode(0): the bucket sort as four 4-bit LSD steps on chip (ballot ranks) instead "
                    "of the counting placement; the same 4 MSD digit passes"}


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_leg(torch, pylibsort, keys, sorted_keys, sample_log2):
    """SURVEY.md section 8(d) CPU baseline: this library's exported
    providedCpu (std::sort, invokers.cu:68-71; single thread, as the
    reference) on the first 2^k keys of the same workload, timed on this
    box's host; the result is checked equal to the GPU sort when the sample
    is the whole workload."""
    import numpy as np
    m = min(1 << sample_log2, keys.numel())
    buf = np.ascontiguousarray(keys[:m].cpu().numpy().view(np.uint32))
    L = pylibsort.lib()
    c0 = time.perf_counter()
    if L.providedCpu(buf.ctypes.data, buf.size) != 1:
        raise RuntimeError("providedCpu failed: %s" % pylibsort.last_error())
    c1 = time.perf_counter()
    checked = m == keys.numel()
    if checked and not np.array_equal(buf, sorted_keys.cpu().numpy().view(np.uint32)):
        raise RuntimeError("providedCpu disagrees with the GPU sort")
    return {"value": round(m / (c1 - c0) / 1e9, 5), "unit": "Gkeys/s", "cores": 1, "kind": "port",
            "sample": "libsort providedCpu (std::sort, invokers.cu:68-71), 1 thread, on the first 2^%d keys of the "
                      "bench workload: %.2f s%s" % (sample_log2, c1 - c0,
                                                    "; output equal to the GPU sort" if checked else ""),
            "host_cpu": _cpu_model(), "nproc": os.cpu_count()}


def config_leg(torch, pylibsort, D, which, reps):
    """configs[2] (2^30 uint32 keys, 8-bit digits) or configs[4]'s per-GPU
    share (2^28 (u64 key, u32 payload) pairs, stable), timed like the main
    line with live per-kernel events; verified by sortedness + checksums
    (tests/test_gpu_parity.py pins both bit-exact)."""
    kind = {"c3": (30, 8), "c5": (28, 8)}[which]
    n = 1 << kind[0]
    prev = pylibsort.setDigitBits(kind[1])
    try:
        if which == "c3":
            keys = D.populate_u32(n)
            out, tmp = torch.empty_like(keys), torch.empty_like(keys)
            vals = None

            def step():
                return D.sort_keys_u32(keys, out=out, tmp=tmp)
        else:
            w = D.populate_u32(2 * n).view(n, 2).to(torch.int64)
            keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
            del w
            vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32)
            out, outv = torch.empty_like(keys), torch.empty_like(vals)
            tmp, tmpv = torch.empty_like(keys), torch.empty_like(vals)

            def step():
                return D.sort_pairs_u64_u32(keys, vals, out_keys=out, out_vals=outv, tmp_keys=tmp, tmp_vals=tmpv)
        settle(step, torch)
        D.timing_reset()
        D.timing_filter("tilepass")  # events around the pass only while timed (as the main line)
        D.timing_sample(3)           # every 3rd launch: rotates over the leg's two digit passes
        D.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            res = step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        D.timing_enable(False)
        launches, tms, _ = D.timing_query("tilepass")
        D.timing_reset()
        D.timing_sample(1)
        D.timing_filter(None)
        D.timing_enable(True)
        for _ in range(2):
            res = step()
        torch.cuda.synchronize()
        D.timing_enable(False)
        kern = {}
        for name in ("tilecounts", "colscan", "tilepass", "hybplan", "bucketsort"):
            launches_, ms_, _ = D.timing_query(name)
            if launches_:
                kern[name] = {"launches": launches_, "avg_us": round(1e3 * ms_ / launches_, 2),
                              "from": "2 steps after the timed ones"}
        if launches:
            kern["tilepass"] = {"launches": launches, "avg_us": round(1e3 * tms / launches, 2),
                                "from": "the timed steps"}
        ok = verify(torch, None, 1, keys, res, vals)
        ms = 1e3 * (t1 - t0) / reps
        unit_bytes = 24.0 if which == "c5" else 8.0
        tp = kern.get("tilepass")
        leg = {"ms_per_step": round(ms, 4), "value": round(n / (ms * 1e-3) / 1e9, 3),
               "unit": "Gpairs/s" if which == "c5" else "Gkeys/s", "verified": ok, "kernels": kern,
               "workload": ("configs[2]: 2^30 uint32 keys, 8-bit digits, full sort" if which == "c3" else
                            "configs[4] per-GPU share: 2^28 (u64 key, u32 payload) pairs, 8-bit digits, stable")}
        if tp:
            ach = unit_bytes * n / (tp["avg_us"] * 1e-6) / 1e9
            leg["scatter_roofline"] = {"achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                       "frac": round(ach / HBM_PEAK_GBPS, 4),
                                       "bytes_per_unit": unit_bytes}
            # cross-checks from this round's committed profiles (pairs: the
            # 16384-pair depth-0 and the 8192-pair table-depth passes)
            for name in (("c3_pass",) if which == "c3" else ("c5_pass_depth0", "c5_pass_table")):
                got = committed_leg(name)
                if got:
                    leg["scatter_roofline"].setdefault("committed", {})[name] = got
        bk = kern.get("bucketsort")
        if bk:
            ach = unit_bytes * n / (bk["avg_us"] * 1e-6) / 1e9
            bk["achieved_gbps"] = round(ach, 1)
            bk["frac"] = round(ach / HBM_PEAK_GBPS, 4)
            bk["bytes_per_unit"] = unit_bytes
            got = committed_leg("c3_bucket" if which == "c3" else "c5_bucket")
            if got:
                bk["committed"] = got
        if not ok:
            raise RuntimeError("%s leg failed verification" % which)
        return leg
    finally:
        pylibsort.setDigitBits(prev)
        torch.cuda.empty_cache()


# The reference's only published numbers are gpuPartial at 2^28 keys
# (analysis/libsort8b.csv:6-12, libsort16b.csv:6-12).
REF_PARTIAL = {8: {"kernels_gkeys_s": 0.361, "with_memcpy_gkeys_s": 0.193,
                   "source": "analysis/libsort8b.csv:6-12 (743.9 ms kernels, 1,392 ms with memcpy)"},
               16: {"kernels_gkeys_s": 0.182, "with_memcpy_gkeys_s": None,
                    "source": "analysis/libsort16b.csv:6-12 (1,475 ms kernels)"}}


def partial_leg(torch, pylibsort, D, keys, out, tmp, width, reps, calls=3):
    """gpuPartial at the reference's own benchmark workload
    (localTest/benchmarks.cpp:38-51,212-215: the first 2^28 PCG keys, offset
    0, width 16; libsort8b.csv is the same call at width 8).  Device-resident
    (libsortSortKeysU32 with d_boundaries: the stable partition + the 2^width
    group boundaries) with live per-kernel events, and the host ABI gpuPartial
    on a pageable buffer (PCIe-inclusive).  Checked: the output equals the
    input stably sorted by the group (torch.sort(stable=True) on the device),
    the boundaries equal the exclusive prefix of the group counts, and the
    host ABI returns the same data and boundaries."""
    import ctypes
    import numpy as np
    # the library's default digit width (8 bits: LIBSORT_DIGIT_BITS unset),
    # what gpuPartial callers get, not the 4-bit digits configs[1] names for
    # the full sort
    prev_bits = pylibsort.setDigitBits(8)
    try:
        return _partial_leg(torch, pylibsort, D, keys, out, tmp, width, reps, calls, ctypes, np)
    finally:
        pylibsort.setDigitBits(prev_bits)


def _partial_leg(torch, pylibsort, D, keys, out, tmp, width, reps, calls, ctypes, np):
    n = keys.numel()
    b = torch.empty(1 << width, dtype=torch.int32, device="cuda")

    def step():
        return D.sort_keys_u32(keys, out=out, tmp=tmp, offset=0, width=width, boundaries=b)
    settle(step, torch)
    D.timing_reset()
    D.timing_filter("tilepass")
    D.timing_sample(1)
    D.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.timing_enable(False)
    launches, tms, tk = D.timing_query("tilepass")
    D.timing_reset()
    D.timing_filter(None)
    D.timing_enable(True)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    D.timing_enable(False)
    kern = {}
    for name in ("tilecounts", "colscan", "tilepass", "onesweep", "whist", "bounds"):
        l_, ms_, _ = D.timing_query(name)
        if l_:
            kern[name] = {"launches": l_, "avg_us": round(1e3 * ms_ / l_, 2), "from": "2 steps after the timed ones"}
    if launches:
        kern["tilepass"] = {"launches": launches, "avg_us": round(1e3 * tms / launches, 2),
                            "keys_per_launch": tk / launches, "from": "the timed steps"}
    # checks (outside the timed region)
    mask = (1 << width) - 1
    grp = keys & mask
    _, idx = torch.sort(grp, stable=True)
    ok = bool(torch.equal(keys[idx], out))
    del idx
    cnt = torch.bincount(grp.to(torch.int64), minlength=1 << width)
    pref = torch.cumsum(cnt, 0) - cnt
    ok = ok and bool(torch.equal(pref.to(torch.int32), b))
    del grp, cnt, pref
    ms = 1e3 * (t1 - t0) / reps
    leg = {"call": "libsortSortKeysU32(d_keys, ..., offset 0, width %d, d_boundaries): device-resident gpuPartial"
                   % width,
           "ms_per_step": round(ms, 4), "value": round(n / (ms * 1e-3) / 1e9, 3), "unit": "Gkeys/s",
           "digit_bits": pylibsort.getDigitBits(), "kernels": kern, "verified": ok,
           "reference": dict(REF_PARTIAL[width], note="agpu1 (2 x 4 GiB GPUs, model unnamed), same call and keys")}
    leg["vs_reference_kernels"] = round(leg["value"] / REF_PARTIAL[width]["kernels_gkeys_s"], 1)
    tp = kern.get("tilepass")
    if tp and tp.get("keys_per_launch"):
        ach = 8.0 * tp["keys_per_launch"] / (tp["avg_us"] * 1e-6) / 1e9
        leg["pass_roofline"] = {"achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                "frac": round(ach / HBM_PEAK_GBPS, 4), "bytes_per_key": 8.0}
        got = committed_leg("partial_pass")
        if got:
            leg["pass_roofline"]["committed"] = got
    # the whole call against HBM: per digit pass one count read (4 B/key) and
    # the pass (8 B/key); the boundaries are 2^width words
    passes = -(-width // pylibsort.getDigitBits())
    step_bytes = n * 12.0 * passes
    leg["step_roofline"] = {"bytes_per_key": 12.0 * passes, "achieved": round(step_bytes / (ms * 1e-3) / 1e9, 1),
                            "frac": round(step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                            "note": "%d digit pass(es), each a 4 B/key count read + an 8 B/key pass" % passes}
    # host ABI (pageable buffer: H2D + partition + boundaries + D2H)
    src = keys.cpu().numpy()
    want = out.cpu().numpy()
    want_b = b.cpu().numpy().view(np.uint32).copy()
    buf = np.empty_like(src)
    bnd = (ctypes.c_uint32 * (1 << width))()
    L = pylibsort.lib()
    ts = []
    for _ in range(calls):
        np.copyto(buf, src)
        h0 = time.perf_counter()
        if L.gpuPartial(buf.ctypes.data, ctypes.addressof(bnd), buf.size, 0, width) != 1:
            raise RuntimeError("gpuPartial failed: %s" % pylibsort.last_error())
        ts.append(time.perf_counter() - h0)
    same = bool(np.array_equal(buf, want)) and bool(np.array_equal(np.frombuffer(bnd, dtype=np.uint32), want_b))
    t = sorted(ts)[len(ts) // 2]
    leg["host_abi"] = {"call": "gpuPartial (libsort.h, invokers.cu:15-41) on a pageable host buffer",
                       "ms": round(t * 1e3, 2), "value": round(n / t / 1e9, 3), "calls": calls,
                       "equal_to_device_result": same,
                       "note": "PCIe-inclusive (H2D + partition + boundaries + D2H), median of %d calls" % calls}
    if REF_PARTIAL[width]["with_memcpy_gkeys_s"]:
        leg["host_abi"]["vs_reference_with_memcpy"] = round(leg["host_abi"]["value"] /
                                                            REF_PARTIAL[width]["with_memcpy_gkeys_s"], 1)
    if not (ok and same):
        raise RuntimeError("partial%d leg failed verification (device %s, host ABI %s)" % (width, ok, same))
    return leg


def host_abi_leg(torch, pylibsort, keys, sorted_keys, calls=3):
    """the C-ABI end-to-end time (providedGpu on a
    pageable host buffer: H2D + sort + D2H), as the reference's callers see
    it.  Reported beside `value`, never as it; checked against the
    device-resident sort."""
    import numpy as np
    src = keys.cpu().numpy()
    want = sorted_keys.cpu().numpy()
    buf = np.empty_like(src)
    L = pylibsort.lib()
    ts = []
    for _ in range(calls):
        np.copyto(buf, src)
        t0 = time.perf_counter()
        if L.providedGpu(buf.ctypes.data, buf.size) != 1:
            raise RuntimeError("providedGpu failed: %s" % pylibsort.last_error())
        ts.append(time.perf_counter() - t0)
    if not np.array_equal(buf, want):
        raise RuntimeError("providedGpu disagrees with the device-resident sort")
    t = sorted(ts)[len(ts) // 2]
    return {"call": "providedGpu (libsort.h, invokers.cu:45-64) on a pageable host buffer", "ms": round(t * 1e3, 2),
            "value": round(keys.numel() / t / 1e9, 3), "unit": "Gkeys/s", "calls": calls,
            "note": "PCIe-inclusive (H2D + sort + D2H, median of %d calls), never `value`; "
                    "output checked equal to the device-resident sort" % calls}


def make_shards(torch, D, devs, n, pairs):
    """The C engine's input: shard r (on devs[r]) = the keys (pairs) rank r
    of the torch engine holds -- the populate stream's r-th block of n."""
    shards, vshards = [], []
    for rr, dv in enumerate(devs):
        if pairs:
            w = D.populate_u32(2 * n, first=rr * 2 * n, device=dv).view(n, 2).to(torch.int64)
            shards.append((w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF))
            del w
            vshards.append(torch.arange(rr * n, (rr + 1) * n, dtype=torch.int64,
                                        device=torch.device("cuda", dv)).to(torch.int32))
        else:
            shards.append(D.populate_u32(n, first=rr * n, device=dv))
    for dv in sorted(set(devs)):
        torch.cuda.synchronize(dv)
    return shards, vshards


def cabi_flags_for(D, schedule):
    return {"msdz": D.LIBSORT_DISTRIB_CODED, "lsd": D.LIBSORT_DISTRIB_LSD}.get(schedule, 0)


def cabi_probe_on(rehearsal):
    """The probe runs on a real multi-GPU node (distinct devices: the paths
    a one-GPU box never runs); BENCH_CABI_PROBE=1 / 0 forces it on / off."""
    v = os.environ.get("BENCH_CABI_PROBE")
    return v == "1" if v in ("0", "1") else not rehearsal


def run_cabi_probe(timeout):
    """Rank 0: `bench.py <same args> --cabi-probe` as a child process (never
    exec), its stderr (the engine's stage trace) passed through.  Returns
    (ok, note)."""
    import subprocess
    cmd = [sys.executable, str(pathlib.Path(__file__).resolve())] + sys.argv[1:] + ["--cabi-probe"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK")}
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    try:
        out, err = p.communicate(timeout=timeout)
        why = None if p.returncode == 0 else "exited with %d" % p.returncode
    except subprocess.TimeoutExpired:
        p.kill()
        out, err = p.communicate()
        why = "timed out after %.0f s (killed)" % timeout
    for ln in (err or "").splitlines()[-60:]:
        sys.stderr.write("bench.py [cabi probe]: %s\n" % ln)
    sys.stderr.flush()
    got = None
    for ln in (out or "").splitlines():
        if ln.startswith("{"):
            try:
                got = json.loads(ln)
            except ValueError:
                pass
    if why is None and not (got and got.get("cabi_probe") is True):
        why = "did not verify"
    dt = time.perf_counter() - t0
    if why:
        return False, "%s (%.1f s)" % (why, dt)
    return True, "verified in a child process: first step %.3f s, %.1f s with start-up" % (got["first_step_s"], dt)


def cabi_probe(args):
    """--cabi-probe (rank 0's child, no process group): ONE C-engine step over
    the line's shards on devices 0..N-1 with the stage trace on, verified
    like the parent's first step; prints one JSON line, exits 0 when it
    verified.  BENCH_CABI_PROBE_FAULT=hang|fail rehearses the parent's
    timeout / failure handling (tests only)."""
    fault = os.environ.get("BENCH_CABI_PROBE_FAULT")
    if fault == "hang":
        time.sleep(3600)
    import torch
    import pylibsort
    import pylibsort.device as D
    world = args.gpus
    devs = [0] * world if os.environ.get("BENCH_REHEARSAL") == "1" else list(range(world))
    pylibsort.setDigitBits(args.digit_bits)
    pairs = args.workload == "c5"
    shards, vshards = make_shards(torch, D, devs, 1 << args.keys_log2, pairs)
    pylibsort.lib().libsortSetDistribTrace(1)
    t0 = time.perf_counter()
    res = D.distrib_sort_pairs_u64_u32(shards, vshards) if pairs else D.distrib_sort_u32(
        shards, cabi_flags_for(D, args.schedule))
    for dv in sorted(set(devs)):
        torch.cuda.synchronize(dv)
    t1 = time.perf_counter()
    ok = verify_cabi(torch, shards, res, vshards if pairs else None) and fault != "fail"
    print(json.dumps({"cabi_probe": bool(ok), "first_step_s": round(t1 - t0, 3)}), flush=True)
    return 0 if ok else 1


def verify_cabi(torch, shards, res, vshards=None):
    """The C-ABI engine's result on rank 0: every output shard sorted (and,
    pairs, stable), the shards in order across their edges, the same
    multiset as the input shards (checksums over all devices)."""
    def csum(ts, vs=None):
        acc = [0, 0, 0]
        for i, t in enumerate(ts):
            if vs is None:
                k = t.to(torch.int64) & 0xFFFFFFFF
                acc[0] += int(k.sum())
                acc[1] += int((k * k % 1000000007).sum())
            else:
                v = vs[i].to(torch.int64) & 0xFFFFFFFF
                acc[0] += int((((t & 0xFFFFFF) * 1000003 + (t >> 40) * 7 + v) % 1000000007).sum())
                acc[1] += int(v.sum())
            acc[2] += t.numel()
        return acc
    if vshards is None:
        outs = res
        ok = csum(shards) == csum(outs)
        prev = None
        for t in outs:
            if t.numel() == 0:
                continue
            k = t.to(torch.int64) & 0xFFFFFFFF
            ok = ok and bool((k[1:] >= k[:-1]).all()) and (prev is None or prev <= int(k[0]))
            prev = int(k[-1])
        return ok
    ko, vo = res
    ok = csum(shards, vshards) == csum(ko, vo)
    prev = None
    flip = -(1 << 63)
    for k, v in zip(ko, vo):
        if k.numel() == 0:
            continue
        s_ = torch.bitwise_xor(k, torch.tensor(flip, dtype=torch.int64, device=k.device))
        vv = v.to(torch.int64) & 0xFFFFFFFF
        eq = s_[1:] == s_[:-1]
        ok = ok and bool((s_[1:] >= s_[:-1]).all()) and bool((vv[1:][eq] > vv[:-1][eq]).all())
        first = (int(s_[0]), int(vv[0]))
        ok = ok and (prev is None or prev[0] < first[0] or (prev[0] == first[0] and prev[1] < first[1]))
        prev = (int(s_[-1]), int(vv[-1]))
    return ok


def verify(torch, dist, world, keys, res, vals=None):
    """Sorted (unsigned order) on every rank and across shard edges, same
    multiset as the input (checksums); pairs: payloads increase within equal
    keys (stability; payload = global input index) and move with their keys."""
    if vals is None:
        r = res.to(torch.int64) & 0xFFFFFFFF
        k = keys.to(torch.int64) & 0xFFFFFFFF
        ok = bool((r[1:] >= r[:-1]).all().item()) if r.numel() > 1 else True
        sums = torch.stack([k.sum(), (k * k % 1000000007).sum(), torch.tensor(k.numel(), device=k.device)])
        rs = torch.stack([r.sum(), (r * r % 1000000007).sum(), torch.tensor(r.numel(), device=r.device)])
        z = torch.zeros(2, dtype=torch.int64, device="cuda")
        lo_hi = torch.stack([r[0], r[-1]]) if r.numel() else z
        first_last = lo_hi
    else:
        rk, rv = res
        flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=rk.device)
        s = torch.bitwise_xor(rk, flip)                       # uint64 order -> int64 order
        v = rv.to(torch.int64) & 0xFFFFFFFF
        ok = True
        if s.numel() > 1:
            ok = bool((s[1:] >= s[:-1]).all().item())
            eq = s[1:] == s[:-1]
            ok = ok and bool((v[1:][eq] > v[:-1][eq]).all().item())

        def mix(kk, vv):  # keys and payloads moved together
            return ((kk & 0xFFFFFF) * 1000003 + (kk >> 40) * 7 + vv) % 1000000007
        v0 = vals.to(torch.int64) & 0xFFFFFFFF
        sums = torch.stack([mix(keys, v0).sum(), v0.sum(), torch.tensor(keys.numel(), device=keys.device)])
        rs = torch.stack([mix(rk, v).sum(), v.sum(), torch.tensor(rk.numel(), device=rk.device)])
        z = torch.zeros(2, dtype=torch.int64, device="cuda")
        lo_hi = torch.stack([s[0], s[-1]]) if s.numel() else z
        first_last = torch.stack([v[0], v[-1]]) if v.numel() else z
    if world > 1:
        dist.all_reduce(sums)
        dist.all_reduce(rs)
        edge = torch.stack([lo_hi, first_last])
        allb = [torch.empty_like(edge) for _ in range(world)]
        dist.all_gather(allb, edge)
        edges = True
        for i in range(world - 1):
            a_hi, b_lo = int(allb[i][0][1]), int(allb[i + 1][0][0])
            if vals is None:
                edges = edges and a_hi <= b_lo
            else:  # key order, and payload order between equal keys across the shard edge
                edges = edges and (a_hi < b_lo or (a_hi == b_lo and int(allb[i][1][1]) < int(allb[i + 1][1][0])))
        okt = torch.tensor([1 if ok else 0], device="cuda")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item()) and edges
    return ok and bool(torch.equal(sums, rs))


if __name__ == "__main__":
    sys.exit(main() or 0)
