#!/usr/bin/env python3
"""Benchmark: uint32 full sort, keys resident in HBM (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N=1  : configs[1] = "256M uint32, 4-bit digits, gpuFullSort on 1 MI355X":
       2^28 keys of the reference populateInput stream (generated on the GPU by
       skip-ahead), one step = one full 32-bit LSD sort through the libsort C
       ABI (libsortSortKeysU32 = the device-resident form of providedGpu).
N>1  : launched by torch.distributed.run, one rank per GPU; rank r holds keys
       [r*2^28, (r+1)*2^28) of the same stream (weak scaling); one step = one
       distributed sort (pylibsort.distrib, "msd" schedule: one RCCL alltoallv)
       ending with rank r holding keys [r*S, (r+1)*S) of the sorted array.

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--keys-log2", type=int, default=28, help="keys per GPU = 2^k")
    ap.add_argument("--digit-bits", type=int, default=4, help="configs[1] names 4-bit digits")
    ap.add_argument("--schedule", default="msd", choices=["msd", "lsd"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log2", type=int, default=26)
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--algo", default=None, choices=["auto", "tiles", "onesweep", "rts"],
                    help="force the pass algorithm (LIBSORT_ALGO)")
    return ap.parse_args()


def main():
    args = parse()
    if args.algo:
        os.environ["LIBSORT_ALGO"] = args.algo
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus %d needs torch.distributed.run with %d processes" % (args.gpus, args.gpus))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import pylibsort
    import pylibsort.device as D
    from pylibsort import distrib

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    pylibsort.setDigitBits(args.digit_bits)

    n = 1 << args.keys_log2
    keys = D.populate_u32(n, first=rank * n)
    torch.cuda.synchronize()
    out = torch.empty_like(keys)
    tmp = torch.empty_like(keys)
    ops = distrib.HipOps() if world > 1 else None

    def step():
        if world == 1:
            return D.sort_keys_u32(keys, out=out, tmp=tmp)
        return distrib.distrib_sort(keys, ops=ops, schedule=args.schedule)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    barrier()

    D.timing_reset()
    D.timing_enable(True)
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
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # live per-kernel durations (hipEvents on libsort's launch stream)
    kern = {}
    for name in ("whist", "onesweep", "upsweep", "scan", "downsweep", "tilecounts", "colscan", "tilepass", "histogram", "segcopy"):
        launches, ms, kk = D.timing_query(name)
        if launches:
            kern[name] = {"launches": launches, "avg_us": 1e3 * ms / launches, "keys_per_launch": kk / launches}

    # verification outside the timed region: sorted + same multiset (checksums)
    verified = None
    if not args.no_verify:
        r64 = res.to(torch.int64) & 0xFFFFFFFF
        ok = bool((r64[1:] >= r64[:-1]).all().item()) if r64.numel() > 1 else True
        k64 = keys.to(torch.int64) & 0xFFFFFFFF
        sums = torch.stack([k64.sum(), (k64 * k64 % 1000000007).sum(), torch.tensor(k64.numel(), device=k64.device)])
        rs = torch.stack([r64.sum(), (r64 * r64 % 1000000007).sum(), torch.tensor(r64.numel(), device=r64.device)])
        lo_hi = torch.stack([r64[0], r64[-1]]) if r64.numel() else torch.zeros(2, dtype=torch.int64, device="cuda")
        if world > 1:
            dist.all_reduce(sums)
            dist.all_reduce(rs)
            # boundaries between neighbouring shards
            allb = [torch.empty_like(lo_hi) for _ in range(world)]
            dist.all_gather(allb, lo_hi)
            edges = all(int(allb[i][1]) <= int(allb[i + 1][0]) for i in range(world - 1))
            okt = torch.tensor([1 if ok else 0], device="cuda")
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
            ok = bool(okt.item()) and edges
        verified = ok and bool(torch.equal(sums, rs))

    total_keys = n * world
    ms_per_step = 1e3 * elapsed / args.steps
    value = total_keys / (elapsed / args.steps) / 1e9

    line = None
    if rank == 0:
        ds_name = next((k for k in ("tilepass", "onesweep", "downsweep") if k in kern), "downsweep")
        ds = kern.get(ds_name)
        roofline = None
        if ds:
            bytes_per_launch = 8.0 * ds["keys_per_launch"]  # read 4 B + write 4 B per key
            achieved = bytes_per_launch / (ds["avg_us"] * 1e-6) / 1e9
            traffic = None
            pmc = ROOT / "profiles" / ("pmc_%s.json" % ds_name)
            if pmc.exists():
                try:
                    traffic = json.loads(pmc.read_text()).get("hbm_bytes_per_launch")
                except Exception:
                    traffic = None
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                        "kernel": "k_%s (rank + scatter pass)" % ds_name, "algorithmic_bytes_per_launch": bytes_per_launch,
                        "avg_launch_us": round(ds["avg_us"], 2)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            from oracle import oracle  # CPU baseline leg only (the checker's std::sort)
            m = 1 << args.cpu_sample_log2
            x = oracle.pcg(m)
            c0 = time.perf_counter()
            oracle.lib().oracle_sort_u32(oracle._p32(x), x.size)
            c1 = time.perf_counter()
            cpu = {"value": round(m / (c1 - c0) / 1e9, 5), "unit": "Gkeys/s", "cores": 1, "kind": "port",
                   "sample": "std::sort (providedCpu, invokers.cu:68-71) of the first 2^%d populateInput keys, "
                             "1 thread, %.2f s" % (args.cpu_sample_log2, c1 - c0)}
        variants = {}
        if world == 1 and not args.no_variants:
            ref_out = out.clone()
            prev = pylibsort.setDigitBits(8)
            for _ in range(2):
                D.sort_keys_u32(keys, out=out, tmp=tmp)
            torch.cuda.synchronize()
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
        line = {
            "metric": "Gkeys/sec uint32 full sort",
            "value": round(value, 3),
            "unit": "Gkeys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: reference populateInput PCG32 stream, generated on device",
            "config": {"workload": "configs[1]: 2^%d uint32 keys per GPU, %d-bit digits, full sort%s"
                       % (args.keys_log2, args.digit_bits,
                          "" if world == 1 else ", %s schedule over %d GPUs (RCCL alltoallv)" % (args.schedule, world)),
                       "keys_per_gpu": n, "digit_bits": args.digit_bits, "global_keys": total_keys,
                       "parallelism": "shards%d" % world},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": kern,
            "verified": verified,
            "variants": variants or None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
