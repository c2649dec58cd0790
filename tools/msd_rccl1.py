#!/usr/bin/env python3
"""Times the msd round schedule over a one-rank RCCL communicator at 2^28
keys (MSD_LG=29: 2^29; every step of the multi-GPU path except the network: sampled
histogram, partition, RCCL self all_to_all per round, per-round range sorts)
against the plain single-GPU sort.  python tools/msd_rccl1.py [rounds...]"""
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29994")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import pylibsort
    import pylibsort.device as D
    from pylibsort import distrib
    pylibsort.setDigitBits(4)
    ops = distrib.HipOps()
    n = 1 << int(os.environ.get("MSD_LG", "28"))  # keys per rank (29: configs[3]'s share)
    keys = D.populate_u32(n)
    if os.environ.get("MSD_SHAPE8") == "arith":  # rounds 1-3's variant (see below), for comparison
        keys >>= 3
    elif os.environ.get("MSD_SHAPE8") == "1":
        # the per-rank shape of an 8-GPU run on one rank: keep the top 5 bits
        # at 0, so the 2^29 keys fall in 32 top digits -- the 1/8 of the key
        # space one of 8 ranks receives; the rounds then hold ~8 digits of
        # ~2^24 keys each, as on every rank of configs[3] (the local
        # partition, which sees all 256 digits at 8 GPUs, is measured on the
        # uniform keys)
        # (a LOGICAL shift: the tensor is int32, and an arithmetic one put
        # the keys >= 2^31 in 16 top digits 0xF0-0xFF -- rounds 1-3's
        # "shape8" was that 48-digit variant)
        keys >>= 3
        keys &= 0x1FFFFFFF
    out = torch.empty_like(keys)
    tmp = torch.empty_like(keys)

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    if os.environ.get("MSD_PROFILE"):
        # for rocprofv3 --kernel-trace --stats: only the K = 4 schedule,
        # 2 warm-up + MSD_PROFILE timed steps (kernel totals / steps = the
        # GPU work of one step, by kernel)
        reps = int(os.environ["MSD_PROFILE"])
        cabi = os.environ.get("MSD_ENGINE") == "cabi"
        for _ in range(2 + reps):
            if cabi:
                D.distrib_sort_u32([keys], D.LIBSORT_DISTRIB_WIRE32 if os.environ.get("MSD_WIRE32") else 0)
            else:
                distrib.sort_msd(keys, ops, rounds=4)
        torch.cuda.synchronize()
        print({"msd_profile_steps": reps, "warmup": 2})
        dist.destroy_process_group()
        return
    res = {"plain_sort_ms": timed(lambda: D.sort_keys_u32(keys, out=out, tmp=tmp))}
    # at one rank the "self piece" of every round is the whole round (a
    # device copy of all n keys); at R ranks it is 1/R of the keys -- the
    # copy's own time is reported so it can be taken out of the schedule
    res["selfcopy_all_keys_ms"] = timed(lambda: out.copy_(keys))
    for K in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
        res["msd_rounds%d_selfcopy_ms" % K] = timed(lambda: distrib.sort_msd(keys, ops, rounds=K))
        res["msd_rounds%d_minus_selfcopy_ms" % K] = res["msd_rounds%d_selfcopy_ms" % K] - res["selfcopy_all_keys_ms"]
        res["msd_rounds%d_via_rccl_ms" % K] = timed(lambda: distrib.sort_msd(keys, ops, rounds=K, self_local=False))
    # the C-ABI engine (libsortDistribSortU32) on the same keys: one rank over
    # a one-device RCCL communicator, self pieces as device copies
    # (4-bit digits: the engine's default wire format is 24-bit planes, so
    # its self piece is a copy of 3 bytes per key; WIRE32 = 32-bit words)
    p16, q16 = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    p8, q8 = torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")
    res["selfcopy24_all_keys_ms"] = timed(lambda: (q16.copy_(p16), q8.copy_(p8)))
    del p16, q16, p8, q8
    res["cabi_rounds4_selfcopy_ms"] = timed(lambda: D.distrib_sort_u32([keys]))
    res["cabi_rounds4_minus_selfcopy_ms"] = res["cabi_rounds4_selfcopy_ms"] - res["selfcopy24_all_keys_ms"]
    res["cabi_wire32_selfcopy_ms"] = timed(lambda: D.distrib_sort_u32([keys], D.LIBSORT_DISTRIB_WIRE32))
    res["cabi_wire32_minus_selfcopy_ms"] = res["cabi_wire32_selfcopy_ms"] - res["selfcopy_all_keys_ms"]
    if os.environ.get("MSD_DIGIT8", "1") == "1":
        pylibsort.setDigitBits(8)
        res["digit8_msd_rounds4_selfcopy_ms"] = timed(lambda: distrib.sort_msd(keys, ops, rounds=4))
        pylibsort.setDigitBits(4)
    print({k: round(v, 3) for k, v in res.items()})
    for K in (1, 4):
        tr = []
        distrib.sort_msd(keys, ops, rounds=K, trace=tr)
        print("trace K=%d:" % K, ", ".join("%s %.3f ms" % (tr[i][0], 1e3 * (tr[i][1] - tr[i - 1][1]))
                                          for i in range(1, len(tr))))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
