#!/usr/bin/env python3
"""Interleaved A/B timing of libsort configurations in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Each config is "bits:algo:osblock".

    python tools/ab_sort.py --keys-log2 28 --rounds 5 --reps 5 8:onesweep:256 8:rts:256 ...
"""
import argparse
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--keys-log2", type=int, default=28)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kernels", action="store_true", help="also report per-kernel event times")
    a = ap.parse_args()
    import torch
    import pylibsort
    import pylibsort.device as D
    n = 1 << a.keys_log2
    keys = D.populate_u32(n)
    out = torch.empty_like(keys)
    tmp = torch.empty_like(keys)
    ref = None
    res = {c: [] for c in a.configs}
    kern = {c: {} for c in a.configs}

    def setup(c):
        f = c.split(":")
        bits, algo, blk = f[:3]
        pylibsort.setDigitBits(int(bits))
        pylibsort.setAlgorithm(algo)
        os.environ["LIBSORT_OS_BLOCK"] = blk
        os.environ["LIBSORT_TP_BLOCK"] = blk
        os.environ["LIBSORT_DIAG_ABLATION"] = f[3] if len(f) > 3 else "0"
        return len(f) > 3 and f[3] != "0"

    for c in a.configs:  # warm-up + correctness of every config
        diag = setup(c)
        D.sort_keys_u32(keys, out=out, tmp=tmp)
        torch.cuda.synchronize()
        if diag:
            continue
        h = out.cpu()
        if ref is None:
            ref = h
        assert torch.equal(h, ref), "config %s disagrees" % c
        assert pylibsort.lib().libsortDeviceErrors() == 0, c
    for r in range(a.rounds):
        for c in a.configs:
            setup(c)
            if a.kernels and r == a.rounds - 1:
                D.timing_reset()
                D.timing_enable(True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                D.sort_keys_u32(keys, out=out, tmp=tmp)
            torch.cuda.synchronize()
            res[c].append((time.perf_counter() - t0) / a.reps * 1e3)
            if a.kernels and r == a.rounds - 1:
                D.timing_enable(False)
                for k in ("whist", "onesweep", "upsweep", "scan", "downsweep", "tilecounts", "colscan", "tilepass"):
                    nl, ms, _ = D.timing_query(k)
                    if nl:
                        kern[c][k] = round(1e3 * ms / nl, 1)
    print("keys=2^%d" % a.keys_log2)
    for c in a.configs:
        med = statistics.median(res[c])
        print("%-18s median %.3f ms  min %.3f ms  %.1f Gkeys/s  %s" % (c, med, min(res[c]), n / med / 1e6,
                                                                   kern[c] or ""))
    assert pylibsort.lib().libsortDeviceErrors() == 0


if __name__ == "__main__":
    main()
