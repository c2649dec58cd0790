#!/usr/bin/env python3
"""Timing only (no check): one 8-bit LSD digit pass (gpuPartial width 8,
device-resident, 2^28 keys) over different inputs, to separate the pass's
cost from the input it reads: the PCG populate stream, a torch.randint
stream, and the populate stream already sorted on its low byte (pass over
bits 8-15, as the second pass of a width-16 sort sees it).  Each phase
prints its per-call pass times, so a slow phase shows whether it is slow
throughout or only at first.  Run under A/B builds with LIBSORT_PATH.
python tools/lsd_pass_input_ab.py [reps]"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.cuda.set_device(0)
    pylibsort.setDigitBits(8)
    n = 1 << 28
    pcg = D.populate_u32(n)
    rnd = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda")
    low = torch.empty_like(pcg)
    tmp = torch.empty_like(pcg)
    out = torch.empty_like(pcg)
    b = torch.empty(256, dtype=torch.int32, device="cuda")
    D.sort_keys_u32(pcg, out=low, tmp=tmp, offset=0, width=8, boundaries=b)
    res = {"lib": pylibsort._state.path.split("/")[-1]}
    D.timing_filter("tilepass")
    for name, src, off in (("pcg", pcg, 0), ("randint", rnd, 0), ("pcg_hi", low, 8),
                           ("pcg_again", pcg, 0), ("pcg_3", pcg, 0)):
        def step():
            D.sort_keys_u32(src, out=out, tmp=tmp, offset=off, width=8, boundaries=b)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        per = []
        for _ in range(reps):
            D.timing_reset()
            D.timing_enable(True)
            step()
            torch.cuda.synchronize()
            D.timing_enable(False)
            l, tms, _ = D.timing_query("tilepass")
            per.append(round(1e3 * tms / max(l, 1)))
        res[name] = {"mean": round(sum(per) / len(per), 1), "per": per}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
