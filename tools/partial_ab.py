#!/usr/bin/env python3
"""The bench's gpuPartial legs alone (bench.partial_leg: the reference's
workload, 2^28 PCG keys, offset 0, widths 8 and 16, device-resident and host
ABI) for an A/B of library builds (LIBSORT_PATH picks the build).
    [LIBSORT_PATH=build_ab/x.so] python tools/partial_ab.py [--no-host]"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import pylibsort
    import pylibsort.device as D
    import bench
    torch.cuda.set_device(0)
    n = 1 << 28
    keys = D.populate_u32(n)
    out, tmp = torch.empty_like(keys), torch.empty_like(keys)
    res = {"lib": pylibsort._state.path}
    for w in (8, 16):
        leg = bench.partial_leg(torch, pylibsort, D, keys, out, tmp, w, 10, calls=1 if "--no-host" not in sys.argv else 1)
        res["partial%d" % w] = {"ms": leg["ms_per_step"], "value": leg["value"],
                                "kernels": {k: v["avg_us"] for k, v in leg["kernels"].items()},
                                "pass_frac": leg.get("pass_roofline", {}).get("frac"), "verified": leg["verified"],
                                "host_ms": leg["host_abi"]["ms"]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
