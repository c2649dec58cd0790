#!/usr/bin/env python3
"""Diagnostics of the C-ABI pair engine (libsortDistribSortPairsU64U32) at
round sizes that take the pair hybrid (>= 2^25 pairs per round): sortedness,
stability and multiset of the result, R = 1 over RCCL and over device copies,
against the single-GPU pair sort of the same input.

    python tools/debug_pairs.py [log2_pairs]
"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import torch
    import pylibsort.device as D
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 27
    n = 1 << lg
    w = D.populate_u32(2 * n).view(n, 2).to(torch.int64)
    keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
    del w
    keys[: n // 64] = keys[: n // 64] & 0x7FF
    vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32)
    rk, rv = D.sort_pairs_u64_u32(keys, vals)
    torch.cuda.synchronize()
    for name, flags in (("rccl_self", 4), ("copy", 2), ("default", 0)):
        ko, vo = D.distrib_sort_pairs_u64_u32([keys], [vals], flags)
        k, v = ko[0], vo[0]
        same_k = bool(torch.equal(k, rk))
        same_v = bool(torch.equal(v, rv))
        info = {"case": name, "n": n, "keys_equal_single_gpu": same_k, "vals_equal_single_gpu": same_v}
        if not (same_k and same_v):
            bad = torch.nonzero((k != rk) | (v != rv)).flatten()
            info["mismatches"] = int(bad.numel())
            i = int(bad[0])
            info["first_bad"] = i
            info["got"] = [hex(int(x) & (2 ** 64 - 1)) for x in k[max(0, i - 2):i + 3].tolist()]
            info["want"] = [hex(int(x) & (2 ** 64 - 1)) for x in rk[max(0, i - 2):i + 3].tolist()]
            info["got_v"] = v[max(0, i - 2):i + 3].tolist()
            info["want_v"] = rv[max(0, i - 2):i + 3].tolist()
            info["top_digit_of_first_bad"] = (int(rk[i]) >> 56) & 0xFF
        print(info, flush=True)


if __name__ == "__main__":
    main()
