#!/usr/bin/env python3
"""Measurements of the SURVEY §8(f) rows beside the bench line (one MI355X):
  row 4  64-bit keys-only sort and (u64 key, u64 payload) stable sort,
         device-resident, 4- and 8-bit digits, checked sorted / stable (the
         MSD hybrid serves both: "passes" are the LSD sort's, for scale);
  row 3  the FaaS worker (pylibsort.faas): f() (host buffers through
         gpuPartial, as faasTest/f.py) against fDevice() (keys stay in HBM
         between the sort and the mapped output file), arrays on tmpfs.
Prints one line per measurement.  python tools/bench_rows.py [4] [3]"""
import pathlib
import shutil
import sys
import tempfile
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def timed(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def row4():
    import torch
    import pylibsort
    import pylibsort.device as D
    n = 1 << 28
    w = D.populate_u32(2 * n).view(n, 2).to(torch.int64)
    keys = (w[:, 0] << 32) | (w[:, 1] & 0xFFFFFFFF)
    del w
    out, tmp = torch.empty_like(keys), torch.empty_like(keys)
    flip = torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")
    for bits in (8, 4):
        pylibsort.setDigitBits(bits)
        t = timed(lambda: D.sort_keys_u64(keys, out=out, tmp=tmp))
        s = torch.bitwise_xor(out, flip)
        ok = bool((s[1:] >= s[:-1]).all())
        passes = 64 // bits
        print("u64 keys 2^28, %d-bit digits: %.3f ms = %.2f Gkeys/s (%d LSD-equivalent passes, %.0f GB/s per pass) "
              "sorted=%s" % (bits, t * 1e3, n / t / 1e9, passes, 16.0 * n * passes / t / 1e9, ok))
    del out, tmp
    m = 1 << 27
    k = keys[:m].contiguous()
    del keys
    k[m // 64: m // 32] = k[: m // 64]                            # ties: stability is visible
    v = torch.arange(m, dtype=torch.int64, device="cuda")
    ok_, ov, tk, tv = (torch.empty_like(k), torch.empty_like(v), torch.empty_like(k), torch.empty_like(v))
    for bits in (8, 4):
        pylibsort.setDigitBits(bits)
        t = timed(lambda: D.sort_pairs_u64_u64(k, v, out_keys=ok_, out_vals=ov, tmp_keys=tk, tmp_vals=tv))
        s = torch.bitwise_xor(ok_, flip)
        eq = s[1:] == s[:-1]
        ok = bool((s[1:] >= s[:-1]).all()) and bool((ov[1:][eq] > ov[:-1][eq]).all())
        passes = 64 // bits
        print("u64+u64 pairs 2^27, %d-bit digits: %.3f ms = %.2f Gpairs/s (%.0f GB/s per LSD-equivalent pass) "
              "sorted+stable=%s" % (bits, t * 1e3, m / t / 1e9, 32.0 * m * passes / t / 1e9, ok))


def rowp():
    """(u32 key, u32 payload) stable pairs, 2^28, PCG keys, LSD vs the MSD hybrid."""
    import torch
    import pylibsort
    import pylibsort.device as D
    n = 1 << 28
    k = D.populate_u32(n)
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    ok_, ov, tk, tv = (torch.empty_like(k), torch.empty_like(v), torch.empty_like(k), torch.empty_like(v))
    flip = torch.tensor(-(1 << 31), dtype=torch.int32, device="cuda")
    for bits in (4, 8):
        pylibsort.setDigitBits(bits)
        for mode in ("off", "auto"):
            prev = pylibsort.setHybrid(mode)
            t = timed(lambda: D.sort_pairs_u32_u32(k, v, out_keys=ok_, out_vals=ov, tmp_keys=tk, tmp_vals=tv))
            pylibsort.setHybrid(prev)
            s = torch.bitwise_xor(ok_, flip)
            ok = bool((s[1:] >= s[:-1]).all()) and bool((k[ov.to(torch.int64)] == ok_).all())
            print("u32+u32 pairs 2^28, %d-bit digits, hybrid %s: %.3f ms = %.2f Gpairs/s sorted+paired=%s"
                  % (bits, mode, t * 1e3, n / t / 1e9, ok))


def row3():
    import numpy as np
    from pylibsort import data, faas
    from oracle import oracle
    n = 1 << 26
    x = oracle.pcg(n)
    root = pathlib.Path(tempfile.mkdtemp(dir="/dev/shm" if pathlib.Path("/dev/shm").exists() else None))
    try:
        data.SetDistribMount(root)
        raw = x.tobytes()
        per = len(raw) // 4
        refs = []
        for a in range(2):
            arr = data.fileDistribArray.Create(root / ("in%d" % a), data.ArrayShape.fromUniform(per, 2))
            arr.WriteAll(raw[a * 2 * per:(a + 1) * 2 * per])
            arr.Close()
            refs += [{"arrayName": "in%d" % a, "partID": p, "start": 0, "nbyte": -1} for p in range(2)]
        d_ref, _ = oracle.partial_u32(x, 0, 8)
        for name, fn in (("f (host buffers, gpuPartial)", faas.f), ("fDevice (HBM-resident)", faas.fDevice)):
            ts = []
            for i in range(4):
                req = {"offset": 0, "width": 8, "arrType": "file", "input": refs, "output": "o%d" % i}
                t0 = time.perf_counter()
                resp = fn(req)
                assert resp["success"], resp["err"]
                ts.append(time.perf_counter() - t0)
                data.closeOpenArrays()
            got = np.fromfile(root / "o3" / "data.dat", dtype=np.uint32)
            print("FaaS worker %s, 2^26 keys w8 from tmpfs: %.1f ms per request (%.2f Gkeys/s), output==oracle: %s"
                  % (name, 1e3 * min(ts[1:]), n / min(ts[1:]) / 1e9, bool(np.array_equal(got, d_ref))))
            for i in range(4):
                shutil.rmtree(root / ("o%d" % i))
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    rows = sys.argv[1:] or ["4", "3"]       # e.g. `python tools/bench_rows.py 4`
    if "4" in rows:
        row4()
    if "3" in rows:
        row3()
    if "p" in rows:
        rowp()
