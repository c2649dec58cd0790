#!/usr/bin/env python3
"""GPU work of one rank of the delta-coded schedule (distrib.sort_msdz) at 2
ranks and 2^28 keys per rank, on one GPU: table partition into 2 x K
buckets, K round sorts of the round slices, gap coding of the piece for the
other rank, and (as if that piece had been received) its decode and the
merge with the own piece.  Prints the time of each piece and the coded size
against the raw size; the exchange itself (one xGMI link) is not here.
    python tools/msdz_parts.py [rounds]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]


def main():
    import numpy as np
    import torch
    import pylibsort
    import pylibsort.device as D
    from pylibsort import distrib
    pylibsort.setDigitBits(4)
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    R, r = 2, 0
    n = 1 << 28
    keys = D.populate_u32(n)
    ops = distrib.HipOps()
    row = D.plan_histogram_u32(keys)
    rows = torch.stack([row, row])
    lut_t, _ = D.plan_rounds(rows, R, K)
    lut = lut_t.cpu().numpy()
    NB = R * K

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    res = {}
    for rep in range(3):
        t = {}
        e0 = ev()
        part, starts = D.partition_lut_u32(keys, lut_t, 20, NB)
        e1 = ev()
        st = starts.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        sizes = np.diff(np.append(st, n))
        srt = torch.empty_like(keys)
        e2 = ev()
        for i in range(K):
            s0, s1 = int(st[i * R]), int(st[i * R]) + int(sizes[i * R:(i + 1) * R].sum())
            bk = np.nonzero((lut >= i * R) & (lut < (i + 1) * R))[0]
            ops.sort_range(part[s0:s1], int(bk[0]) << 20, (int(bk[-1]) + 1) << 20, out=srt[s0:s1])
        e3 = ev()
        mg = torch.zeros(NB, dtype=torch.int32, device="cuda")
        coded, raw_words = [], 0
        bufs = [torch.empty(D.delta_words(int(sizes[i * R + 1]), 32), dtype=torch.int32, device="cuda")
                for i in range(K)]
        e3 = ev()
        for i in range(K):
            j = i * R + 1
            D.delta_maxgap_u32(srt[int(st[j]):int(st[j]) + int(sizes[j])], out=mg[j:j + 1])
        e3b = ev()
        for i in range(K):
            j = i * R + 1
            piece = srt[int(st[j]):int(st[j]) + int(sizes[j])]
            coded.append(D.delta_pack_u32(piece, mg[j:j + 1], out=bufs[i]))
            raw_words += piece.numel()
        e4 = ev()
        m = mg.cpu().numpy().view(np.uint32)
        words = sum(D.delta_words(int(sizes[i * R + 1]), D.delta_bits(int(m[i * R + 1]))) for i in range(K))
        out = torch.empty_like(keys)
        pos = 0
        decs = [torch.empty(int(sizes[i * R + 1]), dtype=torch.int32, device="cuda") for i in range(K)]
        e5 = ev()
        for i in range(K):
            j1 = i * R + 1
            D.delta_unpack_u32(coded[i], int(sizes[j1]), D.delta_bits(int(m[j1])), out=decs[i])
        e5b = ev()
        for i in range(K):
            j0 = i * R
            own = srt[int(st[j0]):int(st[j0]) + int(sizes[j0])]
            D.merge_u32(own, decs[i], out=out[pos:pos + own.numel() + decs[i].numel()])
            pos += own.numel() + decs[i].numel()
        e6 = ev()
        torch.cuda.synchronize()
        t["partition"] = e0.elapsed_time(e1)
        t["round_sorts"] = e2.elapsed_time(e3)
        t["maxgap"] = e3.elapsed_time(e3b)
        t["pack"] = e3b.elapsed_time(e4)
        t["unpack"] = e5.elapsed_time(e5b)
        t["merge"] = e5b.elapsed_time(e6)
        res = t
    # one rank's view: each round's slice = its own piece merged with the
    # (here: its own outgoing) coded piece -> sorted within the round
    pos = 0
    for i in range(K):
        ln = int(sizes[i * R]) + int(sizes[i * R + 1])
        sl = out[pos:pos + ln].to(torch.int64) & 0xFFFFFFFF
        assert bool((sl[1:] >= sl[:-1]).all()), "round %d not sorted" % i
        pos += ln
    print({k: round(v, 3) for k, v in res.items()},
          "coded %.1f MB for %.1f MB raw (%.2f bits/key, gap widths %s)"
          % (words * 4 / 1e6, raw_words * 4 / 1e6, 32.0 * words / raw_words,
             [D.delta_bits(int(m[i * R + 1])) for i in range(K)]))


if __name__ == "__main__":
    main()
