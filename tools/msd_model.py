#!/usr/bin/env python3
"""Per-rank step model of the 8-GPU top-digit schedule.

    python tools/msd_model.py [--partition-ms 1.22] [--gpu-ms 5.00] [--n1 121.5] [--wire-bytes 3]

The step is the partition (exposed), round 0's exchange, then each round
the longer of its sort and the next round's exchange, then the last sort.
Inputs are the measured one-GPU numbers of the 8-GPU shape (tools/msd_rccl1.py
MSD_SHAPE8=1: GPU work per rank without the self copy, the partition's part
of it) and the N = 1 bench line; the per-GPU send rate is the free variable.
A per-round overhead (the round sort's small kernels) is kept fixed when the
round profile changes.

--parts 2: the partition in two parts (round 5, distrib.cpp partition_top):
count and scatter of the first half, count of the second (the plan needs
both counts), scatter of the second; the links carry the first half's pieces
of rounds 0 and 1 from the plan on, then the second half's, then rounds 2..
(event timeline: link and compute stream, a round sorted once it has arrived
and the previous sort is done).
"""
import argparse

KEYS_PER_RANK = 1 << 29


def sent_bytes(wire_bytes):
    """bytes a rank sends at 8 GPUs (7/8 of its keys; 4 B per key as 32-bit
    words, 3 B with the 24-bit wire format of round 5)"""
    return 7 / 8 * KEYS_PER_RANK * wire_bytes

PROFILES = {
    "K4 x1.2 (built)": [1, 1.2, 1.44, 1.728],
    "K4 flat": [1, 1, 1, 1],
    "K4 x0.8": [1, 0.8, 0.64, 0.512],
    "K5 hump": [0.6, 1, 1, 0.9, 0.5],
    "K6 hump": [0.5, 0.9, 1, 1, 0.8, 0.4],
}


def step_ms(weights, rate_gbs, part_ms, sorts_ms, per_round_ms, built_rounds=4, wire_bytes=3):
    t = sum(weights)
    f = [w / t for w in weights]
    e = sent_bytes(wire_bytes) / (rate_gbs * 1e9) * 1e3
    body = sorts_ms - built_rounds * per_round_ms
    s = [x * body + per_round_ms for x in f]
    k = len(f)
    return part_ms + f[0] * e + sum(max(s[i], f[i + 1] * e) for i in range(k - 1)) + s[-1], e


def step_parts_ms(weights, rate_gbs, count_ms, scatter_ms, sorts_ms, per_round_ms, parts, built_rounds=4,
                  wire_bytes=3):
    t = sum(weights)
    f = [w / t for w in weights]
    e = sent_bytes(wire_bytes) / (rate_gbs * 1e9) * 1e3
    body = sorts_ms - built_rounds * per_round_ms
    s = [x * body + per_round_ms for x in f]
    k = len(f)
    P = count_ms + scatter_ms
    arrive = [0.0] * k
    if parts == 1:
        link = P
        for i in range(k):
            link += f[i] * e
            arrive[i] = link
    else:
        part0 = count_ms / 2 + scatter_ms / 2
        link = part0 + count_ms / 2  # the plan (both halves counted)
        early = min(k, 2)
        for i in range(early):
            link += f[i] * e / 2
        link = max(link, P)
        for i in range(early):
            link += f[i] * e / 2
            arrive[i] = link
        for i in range(early, k):
            link += f[i] * e
            arrive[i] = link
    done = P
    for i in range(k):
        done = max(done, arrive[i]) + s[i]
    return done, e


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--partition-ms", type=float, default=1.22)
    ap.add_argument("--gpu-ms", type=float, default=5.00, help="GPU work per rank, 8-GPU shape")
    ap.add_argument("--per-round-ms", type=float, default=0.13)
    ap.add_argument("--n1", type=float, default=121.5, help="N = 1 line, Gkeys/s (BENCH_r04)")
    ap.add_argument("--wire-bytes", type=float, default=3.0, help="bytes per key on the links (4: 32-bit words)")
    ap.add_argument("--count-ms", type=float, default=0.40, help="the partition's count (r05g trace)")
    ap.add_argument("--parts", type=int, default=0, help="1 or 2: event timeline with that many partition parts")
    a = ap.parse_args()
    if a.parts:
        sorts = a.gpu_ms - a.partition_ms
        for name, w in PROFILES.items():
            if not name.startswith("K4 x1.2"):
                continue
            cells = []
            for rate in (700, 450, 400, 360, 300):
                st, e = step_parts_ms(w, rate, a.count_ms, a.partition_ms - a.count_ms, sorts, a.per_round_ms, a.parts,
                                      wire_bytes=a.wire_bytes)
                agg = 8 * KEYS_PER_RANK / (st * 1e-3) / 1e9
                cells.append("%d GB/s: E %.2f step %.2f ms %.0f Gk/s %.2fx" % (rate, e, st, agg, agg / a.n1))
            print("%-16s parts %d  %s" % (name, a.parts, " | ".join(cells)))
        return
    sorts = a.gpu_ms - a.partition_ms
    for name, w in PROFILES.items():
        cells = []
        for rate in (700, 450, 400, 360, 300):
            st, e = step_ms(w, rate, a.partition_ms, sorts, a.per_round_ms, wire_bytes=a.wire_bytes)
            agg = 8 * KEYS_PER_RANK / (st * 1e-3) / 1e9
            cells.append("%d GB/s: E %.2f step %.2f ms %.0f Gk/s %.2fx" % (rate, e, st, agg, agg / a.n1))
        print("%-16s %s" % (name, " | ".join(cells)))


if __name__ == "__main__":
    main()
