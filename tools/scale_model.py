#!/usr/bin/env python3
"""Per-rank step model of the C engine's multi-GPU schedules at N = 2, 4, 8
(DESIGN.md section 7, round 6): the top-digit rounds (msd, 24-bit keys on
the wire, two partition parts across GPUs) and the gap-coded rounds (msdz:
sender sorts, coded exchange, receiver merges).

    python tools/scale_model.py [--json coded_shape.json ...]

The node is fully connected (an MI355X has 7 xGMI links, one per peer), so a
rank's (R-1)/R of its keys leave over R-1 links at once: the exchange of a
rank takes E = keys * bytes_per_key / (R * L) at L GB/s per link and
direction (the free variable).  GPU work per rank comes from the one-GPU
measurement of each schedule with R ranks sharing the GPU
(tools/coded_shape.py: step / R, device-copy exchanges) split by the kernel
trace into partition P, round sorts S (msdz: sender sorts + coding) and
merges M (msdz: decode + merge).  Timelines (events, per rank):
  msd   link: round i leaves once the partition is done (two parts: the first
        half's pieces of rounds 0-1 after half the partition) and round i-1
        has left; GPU: round i's sort starts when it has arrived and the
        previous sort is done.
  msdz  GPU: partition, then every round's sender sort + coding; link: round i
        leaves when it is coded and round i-1 has left; GPU: after the last
        coding, round i's decode + merge once it has arrived.
Value = R * 2^29 keys / step against the N = 1 line (2^28 keys per step at
the line's rate); weak scaling, so 2^29 keys per rank as the bench runs it.
"""
import argparse
import json

KEYS = 1 << 29
GROW = {"msd": 1.2, "msdz": 1.2}


def fracs(K, g):
    w = [g ** i for i in range(K)]
    t = sum(w)
    return [x / t for x in w]


def step_msd(R, L, P, S, wire_bytes=3.0, K=4, parts=2):
    f = fracs(K, GROW["msd"])
    E = KEYS * wire_bytes / (R * L * 1e9) * 1e3  # ms
    # two parts: rounds 0-1 may leave once the first half is scattered and the
    # second half counted (~0.65 P: count ~1/3 of P, scatter ~2/3), the rest
    # after the whole partition (a simplification of msd_model.py --parts 2)
    link = 0.65 * P if parts == 2 else P
    arrive = []
    for i in range(K):
        if parts == 1 or i >= 2:
            link = max(link, P)
        link += f[i] * E
        arrive.append(link)
    t = P
    for i in range(K):
        t = max(t, arrive[i]) + f[i] * S
    return t, E


def step_msdz(R, L, P, S, M, bits_per_key, K=4):
    f = fracs(K, GROW["msdz"])
    E = KEYS * bits_per_key / 8 / (R * L * 1e9) * 1e3
    t = P
    coded = []
    for i in range(K):
        t += f[i] * S
        coded.append(t)
    link = 0.0
    arrive = []
    for i in range(K):
        link = max(link, coded[i]) + f[i] * E
        arrive.append(link)
    for i in range(K):
        t = max(t, arrive[i]) + f[i] * M
    return t, E


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--n1", type=float, default=119.0, help="N = 1 line, Gkeys/s")
    ap.add_argument("--inputs", required=True, help="JSON: {R: {msd: {P, S}, msdz: {P, S, M, bits}}}")
    a = ap.parse_args()
    inp = json.loads(open(a.inputs).read())
    rates = (150, 100, 75, 50)
    print("| N | schedule | GPU work / rank | " + " | ".join("%d GB/s per link" % r for r in rates) + " |")
    print("|---|---|---|" + "---|" * len(rates))
    for R in sorted(inp, key=int):
        for sched in ("msd", "msdz"):
            d = inp[R].get(sched)
            if not d:
                continue
            cells = []
            for L in rates:
                if sched == "msd":
                    st, e = step_msd(int(R), L, d["P"], d["S"], wire_bytes=d.get("wire", 3.0))
                    work = d["P"] + d["S"]
                else:
                    st, e = step_msdz(int(R), L, d["P"], d["S"], d["M"], d["bits"])
                    work = d["P"] + d["S"] + d["M"]
                agg = int(R) * KEYS / (st * 1e-3) / 1e9
                cells.append("E %.2f, step %.2f ms, %.0f Gk/s = %.2fx" % (e, st, agg, agg / a.n1))
            print("| %s | %s | %.2f ms | %s |" % (R, sched, work, " | ".join(cells)))


if __name__ == "__main__":
    main()
