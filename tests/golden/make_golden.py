"""Regenerates tests/golden/vectors.npz from the oracle and checks every array
against the reference's recorded sha256 table (pcg_golden.json) first.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402  (test infrastructure)

HERE = pathlib.Path(__file__).resolve().parent


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u4").tobytes()).hexdigest()[:16]


def main():
    gold = json.loads((HERE / "pcg_golden.json").read_text())
    out = {}
    for n in (1021, 1111, 4099):
        x = oracle.pcg(n)
        s = oracle.sort_u32(x)
        assert sha16(x) == gold["sha256_prefix"][str(n)]["input"], n
        assert sha16(s) == gold["sha256_prefix"][str(n)]["sorted"], n
        out["in_%d" % n] = x
        out["sorted_%d" % n] = s
        for off, w in ((0, 8), (0, 4), (4, 8), (6, 4)):
            d, b = oracle.partial_u32(x, off, w)
            out["partial_%d_%d_%d" % (n, off, w)] = d
            out["bounds_%d_%d_%d" % (n, off, w)] = b
    np.savez_compressed(HERE / "vectors.npz", **out)
    print("wrote", HERE / "vectors.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
