"""Golden sha256 of the configurations too large for the element-wise
oracle comparison (test_gpu_parity.py: test_config3_2pow30,
test_maximum_size, test_config5_pairs_size), computed with the oracle here
(minutes of CPU time), committed as tests/golden/big_golden.json.

  sorted keys:  oracle.sorted_pcg_sha256 -- std::sort (invokers.cu:68-71) of
                the populateInput stream (utils.cu:65-80) restated as a
                counting sort; pinned against the reference's own 2^20 and
                2^28 sorted hashes in pcg_golden.json before anything is written.
  C5 pairs:     std::stable_sort by key (oracle_stable_sort_kv64) of the
                bench/test pair construction: key_i = (draw 2i << 32) | draw
                2i+1, the first n/64 keys masked to 11 bits (many ties),
                payload_i = i.

  2^29 class:   the sorted hashes of the 2^29-class local sorts
                (test_gpu_hybrid.test_hybrid_auto_2pow29_class: n keys from
                element n of the stream) and of the 8-GPU per-rank shape
                (2^29 keys >> 3, test_gpu_distrib_abi.test_shape8_2pow29).

  2^32:         the sorted hash of the first 2^32 keys of the stream, i.e.
                configs[3]'s global input (rank r holds elements [r*2^29,
                (r+1)*2^29)): the concatenated output shards of the 8-rank
                engine (test_gpu_distrib_full.test_config3_full_8ranks).

Run: python tests/golden/make_big_golden.py          (everything)
     python tests/golden/make_big_golden.py 2pow29   (adds the 2^29 class)
     python tests/golden/make_big_golden.py 2pow32   (adds the 2^32 stream)
"""
import hashlib
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402


def c5_pairs(n):
    w = oracle.pcg(2 * n).astype(np.uint64).reshape(n, 2)
    keys = (w[:, 0] << np.uint64(32)) | w[:, 1]
    del w
    keys[: n // 64] &= np.uint64(0x7FF)
    vals = np.arange(n, dtype=np.uint32)
    return keys, vals


def main():
    gold = json.loads((ROOT / "tests" / "golden" / "pcg_golden.json").read_text())["sha256_prefix"]
    out = {"method": __doc__.strip().splitlines()[0], "sorted_u32": {}, "c5_pairs": {}}
    for n in (1 << 20, 1 << 28):           # pin the restatement on the reference's own hashes
        h = oracle.sorted_pcg_sha256(n)
        assert h[:16] == gold[str(n)]["sorted"], (n, h)
        print("pinned", n, h[:16], flush=True)
    for n in (1 << 30, (1 << 32) - 1):
        t = time.time()
        out["sorted_u32"][str(n)] = oracle.sorted_pcg_sha256(n)
        print(n, out["sorted_u32"][str(n)], "%.0f s" % (time.time() - t), flush=True)
    n = 1 << 28
    t = time.time()
    k, v = c5_pairs(n)
    k, v = oracle.stable_sort_kv64(k, v)
    out["c5_pairs"][str(n)] = {"keys": hashlib.sha256(k.astype("<u8").tobytes()).hexdigest(),
                               "payloads": hashlib.sha256(v.astype("<u4").tobytes()).hexdigest()}
    print("c5", out["c5_pairs"][str(n)], "%.0f s" % (time.time() - t), flush=True)
    (ROOT / "tests" / "golden" / "big_golden.json").write_text(json.dumps(out, indent=1) + "\n")


def add_2pow29():
    path = ROOT / "tests" / "golden" / "big_golden.json"
    out = json.loads(path.read_text())
    gold = json.loads((ROOT / "tests" / "golden" / "pcg_golden.json").read_text())["sha256_prefix"]
    h = oracle.sorted_pcg_sha256(1 << 20)  # the pin first
    assert h[:16] == gold[str(1 << 20)]["sorted"], h
    at = out.setdefault("sorted_u32_first", {})
    for n in ((1 << 29) + 12345, 400000007):
        t = time.time()
        at["%d@%d" % (n, n)] = oracle.sorted_pcg_sha256(n, first=n)
        print(n, at["%d@%d" % (n, n)], "%.0f s" % (time.time() - t), flush=True)
    sh = out.setdefault("sorted_u32_shift", {})
    n = 1 << 29
    t = time.time()
    sh["%d>>3" % n] = oracle.sorted_pcg_sha256(n, shift=3)
    print(n, ">> 3", sh["%d>>3" % n], "%.0f s" % (time.time() - t), flush=True)
    path.write_text(json.dumps(out, indent=1) + "\n")


def add_2pow32():
    path = ROOT / "tests" / "golden" / "big_golden.json"
    out = json.loads(path.read_text())
    gold = json.loads((ROOT / "tests" / "golden" / "pcg_golden.json").read_text())["sha256_prefix"]
    h = oracle.sorted_pcg_sha256(1 << 20)  # the pin first
    assert h[:16] == gold[str(1 << 20)]["sorted"], h
    n = 1 << 32
    t = time.time()
    out["sorted_u32"][str(n)] = oracle.sorted_pcg_sha256(n)
    print(n, out["sorted_u32"][str(n)], "%.0f s" % (time.time() - t), flush=True)
    path.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    if sys.argv[1:] == ["2pow29"]:
        add_2pow29()
    elif sys.argv[1:] == ["2pow32"]:
        add_2pow32()
    else:
        main()
