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

  partial:      the reference's own benchmark workload (localTest/benchmarks.cpp:
                38-51, 212-215: gpuPartialProfile of the first 2^28 keys of
                the stream, offset 0, width 16; analysis/libsort8b.csv is the
                same call at width 8): sha256 of the data after the stable
                partition (oracle_partial_u32, a counting sort) and of the
                2^width boundaries (exclusive prefix of the group counts), for
                widths 8 and 16; the reference's GetBoundaries quirk output
                (sort.cu:367-394, oracle_ref_boundaries) is checked equal to the
                prefix and the exact emulation of the reference's Step kernels
                (oracle_ref_step_u32) equal to the data first (group 1 is
                non-empty in both).

Run: python tests/golden/make_big_golden.py          (everything)
     python tests/golden/make_big_golden.py 2pow29   (adds the 2^29 class)
     python tests/golden/make_big_golden.py 2pow32   (adds the 2^32 stream)
     python tests/golden/make_big_golden.py partial  (adds the partial workload)
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


def add_partial():
    path = ROOT / "tests" / "golden" / "big_golden.json"
    out = json.loads(path.read_text())
    gold = json.loads((ROOT / "tests" / "golden" / "pcg_golden.json").read_text())["sha256_prefix"]
    for n in (1 << 20, 1 << 28):  # the pin first
        h = oracle.sorted_pcg_sha256(n)
        assert h[:16] == gold[str(n)]["sorted"], (n, h)
    n = 1 << 28
    x = oracle.pcg(n)
    assert hashlib.sha256(x.astype("<u4").tobytes()).hexdigest()[:16] == gold[str(n)]["input"]
    at = out.setdefault("partial_u32", {})
    for width in (8, 16):
        t = time.time()
        data, bounds = oracle.partial_u32(x, 0, width)
        ref_b = oracle.ref_boundaries(data, 0, width)
        assert np.array_equal(ref_b, bounds), "reference GetBoundaries quirk differs from the prefix"
        # the exact emulation of the reference's Step kernels (2-bit passes
        # over 128-key blocks, oracle_ref_step_u32) gives the same data
        emu = oracle.ref_step_u32(x, 0, width)
        assert np.array_equal(emu, data), "reference kernel emulation differs from the counting partition"
        del emu
        at["%d/0/%d" % (n, width)] = {
            "data": hashlib.sha256(data.astype("<u4").tobytes()).hexdigest(),
            "boundaries": hashlib.sha256(bounds.astype("<u4").tobytes()).hexdigest(),
            "boundaries_head": [int(v) for v in bounds[:4]],
            "boundaries_tail": [int(v) for v in bounds[-4:]],
        }
        print(width, at["%d/0/%d" % (n, width)], "%.0f s" % (time.time() - t), flush=True)
        del data
    path.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    if sys.argv[1:] == ["partial"]:
        add_partial()
    elif sys.argv[1:] == ["2pow29"]:
        add_2pow29()
    elif sys.argv[1:] == ["2pow32"]:
        add_2pow32()
    else:
        main()
