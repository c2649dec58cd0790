"""Records the reference FaaS data layer's on-disk output as fixtures
(tests/golden/faas/): runs faasTest/pylibsort/data.py from /root/reference
(only its file-array code -- no libsort, no GPU) on small inputs and copies
the meta.json / data.dat files it writes.  The fixtures are data: inputs and
the reference's outputs; no reference source is stored.

    python tests/golden/make_faas_golden.py      (needs /root/reference)

Cases:
  out_1021_w8   the worker's output array for the 1021-key PCG input,
                offset 0, width 8: writeOutput(req, partially sorted bytes,
                boundaries) as faasTest/f.py:62 calls it (the sorted bytes and
                boundaries come from the oracle, pinned in vectors.npz)
  in_parts      an input array of 2 partitions of 64 B capacity, 40 B and
                24 B written with WritePart (Lens < Caps)
"""
import importlib.util
import json
import pathlib
import shutil
import sys
import tempfile
import types

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402  (test infrastructure)

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/faasTest/pylibsort/data.py")


def load_reference_data_module():
    pkg = types.ModuleType("refpylibsort")
    pkg.__path__ = []
    setattr(pkg, "__state", types.SimpleNamespace(sortLib=None))  # data.py imports it; unused here
    sys.modules["refpylibsort"] = pkg
    spec = importlib.util.spec_from_file_location("refpylibsort.data", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["refpylibsort.data"] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ref = load_reference_data_module()
    out = HERE / "faas"
    if out.exists():
        shutil.rmtree(out)
    out.mkdir()
    with tempfile.TemporaryDirectory() as t:
        t = pathlib.Path(t)
        ref.SetDistribMount(t)
        x = oracle.pcg(1021)
        d, b = oracle.partial_u32(x, 0, 8)
        req = {"offset": 0, "width": 8, "arrType": "file", "input": [], "output": "out_1021_w8"}
        ref.writeOutput(req, bytearray(d.tobytes()), [int(v) for v in b])
        arr = ref.fileDistribArray.Create(t / "in_parts", ref.ArrayShape.fromUniform(64, 2))
        arr.WritePart(0, bytes(range(40)))
        arr.WritePart(1, bytes(range(100, 124)))
        arr.Close()
        for name in ("out_1021_w8", "in_parts"):
            (out / name).mkdir()
            for f in ("meta.json", "data.dat"):
                shutil.copy(t / name / f, out / name / f)
    meta = json.loads((out / "out_1021_w8" / "meta.json").read_text())
    assert sum(meta["Caps"]) == 4 * 1021 and len(meta["Caps"]) == 256
    assert np.array_equal(np.fromfile(out / "out_1021_w8" / "data.dat", dtype=np.uint32), d)
    print("wrote", out)


if __name__ == "__main__":
    main()
