"""The FaaS worker on the GPU: faasTest/f.py's
request flow -- input partitions read from file arrays, gpuPartial, output
array with one partition per radix group -- through pylibsort.faas.f (host
ABI, as the reference) and fDevice (device-resident sort, D2H into the mapped
output file).  The 1021-key case must reproduce, byte for byte, the array the
reference's own data layer writes for that input (tests/golden/faas)."""
import io
import json
import pathlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = pathlib.Path(__file__).resolve().parent / "golden" / "faas"


@pytest.fixture
def mount(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pylibsort import data as D
    D.SetDistribMount(tmp_path)
    yield tmp_path
    D.closeOpenArrays()


def _make_inputs(D, root, x, narr, npart, prefix):
    """x split over narr arrays of npart uniform partitions (f.py:86-107)."""
    raw = x.tobytes()
    per = len(raw) // (narr * npart)
    refs = []
    for a in range(narr):
        name = "%s%d" % (prefix, a)
        arr = D.fileDistribArray.Create(root / name, D.ArrayShape.fromUniform(per, npart))
        arr.WriteAll(raw[a * npart * per:(a + 1) * npart * per])
        arr.Close()
        refs += [{"arrayName": name, "partID": p, "start": 0, "nbyte": -1} for p in range(npart)]
    return refs


@pytest.mark.parametrize("handler", ["f", "fDevice"])
def test_worker_matches_reference_array(mount, oracle_mod, handler):
    from pylibsort import data as D
    from pylibsort import faas
    x = oracle_mod.pcg(1021)
    # 1021 keys do not split evenly: one array, one partition of the whole input
    refs = _make_inputs(D, mount, x, 1, 1, "in")
    req = {"offset": 0, "width": 8, "arrType": "file", "input": refs, "output": "out"}
    assert getattr(faas, handler)(req) == {"success": True, "err": ""}
    for f in ("meta.json", "data.dat"):
        assert (mount / "out" / f).read_bytes() == (GOLD / "out_1021_w8" / f).read_bytes(), f


@pytest.mark.parametrize("handler", ["f", "fDevice"])
@pytest.mark.parametrize("offset,width", [(0, 8), (8, 8), (0, 16), (5, 3)])
def test_worker_partial_sort(mount, oracle_mod, handler, offset, width):
    from pylibsort import data as D
    from pylibsort import faas
    n = 1 << 18
    x = oracle_mod.pcg(n, first=offset * 1000 + width)
    refs = _make_inputs(D, mount, x, 2, 2, "a")
    req = {"offset": offset, "width": width, "arrType": "file", "input": refs, "output": "o"}
    assert getattr(faas, handler)(req)["success"]
    out = D.fileDistribArray.Open(mount / "o")
    got = np.frombuffer(out.ReadAll(), dtype=np.uint32)
    d, b = oracle_mod.partial_u32(x, offset, width)
    np.testing.assert_array_equal(got, d)
    assert out.shape.caps == np.diff(b.astype(np.int64) * 4, append=4 * n).tolist()
    assert out.shape.lens == out.shape.caps
    out.Close()


def test_direct_invoke(mount, oracle_mod, monkeypatch):
    from pylibsort import data as D
    from pylibsort import faas
    x = oracle_mod.pcg(4096, first=3)
    refs = _make_inputs(D, mount, x, 2, 2, "d")
    monkeypatch.setenv("OL_SHARED_VOLUME", str(mount))
    req = {"offset": 4, "width": 4, "arrType": "file", "input": refs, "output": "dout"}
    out = io.StringIO()
    assert faas.directInvoke(["--device"], stdin=io.StringIO(json.dumps(req)), stdout=out) == 0
    assert json.loads(out.getvalue()) == {"success": True, "err": ""}
    got = np.fromfile(mount / "dout" / "data.dat", dtype=np.uint32)
    np.testing.assert_array_equal(got, oracle_mod.partial_u32(x, 4, 4)[0])


def test_worker_device_path_when_pylibsort_is_imported_first(tmp_path):
    """As faasTest/f.py does: import pylibsort, then the device handler needs
    torch on the GPU (fresh process, so the import order is real)."""
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    code = ("import sys; sys.path[:0] = [%r, %r]; import pylibsort; from pylibsort import data, faas; "
            "import numpy as np; from oracle import oracle; import pathlib; d = pathlib.Path(%r); "
            "data.SetDistribMount(d); x = oracle.pcg(100000); "
            "a = data.fileDistribArray.Create(d / 'in', data.ArrayShape.fromUniform(x.nbytes, 1)); "
            "a.WriteAll(x.tobytes()); a.Close(); "
            "r = faas.fDevice({'offset': 0, 'width': 8, 'arrType': 'file', "
            "'input': [{'arrayName': 'in', 'partID': 0, 'start': 0, 'nbyte': -1}], 'output': 'out'}); "
            "assert r['success'], r; "
            "assert np.array_equal(np.fromfile(d / 'out' / 'data.dat', dtype=np.uint32), oracle.partial_u32(x, 0, 8)[0]); "
            "print('OK')" % (str(root), str(root / "gpu-radix-sort_amd"), str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("handler", ["f", "fDevice"])
def test_distrib_worker_two_partrefs(mount, oracle_mod, handler):
    """The reference's DistribWorkerTest (benchmark/pkg/sort/testHelpers.go:
    324-388, run by distrib_test.go:14-24 as TestLocalDistribWorker /
    ...File): 1021 keys of a fresh generator stream written to one
    partition of array "initial"; the worker reads it as TWO PartRefs (bytes
    [0, 510*4) and [510*4, 1021*4) of partition 0) and partial-sorts their
    concatenation at offset 0, width 4.  The output array must have 16
    partitions holding all 4084 bytes, and reading them back in order gives
    the stable partition by the low 4 bits (checkPartial,
    testHelpers.go:411-448) -- here compared bit for bit with the oracle."""
    from pylibsort import data as D
    from pylibsort import faas
    n, width = 1021, 4
    x = oracle_mod.pcg(n)
    arr = D.fileDistribArray.Create(mount / "initial", D.ArrayShape.fromUniform(n * 4, 1))
    arr.WriteAll(x.tobytes())
    arr.Close()
    half = (n // 2) * 4
    refs = [{"arrayName": "initial", "partID": 0, "start": 0, "nbyte": half},
            {"arrayName": "initial", "partID": 0, "start": half, "nbyte": n * 4 - half}]
    req = {"offset": 0, "width": width, "arrType": "file", "input": refs, "output": "testDistribWorker"}
    assert getattr(faas, handler)(req) == {"success": True, "err": ""}
    out = D.fileDistribArray.Open(mount / "testDistribWorker")
    assert len(out.shape.lens) == 1 << width
    assert sum(out.shape.lens) == n * 4
    got = np.frombuffer(out.ReadAll(), dtype=np.uint32)
    d, b = oracle_mod.partial_u32(x, 0, width)
    np.testing.assert_array_equal(got, d)
    assert out.shape.lens == np.diff(b.astype(np.int64) * 4, append=4 * n).tolist()
    out.Close()
