"""FaaS data layer without a GPU: the file
distributed arrays written by pylibsort.data are byte-identical to what the
reference faasTest/pylibsort/data.py writes (fixtures recorded from it by
tests/golden/make_faas_golden.py), reference-written arrays read back, and
the worker's error paths answer like faasTest/f.py."""
import io
import json
import pathlib
import shutil

import numpy as np
import pytest

GOLD = pathlib.Path(__file__).resolve().parent / "golden" / "faas"


@pytest.fixture
def data(tmp_path):
    from pylibsort import data as D
    D.SetDistribMount(tmp_path)
    yield D
    D.closeOpenArrays()


def _files(p):
    return (p / "meta.json").read_bytes(), (p / "data.dat").read_bytes()


def test_write_output_matches_reference_bytes(data, tmp_path, golden):
    _, v = golden
    d, b = v["partial_1021_0_8"], v["bounds_1021_0_8"]
    req = {"offset": 0, "width": 8, "arrType": "file", "input": [], "output": "o"}
    data.writeOutput(req, bytearray(d.tobytes()), [int(x) for x in b])
    assert _files(tmp_path / "o") == _files(GOLD / "out_1021_w8")


def test_write_output_device_path_matches_reference_bytes(data, tmp_path, golden):
    import torch
    _, v = golden
    d, b = v["partial_1021_0_8"], v["bounds_1021_0_8"]
    req = {"offset": 0, "width": 8, "arrType": "file", "input": [], "output": "od"}
    data.writeOutputDevice(req, torch.from_numpy(d.view(np.int32)), torch.from_numpy(b.view(np.int32)))
    assert _files(tmp_path / "od") == _files(GOLD / "out_1021_w8")


def test_write_part_matches_reference_bytes(data, tmp_path):
    arr = data.fileDistribArray.Create(tmp_path / "p", data.ArrayShape.fromUniform(64, 2))
    arr.WritePart(0, bytes(range(40)))
    arr.WritePart(1, bytes(range(100, 124)))
    arr.Close()
    assert _files(tmp_path / "p") == _files(GOLD / "in_parts")


def test_reads_reference_array(data, tmp_path):
    shutil.copytree(GOLD / "in_parts", tmp_path / "in_parts")
    arr = data.fileDistribArray.Open(tmp_path / "in_parts")
    assert arr.shape.caps == [64, 64] and arr.shape.lens == [40, 24] and arr.shape.starts == [0, 64, 128]
    assert arr.ReadPart(0) == bytearray(range(40))
    assert arr.ReadPart(1, start=4, nbyte=8) == bytearray(range(104, 112))
    with pytest.raises(data.DistribArrayError):
        arr.ReadPart(1, start=20, nbyte=8)
    with pytest.raises(data.DistribArrayError):
        arr.WritePart(0, bytes(25))            # 40 + 25 > 64
    arr.WritePart(0, bytes(24))               # fills partition 0
    arr.Close()
    assert json.loads((tmp_path / "in_parts" / "meta.json").read_text()) == {"Lens": [64, 24], "Caps": [64, 64]}
    # requests reference partitions by name, -1 = whole used length (data.py:245-261)
    req = {"arrType": "file", "input": [{"arrayName": "in_parts", "partID": 1, "start": 0, "nbyte": -1},
                                        {"arrayName": "in_parts", "partID": 0, "start": 2, "nbyte": 3}]}
    got = bytes(data.readPartRefs(data.getPartRefs(req)))
    assert got == bytes(range(100, 124)) + bytes([2, 3, 4])


def test_write_all_read_all_and_shape(data, tmp_path):
    shape = data.ArrayShape.fromCaps([8, 0, 12])
    assert shape.starts == [0, 8, 8, 20] and shape.npart == 3
    arr = data.fileDistribArray.Create(tmp_path / "w", shape)
    with pytest.raises(data.DistribArrayError):
        arr.WriteAll(bytes(19))
    arr.WriteAll(bytes(range(20)))
    assert bytes(arr.ReadAll()) == bytes(range(20)) and arr.shape.lens == [8, 0, 12]
    arr.Close()
    arr.Destroy()
    assert not (tmp_path / "w").exists()


def test_worker_error_paths(data, monkeypatch):
    from pylibsort import faas
    assert faas.f({"arrType": "mem"}) == {"success": False,
                                          "err": "Function currently only supports file distributed arrays"}
    monkeypatch.delenv("OL_SHARED_VOLUME", raising=False)
    out = io.StringIO()
    assert faas.directInvoke([], stdin=io.StringIO("{}"), stdout=out) == 1
    assert "OL_SHARED_VOLUME" in json.loads(out.getvalue())["err"]
    monkeypatch.setenv("OL_SHARED_VOLUME", "/nonexistent")
    out = io.StringIO()
    assert faas.directInvoke([], stdin=io.StringIO("not json"), stdout=out) == 1
    assert json.loads(out.getvalue())["err"].startswith("Argument parsing error")


def test_bad_request_type(data):
    with pytest.raises(ValueError):
        data.getPartRefs({"arrType": "s3", "input": []})
    with pytest.raises(ValueError):
        data.getOutputArray({"arrType": "s3", "output": "x"}, data.ArrayShape.fromCaps([4]))
