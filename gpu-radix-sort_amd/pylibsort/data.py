"""Distributed-array storage of the FaaS sort worker.

Same on-disk format and API names as the reference faasTest/pylibsort/data.py
(and the Go side benchmark/pkg/data/file.go:17-20,146-168): an array is a
directory holding

    meta.json   {"Lens": [bytes used per partition], "Caps": [bytes reserved]}
    data.dat    the partitions back to back, partition i at sum(Caps[:i])

so arrays written here are read by the reference's Go and Python code and
vice versa.  Deliberate differences (reference defects):
getOutputArray passes its shape (data.py:292-296 drops the argument), and
the output of a partial sort can be written straight from a device tensor
(writeOutputDevice: one D2H copy into the mapped data.dat, no intermediate
bytearray).
"""
import abc
import json
import mmap
import pathlib
import shutil

import numpy as np

__all__ = [
    "DistribArrayError", "SetDistribMount", "GetDistribMount", "ArrayShape", "DistribArray",
    "fileDistribArray", "partRef", "readPartRefs", "getPartRefs", "getOutputArray", "writeOutput",
    "writeOutputDevice", "closeOpenArrays",
]

_mount = [pathlib.Path("/shared")]  # default mount of file arrays (data.py:16)


class DistribArrayError(Exception):
    def __init__(self, cause):
        super().__init__(cause)
        self.cause = cause

    def __str__(self):
        return self.cause


def SetDistribMount(newRoot):
    """Directory under which request array names are resolved (default /shared)."""
    _mount[0] = pathlib.Path(newRoot)


def GetDistribMount():
    return _mount[0]


class ArrayShape:
    """Per-partition capacities and used lengths, in bytes; `starts` holds the
    byte offset of every partition plus a final entry = total capacity."""

    def __init__(self, caps, lens):
        self.caps = [int(c) for c in caps]
        self.lens = [int(n) for n in lens]
        if len(self.caps) != len(self.lens):
            raise DistribArrayError("caps and lens differ in length")
        self.npart = len(self.caps)
        self.starts = [0] + np.cumsum(self.caps, dtype=np.int64).tolist() if self.caps else [0]

    @classmethod
    def fromUniform(cls, cap, npart):
        return cls([cap] * npart, [0] * npart)

    @classmethod
    def fromCaps(cls, caps):
        return cls(caps, [0] * len(caps))


class DistribArray(abc.ABC):
    """Interface of a partitioned array (reference data.py:60-110, interface.go:74-99)."""
    shape = None

    @abc.abstractmethod
    def Close(self): ...

    @abc.abstractmethod
    def Destroy(self): ...

    @abc.abstractmethod
    def ReadPart(self, partID, start=0, nbyte=-1): ...

    @abc.abstractmethod
    def WritePart(self, partID, buf): ...

    @abc.abstractmethod
    def ReadAll(self): ...

    @abc.abstractmethod
    def WriteAll(self, buf): ...


class fileDistribArray(DistribArray):
    """File-backed array: <root>/meta.json + <root>/data.dat."""

    def __init__(self, rootPath):
        self.rootPath = pathlib.Path(rootPath)
        self.datPath = self.rootPath / "data.dat"
        self.metaPath = self.rootPath / "meta.json"
        self.closed = False
        self.dataF = None

    def _write_meta(self):
        with open(self.metaPath, "w") as f:
            json.dump({"Lens": self.shape.lens, "Caps": self.shape.caps}, f)

    @classmethod
    def Create(cls, rootPath, shape):
        arr = cls(rootPath)
        # world-writable, as the reference does for containers running as
        # another user (data.py:128-131)
        arr.rootPath.mkdir(0o777)
        arr.datPath.touch(0o666)
        arr.metaPath.touch(0o666)
        arr.shape = ArrayShape(shape.caps, shape.lens)
        arr.dataF = open(arr.datPath, "r+b")
        return arr

    @classmethod
    def Open(cls, rootPath):
        arr = cls(rootPath)
        if not arr.rootPath.exists():
            raise DistribArrayError("Array {} does not exist".format(rootPath))
        with open(arr.metaPath) as f:
            meta = json.load(f)
        arr.shape = ArrayShape(meta["Caps"], meta["Lens"])
        arr.dataF = open(arr.datPath, "r+b")
        return arr

    def Close(self):
        if self.closed:
            return
        self.dataF.close()
        self._write_meta()
        self.closed = True

    def Destroy(self):
        if not self.closed and self.dataF is not None:
            self.dataF.close()
            self.closed = True
        shutil.rmtree(self.rootPath)

    def ReadPart(self, partID, start=0, nbyte=-1, dest=None):
        used = self.shape.lens[partID]
        if nbyte == -1:
            nbyte = used - start
        if start < 0 or nbyte < 0 or start + nbyte > used:
            raise DistribArrayError("Read beyond end of partition {} (asked for {}+{}, limit {})".format(
                partID, start, nbyte, used))
        self.dataF.seek(self.shape.starts[partID] + start)
        if dest is None:
            return bytearray(self.dataF.read(nbyte))
        got = self.dataF.readinto(memoryview(dest)[:nbyte])
        if got != nbyte:
            raise DistribArrayError("short read of partition {}".format(partID))
        return None

    def WritePart(self, partId, buf):
        room = self.shape.caps[partId] - self.shape.lens[partId]
        if len(buf) > room:
            raise DistribArrayError("Wrote beyond end of partition (asked for {}b, limit {}b)".format(len(buf), room))
        self.dataF.seek(self.shape.starts[partId] + self.shape.lens[partId])
        self.dataF.write(buf)
        self.shape.lens[partId] += len(buf)

    def ReadAll(self):
        self.dataF.seek(0)
        return memoryview(self.dataF.read())

    def WriteAll(self, buf):
        total = self.shape.starts[-1]
        if len(buf) != total:
            raise DistribArrayError("Buffer length {}b does not match array capacity {}b".format(len(buf), total))
        self.dataF.seek(0)
        self.dataF.write(buf)
        self.shape.lens = list(self.shape.caps)

    def WriteAllDevice(self, tensor):
        """WriteAll from a contiguous CUDA (HIP) tensor: data.dat is sized and
        memory-mapped, and the tensor is copied device -> mapped file pages
        in one D2H transfer."""
        import torch
        total = self.shape.starts[-1]
        nbytes = tensor.numel() * tensor.element_size()
        if nbytes != total:
            raise DistribArrayError("Buffer length {}b does not match array capacity {}b".format(nbytes, total))
        self.dataF.truncate(total)
        self.dataF.flush()
        if total:
            mm = mmap.mmap(self.dataF.fileno(), total)
            try:
                host = torch.frombuffer(mm, dtype=torch.uint8)
                host.copy_(tensor.contiguous().view(torch.uint8).view(-1))
                del host
                mm.flush()
            finally:
                mm.close()
        self.shape.lens = list(self.shape.caps)


class partRef:
    """A byte range of one partition of an array (reference data.py:222-236)."""

    def __init__(self, arr, partID=0, start=0, nbyte=-1):
        self.arr = arr
        self.partID = partID
        self.start = start
        self.nbyte = nbyte

    def read(self, dest=None):
        return self.arr.ReadPart(self.partID, start=self.start, nbyte=self.nbyte, dest=dest)


# arrays opened by getPartRefs, keyed by name (one open file per array)
openArrs = {}


def _file_ref(req):
    name = req["arrayName"]
    arr = openArrs.get(name)
    if arr is None:
        arr = fileDistribArray.Open(GetDistribMount() / name)
        openArrs[name] = arr
    nbyte = req["nbyte"]
    if nbyte == -1:
        nbyte = arr.shape.lens[req["partID"]]
    return partRef(arr, partID=req["partID"], start=req["start"], nbyte=nbyte)


def readPartRefs(refs):
    """Concatenation of every ref's bytes in one buffer (a memoryview)."""
    out = memoryview(bytearray(sum(r.nbyte for r in refs)))
    pos = 0
    for r in refs:
        r.read(dest=out[pos:pos + r.nbyte])
        pos += r.nbyte
    return out


def getPartRefs(req):
    """partRefs of a sort request's "input" list (arrType "file")."""
    if req["arrType"] != "file":
        raise ValueError("Invalid request type: " + str(req["arrType"]))
    return [_file_ref(r) for r in req["input"]]


def getOutputArray(req, shape):
    """The file array named by req["output"], created with `shape`."""
    if req["arrType"] != "file":
        raise ValueError("Invalid request type: " + str(req["arrType"]))
    return fileDistribArray.Create(GetDistribMount() / req["output"], shape)


def _caps_from_boundaries(boundaries, nbytes):
    # bucket g spans [b[g], b[g+1]) elements; capacities in bytes (data.py:301-304)
    b = np.asarray(boundaries, dtype=np.int64) * 4
    return np.diff(b, append=nbytes).tolist()


def writeOutput(req, rawBytes, boundaries):
    """Write a partially sorted buffer as the output array: one partition per
    radix group, capacity = group size in bytes."""
    shape = ArrayShape.fromCaps(_caps_from_boundaries(boundaries, len(rawBytes)))
    arr = getOutputArray(req, shape)
    arr.WriteAll(rawBytes)
    arr.Close()


def writeOutputDevice(req, keys, boundaries):
    """writeOutput from device-resident sorted keys (uint32 in an int32 CUDA
    tensor) and their group boundaries (host sequence or tensor)."""
    if hasattr(boundaries, "cpu"):
        boundaries = boundaries.cpu().numpy().view(np.uint32)
    nbytes = keys.numel() * 4
    shape = ArrayShape.fromCaps(_caps_from_boundaries(boundaries, nbytes))
    arr = getOutputArray(req, shape)
    arr.WriteAllDevice(keys)
    arr.Close()


def closeOpenArrays():
    """Close every array getPartRefs opened (they stay open for reuse)."""
    for a in list(openArrs.values()):
        a.Close()
    openArrs.clear()
