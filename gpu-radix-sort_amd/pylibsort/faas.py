"""FaaS sort worker -- the handler of the reference faasTest/f.py:46-70
(`f(event)`) and its command-line entry (`directInvoke`, f.py:150-182), over
this package's file distributed arrays and the MI355X libsort.

Request (JSON, same fields as benchmark/pkg/faas/inputs.go:13-33):
    {"offset": bit offset, "width": group bits, "arrType": "file",
     "input": [{"arrayName", "partID", "start", "nbyte"}, ...],
     "output": name of the array to create}
Response: {"success": bool, "err": str}.

f() follows the reference exactly: the referenced partitions are read into one
host buffer, partially sorted in place by gpuPartial, and written as an array
with one partition per radix group.  fDevice() produces the same output array
without host copies of the keys: each input piece goes host -> device straight
from the memory-mapped data.dat, the partial sort runs device-resident, and
one D2H lands in the mapped output data.dat.
"""
import json
import os
import pathlib
import sys

from . import data
from . import sort as _sort


def _fail(msg):
    return {"success": False, "err": msg}


def f(event):
    if event.get("arrType") != "file":
        return _fail("Function currently only supports file distributed arrays")
    raw = data.readPartRefs(data.getPartRefs(event))
    try:
        bounds = _sort.sortPartial(raw, event["offset"], event["width"])
    except Exception as e:  # the reference reports sort errors in the response (f.py:55-60)
        return _fail(str(e))
    data.writeOutput(event, raw, bounds)
    return {"success": True, "err": ""}


def fDevice(event):
    if event.get("arrType") != "file":
        return _fail("Function currently only supports file distributed arrays")
    import numpy as np
    import torch

    from . import device as D
    refs = data.getPartRefs(event)
    try:
        keys = _gather_to_device(refs, np, torch)
        width = int(event["width"])
        bounds = torch.empty(1 << width, dtype=torch.int32, device=keys.device)
        out = D.sort_keys_u32(keys, offset=int(event["offset"]), width=width, boundaries=bounds)
    except Exception as e:
        return _fail(str(e))
    data.writeOutputDevice(event, out, bounds)
    return {"success": True, "err": ""}


def _gather_to_device(refs, np, torch):
    """The referenced partition bytes, concatenated, as an int32 CUDA tensor:
    each piece is copied host -> device straight from the memory-mapped
    data.dat (no intermediate host buffer)."""
    total = sum(r.nbyte for r in refs)
    if total % 4:
        raise ValueError("input is not a whole number of uint32 keys")
    keys = torch.empty(total // 4, dtype=torch.int32, device="cuda")
    flat = keys.view(torch.uint8)
    pos = 0
    for r in refs:
        if r.nbyte == 0:
            continue
        used = r.arr.shape.lens[r.partID]
        if r.start < 0 or r.start + r.nbyte > used:
            raise data.DistribArrayError("Read beyond end of partition {}".format(r.partID))
        mm = np.memmap(r.arr.datPath, dtype=np.uint8, mode="c", offset=r.arr.shape.starts[r.partID] + r.start,
                       shape=(r.nbyte,))
        flat[pos:pos + r.nbyte].copy_(torch.from_numpy(np.asarray(mm)))
        del mm
        pos += r.nbyte
    return keys


def directInvoke(argv=None, stdin=None, stdout=None):
    """Reads one JSON request from stdin, prints the JSON response, exits 0 on
    success and 1 on failure.  OL_SHARED_VOLUME names the array directory."""
    stdin = sys.stdin if stdin is None else stdin
    stdout = sys.stdout if stdout is None else stdout
    mount = os.environ.get("OL_SHARED_VOLUME", "")
    if not mount:
        print(json.dumps(_fail("OL_SHARED_VOLUME not set, set it to the shared directory for distrib arrays")),
              file=stdout)
        return 1
    data.SetDistribMount(pathlib.Path(mount))
    try:
        cmd = json.loads(stdin.read())
    except Exception as e:
        print(json.dumps(_fail("Argument parsing error: " + str(e))), file=stdout)
        return 1
    handler = fDevice if (argv and "--device" in argv) else f
    resp = handler(cmd)
    data.closeOpenArrays()
    print(json.dumps(resp), file=stdout)
    return 0 if resp["success"] else 1


if __name__ == "__main__":
    sys.exit(directInvoke(sys.argv[1:]))
