#!/usr/bin/env python3
"""RCCL-only repro through torch.distributed (torch's bundled RCCL): one
rank, one batched self send/recv of 2^k bytes of uint64 (as int64), then
the received tensor compared with the sent one.  The companion of
tools/rccl_selfsend.cpp (the image's /opt/rocm RCCL, no torch).
    python tools/rccl_selfsend_torch.py <log2 bytes> [chunks]"""
import os
import sys


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29973")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    nbytes = 1 << int(sys.argv[1])
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n = nbytes // 8
    ver = torch.cuda.nccl.version()
    fails = 0
    for rep in range(3):
        src = (torch.arange(1, n + 1, dtype=torch.int64, device="cuda") * -7046029254386353131) ^ rep
        dst = torch.full_like(src, -6148914691236517206)
        per = -(-n // chunks)
        ops = []
        for o in range(0, n, per):
            ops.append(dist.P2POp(dist.isend, src[o:o + per], 0))
            ops.append(dist.P2POp(dist.irecv, dst[o:o + per], 0))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
        bad = (src != dst)
        nb = int(bad.sum())
        first = int(bad.nonzero()[0, 0]) if nb else -1
        print("torch RCCL %s self send/recv of %d MiB as %d message(s): %d of %d elements differ%s" % (
            ver, nbytes >> 20, chunks, nb, n,
            (", first at element %d (%.3f GiB)" % (first, first * 8 / 2**30)) if nb else ""), flush=True)
        fails += nb > 0
        del src, dst, bad
    dist.destroy_process_group()
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
