"""Runs the multi-GPU round schedules over a real RCCL communicator of one
rank (RCCL refuses two ranks on one GPU): with self_local=False every piece
is a send/receive through RCCL, so the K asynchronous exchanges, their
stream-level waits and the per-round sorts go through RCCL's kernels and
stream as on 8 GPUs.  Invoked by
tests/test_gpu_distrib.py in a fresh process; prints OK on success."""
import os
import sys
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "gpu-radix-sort_amd")]

import numpy as np
import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29991")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import pylibsort.device as D
    from pylibsort import distrib
    ops = distrib.HipOps()
    n = (1 << 22) + 12345
    keys = D.populate_u32(n, first=99)
    ref = np.sort(keys.cpu().numpy().view(np.uint32))
    for rounds in (4, 1):
        out = distrib.sort_msd(keys, ops, rounds=rounds, self_local=False)  # self sends through RCCL
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref), "msd rounds=%d" % rounds
        out = distrib.sort_msdz(keys, ops, rounds=rounds)  # streams, coded widths gathered over RCCL
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref), "msdz rounds=%d" % rounds
        # the coded pieces through RCCL on the comm stream, decoded and merged
        # on the merge stream, widths gathered on the side stream
        out = distrib.sort_msdz(keys, ops, rounds=rounds, self_local=False)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref), "msdz self-send rounds=%d" % rounds
    rng = np.random.default_rng(3)
    m = (1 << 20) + 77
    k = rng.integers(0, 1 << 14, m, dtype=np.uint64) * np.uint64(0x0004000000000101)  # equal keys
    v = np.arange(m, dtype=np.uint32)
    kt = torch.from_numpy(k.view(np.int64)).cuda()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    rk, rv = distrib._sort_pairs_rounds(kt, vt, ops, None, 4, self_local=False)
    torch.cuda.synchronize()
    o = np.argsort(k, kind="stable")
    assert np.array_equal(rk.cpu().numpy().view(np.uint64), k[o]), "pairs keys"
    assert np.array_equal(rv.cpu().numpy().view(np.uint32), v[o]), "pairs payloads (stability)"
    dist.destroy_process_group()
    print("OK")


if __name__ == "__main__":
    main()
