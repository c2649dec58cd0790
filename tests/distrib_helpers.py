"""Helpers for the multi-rank tests: an oracle-backed ops backend (test
infrastructure, CPU) with the same interface as pylibsort.distrib.HipOps, and
the per-rank worker run under torch.multiprocessing with gloo."""
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "gpu-radix-sort_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


class OracleOps:
    """CPU restatement of the local operations (checker, never the product)."""

    def __init__(self):
        import torch
        self.torch = torch
        from oracle import oracle
        self.o = oracle

    def _np(self, t):
        return t.numpy().view(np.uint32)

    def _t(self, a):
        return self.torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32).copy())

    def empty(self, n):
        return self.torch.empty(n, dtype=self.torch.int32)

    def empty64(self, n):
        return self.torch.empty(n, dtype=self.torch.int64)

    def sort_pairs(self, keys, vals, out_keys=None, out_vals=None):
        k, v = self.o.stable_sort_kv64(keys.numpy().view(np.uint64), vals.numpy().view(np.uint32))
        kt = self.torch.from_numpy(np.ascontiguousarray(k).view(np.int64).copy())
        vt = self._t(v)
        if out_keys is None:
            return kt, vt
        out_keys.copy_(kt)
        out_vals.copy_(vt)
        return out_keys, out_vals

    def partition_lut_pairs(self, keys, vals, lut, shift, nbuckets):
        k = keys.numpy().view(np.uint64)
        b = np.asarray(lut, dtype=np.uint8)[(k >> np.uint64(32 + shift)).astype(np.int64)].astype(np.int64)
        o = np.argsort(b, kind="stable")
        starts = np.concatenate([[0], np.cumsum(np.bincount(b, minlength=nbuckets))[:-1]])
        return (self.torch.from_numpy(k[o].view(np.int64).copy()), self._t(vals.numpy().view(np.uint32)[o]),
                starts.astype(np.int64))

    def sample_hi(self, keys, stride, block=4096):
        return self.sample(keys, stride, block).view(self.torch.int32)[1::2].contiguous()

    def sort(self, keys, out=None):
        res = self._t(self.o.sort_u32(self._np(keys)))
        if out is None:
            return res
        out.copy_(res)
        return out

    def partial_sort(self, keys, offset, width, out=None):
        d, b = self.o.partial_u32(self._np(keys), offset, width)
        return self._t(d), np.diff(b.astype(np.int64), append=keys.numel())

    def histogram(self, keys, shift, bits):
        x = self._np(keys)
        h = np.bincount((x >> np.uint32(shift)) & np.uint32((1 << bits) - 1), minlength=1 << bits)
        return self.torch.from_numpy(h.astype(np.int32))

    def partition(self, keys, splitters, out=None):
        x = self._np(keys)
        b = np.searchsorted(np.asarray(splitters, dtype=np.uint64), x.astype(np.uint64), side="right")
        return self._t(x[np.argsort(b, kind="stable")])

    def partition_lut(self, keys, lut, shift, nbuckets):
        x = self._np(keys)
        b = np.asarray(lut, dtype=np.uint8)[x >> np.uint32(shift)].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(np.bincount(b, minlength=nbuckets))[:-1]])
        return self._t(x[np.argsort(b, kind="stable")]), starts.astype(np.int64)

    def partition_lut_t(self, keys, lut, shift, nbuckets):
        out, starts = self.partition_lut(keys, lut.numpy(), shift, nbuckets)
        return out, self.torch.from_numpy(starts)

    def partition_lut_pairs_t(self, keys, vals, lut, shift, nbuckets):
        k, v, starts = self.partition_lut_pairs(keys, vals, lut.numpy(), shift, nbuckets)
        return k, v, self.torch.from_numpy(starts)

    # top-digit rounds (distrib.sort_msd / sort_msdz / pairs)
    def top_count_t(self, keys):
        x = self._np(keys)
        c = np.bincount(x >> np.uint32(24), minlength=256)
        return self.torch.from_numpy(np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64))

    def top_scatter_t(self, keys):
        x = self._np(keys)
        return self._t(x[np.argsort(x >> np.uint32(24), kind="stable")])

    def top_pairs_count_t(self, keys, vals):
        k = keys.numpy().view(np.uint64)
        c = np.bincount((k >> np.uint64(56)).astype(np.int64), minlength=256)
        return self.torch.from_numpy(np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64))

    def top_pairs_scatter_t(self, keys, vals):
        k = keys.numpy().view(np.uint64)
        o = np.argsort(k >> np.uint64(56), kind="stable")
        return self.torch.from_numpy(k[o].view(np.int64).copy()), self._t(vals.numpy().view(np.uint32)[o])

    # range digit (pylibsort.distrib.RangeDigit): digit = (key - bias) >> shift
    def minmax_t(self, keys):
        x = self._np(keys).astype(np.int64)
        return self.torch.tensor([x.min(), x.max()] if x.size else [0xFFFFFFFF, 0], dtype=self.torch.int64)

    def minmax64_t(self, keys):
        k = keys.numpy().view(np.uint64)
        mm = np.array([k.min(), k.max()] if k.size else [np.iinfo(np.uint64).max, 0], dtype=np.uint64)
        return self.torch.from_numpy(mm.view(np.int64).copy())

    def _rdig(self, x, rd, bits):
        if bits == 32:
            return ((x - np.uint32(rd.bias)) >> np.uint32(rd.shift)).astype(np.int64)
        return ((x - np.uint64(rd.bias)) >> np.uint64(rd.shift)).astype(np.int64)

    def range_count_t(self, keys, rd):
        d = self._rdig(self._np(keys), rd, 32)
        assert d.size == 0 or d.max() < 256, "range digit >= 256"
        c = np.bincount(d, minlength=256)
        return self.torch.from_numpy(np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64))

    def range_scatter_t(self, keys, rd):
        x = self._np(keys)
        return self._t(x[np.argsort(self._rdig(x, rd, 32), kind="stable")])

    def range_pairs_count_t(self, keys, vals, rd):
        d = self._rdig(keys.numpy().view(np.uint64), rd, 64)
        assert d.size == 0 or d.max() < 256, "range digit >= 256"
        c = np.bincount(d, minlength=256)
        return self.torch.from_numpy(np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64))

    def range_pairs_scatter_t(self, keys, vals, rd):
        k = keys.numpy().view(np.uint64)
        o = np.argsort(self._rdig(k, rd, 64), kind="stable")
        return self.torch.from_numpy(k[o].view(np.int64).copy()), self._t(vals.numpy().view(np.uint32)[o])

    def sort_pieces(self, keys, off, lens, segs, nseg, out, rd=None):
        """libsortSortPiecesU32's contract, checked: every key of a segment
        shares its top 8 bits (rd: its range digit) and those increase with
        the segment."""
        x = self._np(keys)
        parts, tops = [], []
        for o, ln, sg in zip(off, lens, segs):
            p = x[int(o):int(o) + int(ln)]
            if p.size:
                t = np.unique(p >> np.uint32(24) if rd is None else self._rdig(p, rd, 32))
                assert t.size == 1, "piece spans several top digits"
                tops.append((int(sg), int(t[0])))
            parts.append(p)
        assert all(a[1] - a[0] == tops[0][1] - tops[0][0] for a in tops), "segment != top digit - first digit"
        assert all(0 <= sg < nseg for sg in segs)
        res = np.sort(np.concatenate(parts)) if parts else np.empty(0, np.uint32)
        out.copy_(self._t(res))
        return out

    def sample(self, keys, stride, block=4096):
        nb = keys.numel() // block
        if stride <= 1 or nb < 4 * stride:
            return keys
        return keys[:nb * block].view(nb, block)[::stride].contiguous().view(-1)

    @staticmethod
    def _groups(x):
        ng = -(-x.size // 64)
        pad = np.zeros(ng * 64, dtype=np.int64)
        pad[:x.size] = x
        g = pad.reshape(ng, 64)
        gaps = np.zeros_like(g)
        gaps[:, 1:] = g[:, 1:] - g[:, :-1]
        valid = (np.arange(ng * 64) < x.size).reshape(ng, 64)
        gaps[~valid] = 0
        return g, gaps

    def delta_maxgap(self, keys, out):
        x = self._np(keys)
        m = int(self._groups(x)[1].max()) if x.size > 1 else 0
        out.numpy().view(np.uint32)[0] = m
        return out

    def delta_pack(self, keys, maxgap, out):
        x = self._np(keys)
        w = int(maxgap.numpy().view(np.uint32)[0]).bit_length()
        g, gaps = self._groups(x)
        words = list(g[:, 0].astype(np.uint32))
        for row in gaps:
            acc = 0
            for lane, v in enumerate(row):
                acc |= int(v) << (lane * w)
            words += [(acc >> (32 * q)) & 0xFFFFFFFF for q in range(2 * w)]
        o = out.numpy().view(np.uint32)
        o[:len(words)] = np.array(words, dtype=np.uint32)
        return out

    def delta_unpack(self, coded, n, bits, out):
        c = coded.numpy().view(np.uint32)
        ng = -(-n // 64)
        res = np.empty(ng * 64, dtype=np.uint64)
        for g in range(ng):
            acc = 0
            for q in range(2 * bits):
                acc |= int(c[ng + g * 2 * bits + q]) << (32 * q)
            run = int(c[g])
            for lane in range(64):
                run += (acc >> (lane * bits)) & ((1 << bits) - 1) if bits else 0
                res[g * 64 + lane] = run
        out.numpy().view(np.uint32)[:] = res[:n].astype(np.uint32)
        return out

    def merge(self, a, b, out):
        out.copy_(self._t(np.sort(np.concatenate([self._np(a), self._np(b)]))))
        return out

    def segment_copy(self, src, dst, so, do, ln):
        s = src.numpy()
        d = dst.numpy()
        for a, b, c in zip(so, do, ln):
            d[int(b):int(b + c)] = s[int(a):int(a + c)]
        return dst


def shard_inputs(x, R):
    """The reference's ceil(N/R) cut of one array into R shards."""
    N = x.size
    S = -(-N // R)
    return [x[min(N, r * S):min(N, (r + 1) * S)] for r in range(R)]


def rank_worker(rank, world, port, x, schedule, outdir, use_gpu, kw=None):
    """Runs distrib_sort on this rank's shard and saves the result."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from pylibsort import distrib
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = shard_inputs(x, world)[rank]
    kw = dict(kw or {})
    no_lsd = kw.pop("no_lsd", False)  # the LSD rounds must not run (range-digit tests)
    if use_gpu:
        torch.cuda.set_device(0)
        ops = distrib.HipOps()
        keys = torch.from_numpy(shard.view(np.int32).copy()).cuda()
    else:
        ops = OracleOps()
        keys = torch.from_numpy(shard.view(np.int32).copy())
    if no_lsd:
        def _forbidden(*a, **k):
            raise AssertionError("the LSD rounds ran (partial_sort) where the range digit should have")
        ops.partial_sort = _forbidden
    res = distrib.distrib_sort(keys, ops=ops, schedule=schedule, **kw)
    np.save(os.path.join(outdir, "rank%d.npy" % rank), res.cpu().numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


def pairs_worker(rank, world, port, k, outdir, use_gpu, kw=None):
    """distrib_sort_pairs on this rank's shard of (k, global index)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from pylibsort import distrib
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = k.size
    S = -(-N // world)
    lo, hi = min(N, rank * S), min(N, (rank + 1) * S)
    kt = torch.from_numpy(k[lo:hi].view(np.int64).copy())
    vt = torch.from_numpy(np.arange(lo, hi, dtype=np.uint32).view(np.int32).copy())
    kw = dict(kw or {})
    expect_range = kw.pop("expect_range", False)  # the range-digit re-partition must run
    if use_gpu:
        torch.cuda.set_device(0)
        ops = distrib.HipOps()
        kt, vt = kt.cuda(), vt.cuda()
    else:
        ops = OracleOps()
    ran = []
    if expect_range:
        inner = ops.range_pairs_count_t

        def counted(*a, **k_):
            ran.append(1)
            return inner(*a, **k_)
        ops.range_pairs_count_t = counted
    rk, rv = distrib.distrib_sort_pairs(kt, vt, ops=ops, **kw)
    assert not expect_range or ran, "the range-digit partition did not run"
    np.save(os.path.join(outdir, "k%d.npy" % rank), rk.cpu().numpy().view(np.uint64))
    np.save(os.path.join(outdir, "v%d.npy" % rank), rv.cpu().numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


def run_pair_ranks(k, world, tmpdir, use_gpu=False, port=29911, kw=None):
    import torch.multiprocessing as mp
    mp.spawn(pairs_worker, args=(world, port, k, str(tmpdir), use_gpu, kw), nprocs=world, join=True)
    return ([np.load(os.path.join(str(tmpdir), "k%d.npy" % r)) for r in range(world)],
            [np.load(os.path.join(str(tmpdir), "v%d.npy" % r)) for r in range(world)])


def run_ranks(x, world, schedule, tmpdir, use_gpu=False, port=29611, kw=None):
    import torch.multiprocessing as mp
    mp.spawn(rank_worker, args=(world, port, x, schedule, str(tmpdir), use_gpu, kw), nprocs=world, join=True)
    return [np.load(os.path.join(str(tmpdir), "rank%d.npy" % r)) for r in range(world)]
