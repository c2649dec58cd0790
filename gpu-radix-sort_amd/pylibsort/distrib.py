"""Multi-GPU sort: one process per GPU, torch.distributed (RCCL over xGMI).

Replaces the reference's distributed drivers -- benchmark/pkg/sort/distrib.go:
90-248 (SortDistribFromArr: BSP LSD rounds, re-cut of the STRIDED bucket
stream into chunks of ceil(N/nworker) keys, distrib.go:113, helpers.go:67-121)
and localTest/benchmarks.cpp:70-160 (distribSort) -- whose "exchange" goes
through host memcpy or files, by device-resident rounds with one
all_to_all_single (alltoallv) per exchange.

Two schedules, identical final result (rank r holds keys [r*S, (r+1)*S) of the
globally sorted array, S = ceil(N/R), the reference's equal re-cut):

  "lsd"  the reference's BSP semantics: per `width`-bit digit, a stable local
         partial sort (gpuPartial on the device), an allgather of the per-rank
         bucket counts, one alltoallv of contiguous slices, and a segment
         gather into bucket-major / rank-minor order.  32/width exchanges.
  "msd"  range-split rounds: a (sampled) 12-bit histogram of the top key
         bits (allgather) assigns contiguous key ranges to (rank, round), R x K
         groups; ONE stable table partition (libsortPartitionLutU32) lays the
         keys out round-major / destination-minor; K alltoallv exchanges are
         issued at once (RCCL's stream runs them back to back) and round i is
         sorted into its final slice of the output as soon as it has arrived,
         overlapping the exchange of the later rounds.  The rounds are
         disjoint key ranges in increasing order, so no merge is needed.  A
         small alltoallv then shifts the few surplus keys to the neighbours so
         the shards are exact.  Falls back to "lsd" when one top-12-bit bucket
         is so large that a rank would receive more than `max_imbalance` x S
         keys.

The local operations come from an `ops` backend.  The product backend is
HipOps (libsort's HIP kernels on torch CUDA tensors).  The CPU tests pass an
oracle backend explicitly; nothing here falls back to the CPU on its own.
"""
import numpy as np
import torch
import torch.distributed as dist

HIST_BITS = 12


class HipOps:
    """Local operations on this rank's GPU through libsort.so."""

    def __init__(self, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("HipOps needs a HIP device")
        from . import device as D
        self.D = D
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        self._tmp = None

    def empty(self, n):
        return torch.empty(n, dtype=torch.int32, device=self.device)

    def empty64(self, n):
        return torch.empty(n, dtype=torch.int64, device=self.device)

    def _scratch64(self, n):
        if getattr(self, "_tmp64", None) is None or self._tmp64.numel() < n:
            self._tmp64 = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        return self._tmp64[:n]

    def _scratch(self, n):
        if self._tmp is None or self._tmp.numel() < n:
            self._tmp = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        return self._tmp[:n]

    def sort(self, keys, out=None):
        out = self.empty(keys.numel()) if out is None else out
        return self.D.sort_keys_u32(keys, out=out, tmp=self._scratch(keys.numel()))

    def partial_sort(self, keys, offset, width, out=None):
        """(sorted, per-bucket counts as host int64 numpy array)."""
        out = self.empty(keys.numel()) if out is None else out
        b = torch.empty(1 << width, dtype=torch.int32, device=self.device)
        self.D.sort_keys_u32(keys, out=out, tmp=self._scratch(keys.numel()), offset=offset,
                             width=width, boundaries=b)
        bounds = b.cpu().numpy().view(np.uint32).astype(np.int64)
        return out, np.diff(bounds, append=keys.numel())

    def histogram(self, keys, shift, bits):
        return self.D.histogram_u32(keys, shift, bits)

    def sort_range(self, keys, lo, hi, out=None):
        """Full sort of keys known to lie in [lo, hi) (fewer passes)."""
        out = self.empty(keys.numel()) if out is None else out
        return self.D.sort_keys_range_u32(keys, lo, hi, out=out, tmp=self._scratch(keys.numel()))

    def sort_pairs(self, keys, vals, out_keys=None, out_vals=None):
        """Stable sort of (uint64 key, uint32 payload) pairs."""
        n = keys.numel()
        ok_ = self.empty64(n) if out_keys is None else out_keys
        ov = self.empty(n) if out_vals is None else out_vals
        return self.D.sort_pairs_u64_u32(keys, vals, out_keys=ok_, out_vals=ov, tmp_keys=self._scratch64(n),
                                         tmp_vals=self._scratch(n))

    def partition(self, keys, splitters, out=None):
        out = self.empty(keys.numel()) if out is None else out
        return self.D.partition_u32(keys, splitters, out=out)[0]

    def partition_lut_pairs(self, keys, vals, lut, shift, nbuckets):
        """(keys, payloads, bucket starts as host int64) of the stable pair partition."""
        t = torch.from_numpy(np.ascontiguousarray(lut, dtype=np.uint8)).to(self.device)
        n = keys.numel()
        k, v, b = self.D.partition_lut_pairs_u64_u32(keys, vals, t, shift, nbuckets, out_keys=self.empty64(n),
                                                      out_vals=self.empty(n))
        return k, v, b.cpu().numpy().view(np.uint32).astype(np.int64)

    def sample_hi(self, keys, stride, block=4096):
        """High 32-bit words of a block sample of uint64 keys (little endian)."""
        return self.sample(keys, stride, block).view(torch.int32)[1::2].contiguous()

    def partition_lut(self, keys, lut, shift, nbuckets):
        """(partitioned keys, bucket starts as host int64 numpy array)."""
        t = torch.from_numpy(np.ascontiguousarray(lut, dtype=np.uint8)).to(self.device)
        out, b = self.D.partition_lut_u32(keys, t, shift, nbuckets, out=self.empty(keys.numel()))
        return out, b.cpu().numpy().view(np.uint32).astype(np.int64)

    def sample(self, keys, stride, block=4096):
        """Every `stride`-th block of `block` keys (all keys when few)."""
        nb = keys.numel() // block
        if stride <= 1 or nb < 4 * stride:
            return keys
        return keys[:nb * block].view(nb, block)[::stride].contiguous().view(-1)

    def segment_copy(self, src, dst, so, do, ln):
        return self.D.segment_copy_u32(src, dst, so, do, ln)


def _host_staged(group):
    """gloo cannot move HIP tensors: stage through host memory.  This is only
    for rehearsing several ranks on one GPU; RCCL ("nccl") moves device
    memory directly over xGMI."""
    return dist.get_backend(group) == "gloo"


def _allgather_np(vec, ref_tensor, group):
    """All-gather a small int64 numpy vector; returns [R, len] int64 numpy."""
    R = dist.get_world_size(group)
    dev = "cpu" if _host_staged(group) else ref_tensor.device
    t = torch.as_tensor(np.ascontiguousarray(vec, dtype=np.int64), device=dev)
    outs = [torch.empty_like(t) for _ in range(R)]
    dist.all_gather(outs, t, group=group)
    return np.stack([o.cpu().numpy() for o in outs])


def _alltoallv(send, send_counts, recv_counts, ops, group):
    """all_to_all_single with uneven splits (alltoallv): contiguous slices."""
    recv = ops.empty(int(np.sum(recv_counts)))
    rs = [int(c) for c in recv_counts]
    ss = [int(c) for c in send_counts]
    if _host_staged(group) and send.is_cuda:
        r_host = torch.empty(recv.numel(), dtype=recv.dtype)
        dist.all_to_all_single(r_host, send.cpu(), rs, ss, group=group)
        recv.copy_(r_host)
    else:
        dist.all_to_all_single(recv, send, rs, ss, group=group)
    return recv


def _alltoallv_into(recv, send, send_counts, recv_counts, group, async_op=False):
    """all_to_all_single into `recv`; returns the async work handle (or None).
    Device tensors over gloo (the one-GPU rehearsal) are staged through host
    memory synchronously; RCCL, and gloo on host tensors (the CPU tests), run
    the same issue-now / wait-later path as the 8-GPU job."""
    rs = [int(c) for c in recv_counts]
    ss = [int(c) for c in send_counts]
    if _host_staged(group) and send.is_cuda:
        r_host = torch.empty(recv.numel(), dtype=recv.dtype)
        dist.all_to_all_single(r_host, send.cpu(), rs, ss, group=group)
        recv.copy_(r_host)
        return None
    return dist.all_to_all_single(recv, send, rs, ss, group=group, async_op=async_op)


def shard_cut(N, R):
    """The reference's re-cut: chunks of ceil(N/R) keys (distrib.go:113)."""
    S = -(-N // R) if R else 0
    return S, [(min(N, r * S), min(N, (r + 1) * S)) for r in range(R)]


def _interval_counts(starts, lens, S, R):
    """counts[d] = sum_i |[starts[i], starts[i]+lens[i]) ∩ [d*S, (d+1)*S)| (last shard open-ended)."""
    out = np.zeros(R, dtype=np.int64)
    for d in range(R):
        lo = d * S
        hi = (d + 1) * S if d < R - 1 else np.iinfo(np.int64).max
        out[d] = np.clip(np.minimum(starts + lens, hi) - np.maximum(starts, lo), 0, None).sum()
    return out


def _rebalance(sorted_keys, n_all, ops, group):
    """Shift keys between ranks so rank r holds global positions [r*S, (r+1)*S)."""
    R = dist.get_world_size(group)
    r = dist.get_rank(group)
    N = int(n_all.sum())
    S, _ = shard_cut(N, R)
    offs = np.concatenate([[0], np.cumsum(n_all)[:-1]])
    M = np.stack([_interval_counts(np.array([offs[s]]), np.array([n_all[s]]), S, R)
                  for s in range(R)])                       # M[s, d]: keys s sends to d
    if np.array_equal(np.diag(M), n_all):
        return sorted_keys  # identical decision on every rank: nothing moves
    return _alltoallv(sorted_keys, M[r], M[:, r], ops, group)


def sort_lsd(keys, ops, group=None, width=8):
    """Reference BSP LSD schedule (distrib.go:90-179 semantics)."""
    R = dist.get_world_size(group)
    r = dist.get_rank(group)
    if 32 % width:
        raise ValueError("width must divide 32 (distrib.go:109)")
    nb = 1 << width
    cur = keys
    n_all = _allgather_np(np.array([cur.numel()]), cur, group)[:, 0]
    N = int(n_all.sum())
    S, _ = shard_cut(N, R)
    for step in range(32 // width):
        srt, cnt = ops.partial_sort(cur, step * width, width)
        C = _allgather_np(cnt, cur, group)                      # [R, nb]
        col = C.sum(axis=0)
        bstart = np.concatenate([[0], np.cumsum(col)[:-1]])     # global start of bucket b
        G = bstart[None, :] + np.cumsum(C, axis=0) - C          # [R, nb] start of (s, b)
        L = np.cumsum(C, axis=1) - C                            # [R, nb] local start of (s, b)
        send = _interval_counts(G[r], C[r], S, R)
        recv_counts = np.array([_interval_counts(G[s], C[s], S, R)[r] for s in range(R)])
        recv = _alltoallv(srt, send, recv_counts, ops, group)
        # segment table: the clipped (s, b) pieces for this rank, in the order
        # they arrive (source-major, bucket-minor), to bucket-major positions
        lo = r * S
        hi = (r + 1) * S if r < R - 1 else np.iinfo(np.int64).max
        so, do, ln = [], [], []
        recv_off = 0
        for s in range(R):
            g0 = G[s]
            cs = np.maximum(g0, lo)
            ce = np.minimum(g0 + C[s], hi)
            keep = ce > cs
            base = None
            for b in np.nonzero(keep)[0]:
                local_start = L[s][b] + (cs[b] - g0[b])
                if base is None:
                    base = local_start
                so.append(recv_off + (local_start - base))
                do.append(cs[b] - lo)
                ln.append(ce[b] - cs[b])
            recv_off += int(recv_counts[s])
        nxt = ops.empty(int(recv_counts.sum()))
        if so:
            ops.segment_copy(recv, nxt, np.array(so), np.array(do), np.array(ln))
        cur = nxt
    return cur


def plan_msd(H, R, hist_bits=HIST_BITS):
    """Bucket -> rank assignment from the gathered top-bit histograms H[R, 2^b].
    Returns (splitters, dest_of_bucket, n_recv_per_rank)."""
    G = H.sum(axis=0)
    N = int(G.sum())
    S, _ = shard_cut(N, R)
    cum = np.concatenate([[0], np.cumsum(G)[:-1]])
    mid = cum + G // 2
    dest = np.minimum(mid // max(S, 1), R - 1).astype(np.int64)
    dest = np.maximum.accumulate(dest)
    shift = 32 - hist_bits
    splitters = []
    for d in range(1, R):
        idx = np.nonzero(dest >= d)[0]
        if idx.size == 0:
            break
        splitters.append(int(idx[0]) << shift)
    n_recv = np.array([G[dest == d].sum() for d in range(R)], dtype=np.int64)
    return splitters, dest, n_recv


def plan_rounds(H, R, K, hist_bits=HIST_BITS, growth=1.6):
    """Contiguous top-bit bucket ranges for (rank, round) from the gathered
    (possibly sampled) histograms H[R, 2^b]: each rank gets about 1/R of the
    estimated keys, split into K rounds whose sizes grow by `growth` (a small
    first round keeps the exchange before the first sort short; each later
    round's exchange hides behind the previous round's sort).  Group of a
    bucket: rank g // K, round g % K.  Returns (lut, est_per_rank) with lut[b]
    = round * R + rank (the partition bucket)."""
    G = H.sum(axis=0).astype(np.float64)
    T = float(G.sum())
    if T > 0:
        x = (np.cumsum(G) - G / 2.0) / T * R                  # rank coordinate of each bucket's middle
        rank = np.minimum(x.astype(np.int64), R - 1)
        w = growth ** np.arange(K)
        cw = np.cumsum(w) / w.sum()
        rnd = np.minimum(np.searchsorted(cw, x - rank, side="right"), K - 1)
        grp = np.maximum.accumulate(rank * K + rnd)
    else:
        grp = np.zeros(G.size, dtype=np.int64)
    rank, rnd = grp // K, grp % K
    lut = (rnd * R + rank).astype(np.uint8)
    return lut, np.bincount(rank, weights=G, minlength=R)


def _group_range(lut, code, hist_bits=HIST_BITS):
    """[lo, hi) key range of the contiguous buckets with lut == code (None if empty)."""
    idx = np.nonzero(lut == code)[0]
    if idx.size == 0:
        return None
    shift = 32 - hist_bits
    return int(idx[0]) << shift, (int(idx[-1]) + 1) << shift


def sort_msd(keys, ops, group=None, max_imbalance=1.5, balance=True, rounds=4, sample_stride=16):
    """Range-split rounds schedule; see module docstring."""
    R = dist.get_world_size(group)
    r = dist.get_rank(group)
    K = max(1, min(int(rounds), 256 // R))
    n = keys.numel()
    h = ops.histogram(ops.sample(keys, sample_stride), 32 - HIST_BITS, HIST_BITS)
    hv = np.concatenate([h.cpu().numpy().astype(np.int64), [n]])
    HN = _allgather_np(hv, keys, group)                       # [R, 4096 + 1]
    H, n_all = HN[:, :-1], HN[:, -1]
    N = int(n_all.sum())
    S, _ = shard_cut(N, R)
    lut, est = plan_rounds(H, R, K)
    hs = float(H.sum())
    if N and hs and est.max() * N / hs > max_imbalance * S + 4096:
        return sort_lsd(keys, ops, group)
    NB = R * K
    part, b = ops.partition_lut(keys, lut, 32 - HIST_BITS, NB)
    sizes = np.diff(np.asarray(b, dtype=np.int64), append=n)    # bucket j = round * R + dest
    C = _allgather_np(sizes, keys, group)                      # [R, NB]
    recv_tot = np.array([int(C[:, i * R + r].sum()) for i in range(K)], dtype=np.int64)
    roff = np.concatenate([[0], np.cumsum(recv_tot)])
    recv = ops.empty(int(roff[-1]))
    out = ops.empty(int(roff[-1]))
    works = []
    for i in range(K):
        if not C[:, i * R:(i + 1) * R].any():                  # identical on every rank
            works.append(None)
            continue
        s0 = int(b[i * R])
        ss = sizes[i * R:(i + 1) * R]
        works.append(_alltoallv_into(recv[int(roff[i]):int(roff[i + 1])], part[s0:s0 + int(ss.sum())], ss,
                                     C[:, i * R + r], group, async_op=True))
    for i in range(K):
        if works[i] is not None:
            works[i].wait()                                    # stream-level: the sort waits on RCCL
        if recv_tot[i]:
            lo, hi = _group_range(lut, i * R + r)              # every key of the round lies in it
            ops.sort_range(recv[int(roff[i]):int(roff[i + 1])], lo, hi, out=out[int(roff[i]):int(roff[i + 1])])
    if not balance:
        return out
    n_recv = np.array([int(C[:, d::R].sum()) for d in range(R)], dtype=np.int64)
    return _rebalance(out, n_recv, ops, group)


def _rebalance_pairs(keys, vals, n_all, ops, group):
    """_rebalance for (key, payload) pairs: both arrays take the same splits."""
    R = dist.get_world_size(group)
    r = dist.get_rank(group)
    N = int(n_all.sum())
    S, _ = shard_cut(N, R)
    offs = np.concatenate([[0], np.cumsum(n_all)[:-1]])
    M = np.stack([_interval_counts(np.array([offs[s]]), np.array([n_all[s]]), S, R) for s in range(R)])
    if np.array_equal(np.diag(M), n_all):
        return keys, vals
    rk = ops.empty64(int(M[:, r].sum()))
    rv = ops.empty(int(M[:, r].sum()))
    _alltoallv_into(rk, keys, M[r], M[:, r], group)
    _alltoallv_into(rv, vals, M[r], M[:, r], group)
    return rk, rv


def distrib_sort_pairs(keys, vals, ops=None, group=None, rounds=4, sample_stride=16):
    """Stable sort of the distributed (uint64 key, uint32 payload) array whose
    rank-r shard is (keys, vals) -- SURVEY C5.  The "msd" range-split rounds of
    sort_msd on the top 12 bits of the key: one stable pair partition
    (libsortPartitionLutU64U32), per round an alltoallv of the keys and one of
    the payloads (issued up front, RCCL runs them back to back), a stable local
    pair sort of each round as it arrives, then the equal re-cut.  Equal keys
    keep their original global order: the partition and the local sort are
    stable and a round's data arrive in source-rank order.  There is no
    skew fallback: a heavy key range concentrates work on one rank, the result
    stays exact.  Returns this rank's (keys, vals) shard, ceil(N/R) pairs."""
    ops = HipOps() if ops is None else ops
    if dist.get_world_size(group) == 1:
        return ops.sort_pairs(keys, vals)
    return _sort_pairs_rounds(keys, vals, ops, group, rounds, sample_stride)


def _sort_pairs_rounds(keys, vals, ops, group, rounds, sample_stride):
    """The round schedule of distrib_sort_pairs (any world size)."""
    R = dist.get_world_size(group)
    r = dist.get_rank(group)
    K = max(1, min(int(rounds), 256 // R))
    n = keys.numel()
    h = ops.histogram(ops.sample_hi(keys, sample_stride), 32 - HIST_BITS, HIST_BITS)
    HN = _allgather_np(np.concatenate([h.cpu().numpy().astype(np.int64), [n]]), keys, group)
    H = HN[:, :-1]
    lut, _ = plan_rounds(H, R, K)
    NB = R * K
    pk, pv, b = ops.partition_lut_pairs(keys, vals, lut, 32 - HIST_BITS, NB)
    sizes = np.diff(np.asarray(b, dtype=np.int64), append=n)
    C = _allgather_np(sizes, keys, group)
    recv_tot = np.array([int(C[:, i * R + r].sum()) for i in range(K)], dtype=np.int64)
    roff = np.concatenate([[0], np.cumsum(recv_tot)])
    T = int(roff[-1])
    rk, rv, ok_, ov = ops.empty64(T), ops.empty(T), ops.empty64(T), ops.empty(T)
    works = []
    for i in range(K):
        if not C[:, i * R:(i + 1) * R].any():
            works.append(())
            continue
        s0, ss = int(b[i * R]), sizes[i * R:(i + 1) * R]
        a, z = int(roff[i]), int(roff[i + 1])
        works.append((_alltoallv_into(rk[a:z], pk[s0:s0 + int(ss.sum())], ss, C[:, i * R + r], group, async_op=True),
                      _alltoallv_into(rv[a:z], pv[s0:s0 + int(ss.sum())], ss, C[:, i * R + r], group, async_op=True)))
    for i in range(K):
        for w in works[i]:
            if w is not None:
                w.wait()
        a, z = int(roff[i]), int(roff[i + 1])
        if z > a:
            ops.sort_pairs(rk[a:z], rv[a:z], out_keys=ok_[a:z], out_vals=ov[a:z])
    n_recv = np.array([int(C[:, d::R].sum()) for d in range(R)], dtype=np.int64)
    return _rebalance_pairs(ok_, ov, n_recv, ops, group)


def distrib_sort(keys, ops=None, group=None, schedule="msd", **kw):
    """Sort the distributed uint32 array whose rank-r shard is `keys`.
    Returns this rank's shard of the sorted array (ceil(N/R) keys per rank)."""
    ops = HipOps() if ops is None else ops
    if dist.get_world_size(group) == 1:
        return ops.sort(keys)
    if schedule == "msd":
        return sort_msd(keys, ops, group, **kw)
    if schedule == "lsd":
        return sort_lsd(keys, ops, group, **kw)
    raise ValueError("schedule must be 'msd' or 'lsd'")


__all__ = ["HipOps", "distrib_sort", "distrib_sort_pairs", "sort_lsd", "sort_msd", "plan_msd", "plan_rounds",
           "shard_cut"]
