"""Multi-GPU sharding of the encode and decode paths (one process per GPU).

The sketch is additive: S_k(A ⊎ B) = S_k(A) + S_k(B) mod p
and counts add, so the id stream is cut into contiguous shards, one per rank,
each rank encodes its shard into a partial vector on its own GPU, and ONE
sum-reduce of the partial words (RCCL over xGMI with backend "nccl"; gloo in
the CPU tests) merges them on rank 0.  Partial words are canonical residues
(< 2^32, limbs for the u64 field) stored as uint64, so the integer sum of up
to 2^27 ranks cannot overflow; rank 0 folds the sum mod p.  last_value comes
from the last non-empty shard, which rank 0 learns without communication
(shards are contiguous and their sizes are known to every rank).

Decode shards the same way: rank 0 turns the merged
difference into coefficients (O(t^2), host), ONE broadcast ships
[d, stop flag, stop value, c_1..c_d] to every rank, each rank root-tests its
contiguous log shard on its own GPU (`root_test_shard`, which also reports
where the stop value first occurs in the shard), ONE all-reduce(MIN) finds
the global stop position (the caller's `break` at media_client.rs:307-309
applies to the whole log), and the hit positions — offset by the shard base
and cut at the global stop — are all-gathered (two small collectives: counts,
then the padded positions).  Every rank returns the same ascending list,
identical to the single-GPU root test of the whole log.
"""
from __future__ import annotations

import numpy as np

from ._lib import P32, P64


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, start+count) of rank in a stream of n_total."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def reduce_words(threshold: int, bits: int) -> int:
    """Number of leading partial words that are summed across ranks."""
    return threshold + 1 if bits == 32 else 2 * threshold + 1


def state_to_partial(q) -> np.ndarray:
    """Partial-vector image (include/quack_hip.h) of a host sketch; used by the
    CPU multi-rank tests, where each rank encodes with the host path."""
    t = q.threshold()
    S = q.power_sums()
    if q.BITS == 32:
        out = np.zeros(t + 2, dtype=np.uint64)
        out[:t] = S
        out[t] = q.count()
        out[t + 1] = q.last_value() or 0
    else:
        out = np.zeros(2 * t + 2, dtype=np.uint64)
        for k, v in enumerate(S):
            out[2 * k] = v & 0xFFFFFFFF
            out[2 * k + 1] = v >> 32
        out[2 * t] = q.count()
        out[2 * t + 1] = q.last_value() or 0
    return out


def fold_partial_sum(words, threshold: int, bits: int) -> tuple[list, int]:
    """(canonical power sums, wrapping count) from a summed partial."""
    w = [int(v) for v in np.asarray(words).astype(np.uint64)]
    if bits == 32:
        return [v % P32 for v in w[:threshold]], w[threshold] & 0xFFFFFFFF
    S = [(w[2 * k] + (w[2 * k + 1] << 32)) % P64 for k in range(threshold)]
    return S, w[2 * threshold] & 0xFFFFFFFF


def reduce_partial_(partial_tensor, threshold: int, bits: int, dst: int = 0, group=None) -> None:
    """In-place sum-reduce of the leading partial words to `dst` (one collective)."""
    import torch.distributed as dist
    k = reduce_words(threshold, bits)
    dist.reduce(partial_tensor[:k], dst=dst, op=dist.ReduceOp.SUM, group=group)


def _coll_device(group=None):
    """Device for collective buffers: CUDA for nccl (RCCL), CPU for gloo."""
    import torch
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
        else torch.device("cpu")


def broadcast_coeffs(coeffs, stop_value, threshold: int, bits: int, src: int = 0, group=None):
    """Ship rank src's (coefficients, stop value) to every rank: one broadcast
    of t+3 words.  Other ranks pass coeffs=None.  u64 values travel as their
    two's-complement int64 image."""
    import torch
    import torch.distributed as dist
    dev = _coll_device(group)
    buf = torch.zeros(threshold + 3, dtype=torch.int64, device=dev)
    if dist.get_rank(group) == src:
        w = np.zeros(threshold + 3, dtype=np.uint64)
        w[0] = len(coeffs)
        w[1] = 0 if stop_value is None else 1
        w[2] = 0 if stop_value is None else int(stop_value)
        w[3:3 + len(coeffs)] = [int(c) for c in coeffs]
        buf.copy_(torch.from_numpy(w.view(np.int64)))
    dist.broadcast(buf, src=src, group=group)
    w = buf.cpu().numpy().view(np.uint64)
    d = int(w[0])
    mask = (1 << bits) - 1
    coeffs = [int(c) & mask for c in w[3:3 + d]]
    return coeffs, (int(w[2]) & mask if w[1] else None)


def root_test_sharded(local_test, coeffs, log_shard, shard_start: int, stop_value=None, group=None) -> list:
    """Global ascending hit positions of a root test over a log cut into
    contiguous shards (this rank holds log[shard_start : shard_start+len]).

    local_test(coeffs, log_shard, stop_value) -> (positions, stop_index) is
    the shard root test — PowerSumQuackU32/U64.root_test_shard on the GPU."""
    import torch
    import torch.distributed as dist
    dev = _coll_device(group)
    pos, stop = local_test(coeffs, log_shard, stop_value)
    n_local = len(log_shard)
    big = np.iinfo(np.int64).max
    g_stop = torch.tensor([shard_start + stop if stop < n_local else big], dtype=torch.int64, device=dev)
    dist.all_reduce(g_stop, op=dist.ReduceOp.MIN, group=group)
    cut = int(g_stop.item())
    mine = [shard_start + p for p in pos if shard_start + p < cut]
    world = dist.get_world_size(group)
    cnt = torch.tensor([len(mine)], dtype=torch.int64, device=dev)
    cnts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    width = max(int(c.item()) for c in cnts)
    if width == 0:
        return []
    pad = torch.full((width,), -1, dtype=torch.int64, device=dev)
    if mine:
        pad[: len(mine)] = torch.tensor(mine, dtype=torch.int64)
    bufs = [torch.empty(width, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    out = []
    for b, c in zip(bufs, cnts):
        out.extend(int(v) for v in b[: int(c.item())].cpu().tolist())
    return out
