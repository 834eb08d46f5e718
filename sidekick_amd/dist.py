"""Multi-GPU sharding of the encode path (one process per GPU).

The sketch is additive: S_k(A ⊎ B) = S_k(A) + S_k(B) mod p
and counts add, so the id stream is cut into contiguous shards, one per rank,
each rank encodes its shard into a partial vector on its own GPU, and ONE
sum-reduce of the partial words (RCCL over xGMI with backend "nccl"; gloo in
the CPU tests) merges them on rank 0.  Partial words are canonical residues
(< 2^32, limbs for the u64 field) stored as uint64, so the integer sum of up
to 2^27 ranks cannot overflow; rank 0 folds the sum mod p.  last_value comes
from the last non-empty shard, which rank 0 learns without communication
(shards are contiguous and their sizes are known to every rank).
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
