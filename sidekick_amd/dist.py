"""Multi-GPU sharding of the encode and decode paths.

The product path is the native communicator of libquack_hip.so (`Comm`,
over qk_comm_* in include/quack_hip.h: RCCL over xGMI, one ncclReduce per
sharded encode; comm.hip).  It runs with one process driving several GPUs
(`Comm.create(devices)`, the shape of the reference's single-process callers)
or one process per GPU (`Comm.from_process_group()` ships the RCCL unique id
over an existing torch.distributed group — gloo is enough — and every rank
joins).  `Comm.init_host(channel, ...)` builds the same communicator with its
collectives over a host channel instead of RCCL — the identical native
protocol (payload packing, failed-rank word, root fold, status gathers):
`ProcessGroupChannel` carries them over a torch.distributed group (several
ranks rehearsed on one GPU, which RCCL refuses) and `LoopbackHub` over
threads of one process (world 2-8 on one GPU in the test suite).

The sketch is additive: S_k(A ⊎ B) = S_k(A) + S_k(B) mod p
and counts add, so the id stream is cut into contiguous shards, one per rank,
each rank encodes its shard into a partial vector on its own GPU, and ONE
sum-reduce of the payload merges them on the root.  Payload words are
canonical residues (< 2^32, limbs for the u64 field) stored as uint64, so the
integer sum of up to 2^27 ranks cannot overflow; the root folds the sum mod p
and reads last_value from the per-rank (has_last, last) slots.

Decode (comm.hip decode_sharded): the root turns the merged difference into
coefficients (O(t^2), host) and broadcasts [status, d, stop flag, stop value,
c_1..c_d]; each rank root-tests its contiguous log shard on its own GPU and
finds where the stop value first occurs in it; one all-gather of (n, stop,
hit count, status) per rank gives every rank the global stop (the caller's
`break` at media_client.rs:307-309 applies to the whole log) and the lowest
failing rank's status; then the hit positions — offset by the shard base, cut
at the global stop — are all-gathered in fixed-size rounds.  Every rank
returns the same ascending list, identical to the single-GPU root test.

The torch.distributed helpers at the end (`pack_payload`, `fold_payload`,
`root_test_sharded`, ...) restate that protocol in numpy over any
torch.distributed backend: the CPU-only rehearsal (gloo, world 2-3,
tests/test_dist.py) for a container without a GPU.  (`root_test_sharded`
exchanges the stop with an all-reduce(MIN) instead of the native status
gather; the merge it computes is the same.)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import sys
import threading

from ._lib import P32, P64, QK_E_CAPACITY, check, lib


# --------------------------------------------------------------------------
# Native communicator (qk_comm_*): the product multi-GPU path
# --------------------------------------------------------------------------
COMM_ID_BYTES = 128

_REDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.c_int)
_BCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.c_int)
_GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_size_t)


class _HostOps(C.Structure):
    """qk_comm_host_ops (include/quack_hip.h)."""
    _fields_ = [("user", C.c_void_p), ("reduce_sum_u64", _REDUCE_FN), ("broadcast_u64", _BCAST_FN),
                ("allgather_u64", _GATHER_FN)]


def _u64(ptr, n) -> np.ndarray:
    return np.ctypeslib.as_array(ptr, (n,)) if n else np.zeros(0, dtype=np.uint64)


class HostChannel:
    """Collectives over uint64 numpy arrays (in place) for Comm.init_host:
    reduce_sum(buf, root), broadcast(buf, root), allgather(send, recv) with
    recv[r*n:(r+1)*n] = rank r's send.  Raise on failure."""

    def reduce_sum(self, buf: np.ndarray, root: int) -> None:
        raise NotImplementedError

    def broadcast(self, buf: np.ndarray, root: int) -> None:
        raise NotImplementedError

    def allgather(self, send: np.ndarray, recv: np.ndarray) -> None:
        raise NotImplementedError

    def _ops(self):
        """ctypes qk_comm_host_ops calling this channel (keep the result alive)."""
        def guard(fn):
            def call(*a):
                try:
                    fn(*a)
                    return 0
                except BaseException as e:   # noqa: BLE001 — nothing may unwind through C
                    print(f"host channel collective failed: {e!r}", file=sys.stderr, flush=True)
                    return -1
            return call
        red = _REDUCE_FN(guard(lambda _u, b, n, root: self.reduce_sum(_u64(b, n), root)))
        bc = _BCAST_FN(guard(lambda _u, b, n, root: self.broadcast(_u64(b, n), root)))
        ga = _GATHER_FN(guard(lambda _u, s, r, n: self.allgather(_u64(s, n), _u64(r, n * self.world))))
        return _HostOps(None, red, bc, ga)


class ProcessGroupChannel(HostChannel):
    """The host collectives over a torch.distributed group (CPU tensors: gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    @staticmethod
    def _t(a):
        import torch
        return torch.from_numpy(a.view(np.int64))

    def reduce_sum(self, buf, root):
        import torch.distributed as dist
        dist.reduce(self._t(buf), dst=root, op=dist.ReduceOp.SUM, group=self.group)

    def broadcast(self, buf, root):
        import torch.distributed as dist
        dist.broadcast(self._t(buf), src=root, group=self.group)

    def allgather(self, send, recv):
        import torch.distributed as dist
        n = len(send)
        outs = list(self._t(recv).split(n)) if n else [self._t(recv)[:0] for _ in range(self.world)]
        dist.all_gather(outs, self._t(send.copy()), group=self.group)


class LoopbackHub:
    """Host collectives between `world` ranks living in threads of one process
    (each thread drives its own Comm.init_host rank).  A rank that never
    arrives breaks the barrier after `timeout` s: the others fail instead of
    waiting forever."""

    def __init__(self, world: int, timeout: float = 120.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots = [None] * world

    def channel(self, rank: int) -> "HostChannel":
        return _LoopbackChannel(self, rank)


class _LoopbackChannel(HostChannel):
    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub, self.rank, self.world = hub, rank, hub.world

    def reduce_sum(self, buf, root):
        h = self.hub
        h.slots[self.rank] = buf.copy()
        h.barrier.wait()
        if self.rank == root:
            buf[:] = np.sum(np.stack(h.slots), axis=0, dtype=np.uint64)
        h.barrier.wait()

    def broadcast(self, buf, root):
        h = self.hub
        if self.rank == root:
            h.slots[root] = buf.copy()
        h.barrier.wait()
        if self.rank != root:
            buf[:] = h.slots[root]
        h.barrier.wait()

    def allgather(self, send, recv):
        h = self.hub
        h.slots[self.rank] = send.copy()
        h.barrier.wait()
        recv[:] = np.concatenate(h.slots)
        h.barrier.wait()


class Comm:
    """A qk_comm: local ranks (GPUs driven by this process) of a communicator.

    Array arguments take one entry per local rank, in local rank order."""

    def __init__(self, handle):
        self.handle = handle
        w, nl, fr = C.c_int(), C.c_int(), C.c_int()
        check(lib().qk_comm_info(handle, C.byref(w), C.byref(nl), C.byref(fr)), "qk_comm_info")
        self.world, self.nlocal, self.first_rank = w.value, nl.value, fr.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        check(lib().qk_comm_unique_id(buf), "qk_comm_unique_id")
        return bytes(buf)

    @classmethod
    def create(cls, devices) -> "Comm":
        """One process, several GPUs (ncclCommInitAll): local rank i = devices[i]."""
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(lib().qk_comm_create(len(devices), devs, C.byref(h)), "qk_comm_create")
        return cls(h)

    @classmethod
    def init_rank(cls, uid: bytes, rank: int, world: int, device: int) -> "Comm":
        """One process per GPU: every rank calls this with rank 0's unique id."""
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().qk_comm_init_rank(buf, rank, world, device, C.byref(h)), "qk_comm_init_rank")
        return cls(h)

    @classmethod
    def init_host(cls, channel: HostChannel, rank: int, world: int, device: int) -> "Comm":
        """One rank whose collectives run over `channel` (qk_comm_init_host):
        the native protocol with a host channel instead of RCCL."""
        ops = channel._ops()
        h = C.c_void_p()
        check(lib().qk_comm_init_host(C.byref(ops), rank, world, device, C.byref(h)), "qk_comm_init_host")
        c = cls(h)
        c._keep = (channel, ops)     # the callbacks must outlive the communicator
        return c

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "Comm":
        """Join a communicator spanning the ranks of a torch.distributed group
        (any backend: it only carries the 128-byte unique id)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls.init_rank(obj[0], rank, world, device)

    def close(self):
        if self.handle:
            lib().qk_comm_destroy(self.handle)
            self.handle = None

    def barrier(self):
        check(lib().qk_comm_barrier(self.handle), "qk_comm_barrier")

    def set_timeout(self, ms: int) -> None:
        """Bound every wait on an RCCL collective (0: never); past it the
        communicator aborts and the call raises QK_E_COMM."""
        check(lib().qk_comm_set_timeout(self.handle, int(ms)), "qk_comm_set_timeout")

    def rccl_info(self, local: int = 0):
        """(ranks, device, rank) as RCCL itself reports them (ncclCommCount,
        ncclCommCuDevice, ncclCommUserRank); None for a host-channel
        communicator."""
        if getattr(self, "_keep", None) is not None:
            return None
        k, d, r = C.c_int(), C.c_int(), C.c_int()
        check(lib().qk_comm_rccl_info(self.handle, local, C.byref(k), C.byref(d), C.byref(r)), "qk_comm_rccl_info")
        return k.value, d.value, r.value

    def context(self, local: int = 0):
        """The (communicator-owned) qk_ctx of a local rank."""
        from .quack import Context
        h = C.c_void_p()
        check(lib().qk_comm_context(self.handle, local, C.byref(h)), "qk_comm_context")
        ctx = Context(device=-1, handle=h)
        ctx._owner = self            # valid until this communicator is closed
        return ctx

    @staticmethod
    def _arrays(tensors, bits):
        from .quack import _device_array
        n = len(tensors)
        ptrs, lens, streams = (C.c_void_p * n)(), (C.c_size_t * n)(), (C.c_void_p * n)()
        for i, t in enumerate(tensors):
            ptr, cnt, _, st = _device_array(t, bits)
            ptrs[i], lens[i], streams[i] = ptr, cnt, st
        return ptrs, lens, streams

    def encode_sharded_async(self, shards, threshold: int, bits: int = 32, root: int = 0) -> None:
        """Enqueue: encode local shard i on its GPU, then one RCCL reduce to root."""
        assert len(shards) == self.nlocal
        ptrs, lens, streams = self._arrays(shards, bits)
        check(getattr(lib(), f"qk_u{bits}_encode_sharded_async")(self.handle, ptrs, lens, threshold, root, streams),
              "encode_sharded_async")

    def encode_sharded_wait(self, q) -> None:
        """Drain; on the root merge the whole stream into q (others: q untouched)."""
        check(getattr(lib(), f"qk_u{q.BITS}_encode_sharded_wait")(self.handle, q._buf if q is not None else None),
              "encode_sharded_wait")

    def encode_sharded(self, shards, q, root: int = 0) -> None:
        assert len(shards) == self.nlocal
        ptrs, lens, streams = self._arrays(shards, q.BITS)
        check(getattr(lib(), f"qk_u{q.BITS}_encode_sharded")(self.handle, ptrs, lens, q._buf, root, streams),
              "encode_sharded")

    def decode_sharded(self, diff, logs, bits: int = 32, stop_at_last: bool = True, root: int = 0,
                       cap: int = 1 << 16) -> list:
        """Global ascending hit positions of the root test over the whole log
        (log shard i on local rank i); diff is read on the root only."""
        assert len(logs) == self.nlocal
        ptrs, lens, streams = self._arrays(logs, bits)
        f = getattr(lib(), f"qk_u{bits}_decode_sharded")
        while True:
            hits = (C.c_uint64 * max(cap, 1))()
            nh = C.c_size_t()
            rc = f(self.handle, diff._buf if diff is not None else None, root, ptrs, lens, int(stop_at_last), hits,
                   cap, C.byref(nh), streams)
            if rc == QK_E_CAPACITY:
                cap = nh.value
                continue
            check(rc, "decode_sharded")
            return [int(h) for h in hits[: nh.value]]


# --------------------------------------------------------------------------
# The same protocol over torch.distributed (CPU rehearsal with gloo)
# --------------------------------------------------------------------------


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


def pack_payload(partial, threshold: int, bits: int, rank: int, world: int) -> np.ndarray:
    """The sharded-encode payload of one rank, as comm.hip's k_comm_pack builds
    it: the summed words [S.., n] then one (has_last, last) slot per rank,
    only this rank's filled.  Summing the payloads of all ranks (the one
    reduce) leaves every slot with exactly one contributor."""
    R = reduce_words(threshold, bits)
    part = np.asarray(partial).astype(np.uint64)
    out = np.zeros(R + 2 * world, dtype=np.uint64)
    out[:R] = part[:R]
    if part[R - 1]:
        out[R + 2 * rank] = 1
        out[R + 2 * rank + 1] = part[R]
    return out


def fold_payload(words, threshold: int, bits: int, world: int):
    """(canonical power sums, wrapping count, last_value or None) of a summed
    payload — the root's fold in comm.hip encode_sharded_wait: last_value is
    the last id of the highest non-empty rank."""
    w = np.asarray(words).astype(np.uint64)
    R = reduce_words(threshold, bits)
    S, count = fold_partial_sum(w[:R], threshold, bits)
    last = None
    for r in range(world - 1, -1, -1):
        if int(w[R + 2 * r]):
            last = int(w[R + 2 * r + 1])
            break
    return S, count, last


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
