"""Host-side mirror of the reference `quack` crate API over libquack_hip.so.

Same names, argument meaning and error behaviour as the Rust calls the
reference tree makes:

    PowerSumQuackU32::new(threshold)        sidekick/src/sidekick.rs:32
    quack.insert(id)                        sidekick.rs:42, sidekick_multi.rs:82
    quack.remove(id)                        media_client.rs:319
    quack.count() / quack.last_value()      media_client.rs:231-233,259-260
    diff.sub_assign(quack)                  media_client.rs:296
    diff.to_coeffs()                        media_client.rs:304
    arithmetic::eval(&coeffs, id).value()   media_client.rs:310
    clone(), bincode serialize/deserialize  sidekick.rs:187,204; media_client.rs:227

plus the batch entry points of the MI355X engine:

    insert_batch(ids)        encode an id array on the GPU (device tensor:
                             HBM-resident path; numpy array: host path with
                             pipelined H2D).
    decode_with_log(log)     to_coeffs on the host, root test on the GPU.

Per-packet insert/remove stay on the host (one insert is far cheaper than a
kernel launch); every batch call runs the gfx950 kernels and raises if the
device or the library is unavailable -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from ._lib import (P32, P64, QK_E_CAPACITY, QuackError, check, lib)

__all__ = [
    "PowerSumQuackU32", "PowerSumQuackU64", "ModularInteger", "CoefficientVector",
    "arithmetic", "Context", "get_context", "device_count", "FlowQuacks",
]


# --------------------------------------------------------------------------
# Device contexts (one per device, created lazily)
# --------------------------------------------------------------------------
class Context:
    """Owns a qk_ctx* (device scratch, streams, profiling events)."""

    def __init__(self, device: int = 0, handle=None):
        self.owned = handle is None
        if handle is None:
            handle = C.c_void_p()
            check(lib().qk_ctx_create(int(device), C.byref(handle)), f"qk_ctx_create({device})")
        self.handle = handle
        self.device = int(device)

    def close(self):
        if self.handle and self.owned:
            lib().qk_ctx_destroy(self.handle)
            self.handle = None

    def synchronize(self, stream=None):
        check(lib().qk_ctx_synchronize(self.handle, stream), "synchronize")

    def set_profiling(self, on: bool):
        check(lib().qk_ctx_set_profiling(self.handle, int(bool(on))))

    def kernel_stats(self):
        """(total_ms, launches) of the dominant kernel since the last call."""
        ms = C.c_double()
        n = C.c_uint64()
        check(lib().qk_ctx_kernel_stats(self.handle, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def set_grid(self, blocks: int):
        check(lib().qk_ctx_set_grid(self.handle, int(blocks)))

    def set_knob(self, name: str, value: int):
        """A measurement knob of this context (qk_ctx_set_knob)."""
        check(lib().qk_ctx_set_knob(self.handle, name.encode(), int(value)), f"set_knob({name}={value})")

    def trim(self):
        """Free grown-out scratch buffers (synchronises the device)."""
        check(lib().qk_ctx_trim(self.handle), "trim")

    def clock_probe_async(self, microseconds: int, out, stream) -> None:
        """Enqueue the shader-clock probe (qk_clock_probe) on `stream` (a raw
        stream handle): out (a CUDA int64 tensor of 2) receives (s_memtime
        ticks, 100 MHz ticks) over `microseconds` of wall time."""
        check(lib().qk_clock_probe(self.handle, int(microseconds), out.data_ptr(), stream), "clock_probe")


_ctx_lock = threading.Lock()
_contexts: dict = {}


def device_count() -> int:
    n = C.c_int()
    lib().qk_device_count(C.byref(n))
    return n.value


def get_context(device: int = 0) -> Context:
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = _contexts[device] = Context(device)
        return ctx


# --------------------------------------------------------------------------
# Field values and coefficient vectors
# --------------------------------------------------------------------------
class ModularInteger:
    """quack::arithmetic::ModularInteger: canonical value in [0, p)."""
    __slots__ = ("_v", "bits")

    def __init__(self, v: int, bits: int = 32):
        self.bits = bits
        self._v = int(v) % (P32 if bits == 32 else P64)

    def value(self) -> int:
        return self._v

    def __eq__(self, other):
        if isinstance(other, ModularInteger):
            return self._v == other._v and self.bits == other.bits
        return self._v == other

    def __hash__(self):
        return hash((self._v, self.bits))

    def __repr__(self):
        return f"ModularInteger<u{self.bits}>({self._v})"


class CoefficientVector(list):
    """Result of to_coeffs(): c_1..c_d of prod(z - x_missing), canonical ints."""

    def __init__(self, values, bits: int):
        super().__init__(int(v) for v in values)
        self.bits = bits


class _Arithmetic:
    """quack::arithmetic (media_client.rs:21,310)."""

    @staticmethod
    def eval(coeffs: CoefficientVector, x: int) -> ModularInteger:
        bits = getattr(coeffs, "bits", 32)
        d = len(coeffs)
        if bits == 32:
            arr = (C.c_uint32 * max(d, 1))(*coeffs)
            return ModularInteger(lib().qk_u32_eval(arr, d, int(x) & 0xFFFFFFFF), 32)
        arr = (C.c_uint64 * max(d, 1))(*coeffs)
        return ModularInteger(lib().qk_u64_eval(arr, d, int(x) & 0xFFFFFFFFFFFFFFFF), 64)


arithmetic = _Arithmetic()


# --------------------------------------------------------------------------
# Array plumbing (torch device tensors, numpy host arrays)
# --------------------------------------------------------------------------
def roots(coeffs, bits: int = 32) -> list:
    """The distinct roots in GF(p), ascending, of z^d + c_1 z^(d-1) + ... + c_d
    (qk_u32_roots / qk_u64_roots, roots.cpp): a log entry is a root-test hit
    exactly when it is congruent to one of them."""
    d = len(coeffs)
    T = C.c_uint32 if bits == 32 else C.c_uint64
    c = (T * max(d, 1))(*[int(v) for v in coeffs])
    out = (T * max(d, 1))()
    k = C.c_uint32()
    check(getattr(lib(), f"qk_u{bits}_roots")(c, d, out, d, C.byref(k)), "roots")
    return [int(v) for v in out[:k.value]]


def _device_array(a, bits: int):
    """(ptr, n, device_index, stream_ptr) of a contiguous CUDA tensor, or None."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        return None
    if not isinstance(a, torch.Tensor):
        return None
    if not a.is_cuda:
        raise TypeError("CPU torch tensors are not accepted; pass a numpy array for the host path")
    ok = {32: (torch.int32, getattr(torch, "uint32", None)), 64: (torch.int64, getattr(torch, "uint64", None))}[bits]
    if a.dtype not in ok:
        raise TypeError(f"u{bits} ids must be a torch int{bits}/uint{bits} tensor, got {a.dtype}")
    if not a.is_contiguous():
        raise ValueError("ids tensor must be contiguous")
    dev = a.device.index if a.device.index is not None else torch.cuda.current_device()
    stream = torch.cuda.current_stream(dev).cuda_stream
    return a.data_ptr(), a.numel(), dev, stream


def _host_array(a, bits: int) -> np.ndarray:
    dt = np.uint32 if bits == 32 else np.uint64
    arr = np.asarray(a)
    if arr.dtype != dt:
        arr = arr.astype(dt)
    return np.ascontiguousarray(arr)


# --------------------------------------------------------------------------
# The sketch
# --------------------------------------------------------------------------
class _PowerSumQuack:
    BITS = 32
    _ELEM = C.c_uint32
    _P = P32
    _pre = "qk_u32_"

    def __init__(self, threshold: int):
        if threshold < 0 or threshold > 0xFFFFFFFF:
            raise ValueError("threshold must fit u32")
        self._t = int(threshold)
        self._buf = C.create_string_buffer(self._f("size")(self._t))
        check(self._f("init")(self._buf, self._t), "init")

    # -- plumbing -----------------------------------------------------------
    @classmethod
    def _f(cls, name):
        return getattr(lib(), cls._pre + name)

    @classmethod
    def new(cls, threshold: int):
        return cls(threshold)

    def _hdr(self):
        return np.frombuffer(self._buf, dtype=np.uint32, count=4)

    # -- accessors ----------------------------------------------------------
    def threshold(self) -> int:
        return self._t

    def count(self) -> int:
        return int(self._hdr()[1])

    def last_value(self):
        h = self._hdr()
        if not h[2]:
            return None
        if self.BITS == 32:
            return int(h[3])
        return int(np.frombuffer(self._buf, dtype=np.uint64, count=1, offset=16)[0])

    def power_sums(self) -> list:
        if self.BITS == 32:
            return [int(v) for v in np.frombuffer(self._buf, dtype=np.uint32, count=self._t, offset=16)]
        return [int(v) for v in np.frombuffer(self._buf, dtype=np.uint64, count=self._t, offset=24)]

    def clone(self):
        q = type(self).__new__(type(self))
        q._t = self._t
        q._buf = C.create_string_buffer(self._buf.raw, len(self._buf))
        return q

    __copy__ = clone

    def __eq__(self, other):
        return type(self) is type(other) and self._buf.raw == other._buf.raw

    def __repr__(self):
        return (f"{type(self).__name__}(threshold={self._t}, count={self.count()}, "
                f"last_value={self.last_value()})")

    # -- per-packet host path -------------------------------------------------
    def insert(self, ident: int) -> None:
        check(self._f("insert")(self._buf, int(ident)), "insert")

    def remove(self, ident: int) -> None:
        check(self._f("remove")(self._buf, int(ident)), "remove")

    def sub_assign(self, rhs) -> None:
        check(self._f("sub_assign")(self._buf, rhs._buf), "sub_assign")

    def __isub__(self, rhs):
        self.sub_assign(rhs)
        return self

    def merge(self, later) -> None:
        """Union with the disjoint stream that follows this one (additivity)."""
        check(self._f("merge")(self._buf, later._buf), "merge")

    def to_coeffs(self) -> CoefficientVector:
        d = C.c_uint32()
        cap = max(self._t, 1)
        out = (self._ELEM * cap)()
        check(self._f("to_coeffs")(self._buf, out, cap, C.byref(d)), "to_coeffs")
        return CoefficientVector(out[: d.value], self.BITS)

    # -- bincode wire image ----------------------------------------------------
    def serialize(self) -> bytes:
        n = self._f("serialized_size")(self._buf)
        out = (C.c_uint8 * n)()
        ln = C.c_size_t()
        check(self._f("serialize")(self._buf, out, n, C.byref(ln)), "serialize")
        return bytes(out[: ln.value])

    @classmethod
    def deserialize(cls, data: bytes):
        src = (C.c_uint8 * len(data)).from_buffer_copy(data)
        t = C.c_uint32()
        check(cls._f("deserialize")(src, len(data), None, C.byref(t)), "deserialize")
        q = cls(t.value)
        check(cls._f("deserialize")(src, len(data), q._buf, None), "deserialize")
        return q

    # -- batch (GPU) path -------------------------------------------------------
    def insert_batch(self, ids, ctx: Context | None = None) -> None:
        """Insert every id of `ids` in array order, on the GPU.

        A CUDA tensor is encoded where it lies (HBM-resident path); a numpy
        array / sequence goes through the pipelined host->device path."""
        if self._t == 0:
            raise QuackError(-2, "insert_batch into a threshold-0 quACK")
        dev = _device_array(ids, self.BITS)
        if dev is not None:
            ptr, n, d, stream = dev
            ctx = ctx or get_context(d)
            check(self._f("encode_device")(ctx.handle, ptr, n, self._buf, stream), "encode_device")
            return
        arr = _host_array(ids, self.BITS)
        ctx = ctx or get_context(0)
        check(self._f("encode_host")(ctx.handle, arr.ctypes.data, arr.size, self._buf), "encode_host")

    def root_test(self, coeffs, log, stop_value=None, ctx: Context | None = None, cap: int = 1 << 16):
        """Positions (log order) of entries of `log` that are roots of
        `coeffs`; with stop_value, only positions before its first
        occurrence (media_client.rs:306-313)."""
        return self._root_test(coeffs, log, stop_value, ctx, cap, shard=False)[0]

    def root_test_shard(self, coeffs, log, stop_value=None, ctx: Context | None = None, cap: int = 1 << 16):
        """root_test on one shard of a log: (positions, stop_index) where
        stop_index is the first position equal to stop_value in this shard,
        or len(log) (sidekick_amd.dist.root_test_sharded merges shards)."""
        return self._root_test(coeffs, log, stop_value, ctx, cap, shard=True)

    def _root_test(self, coeffs, log, stop_value, ctx, cap, shard):
        coeffs = list(coeffs)
        d = len(coeffs)
        carr = (self._ELEM * max(d, 1))(*coeffs)
        keep = None
        dev = _device_array(log, self.BITS)
        if dev is None:
            import torch  # device memory for a host log: one H2D copy, then the GPU test
            arr = _host_array(log, self.BITS)
            keep = torch.from_numpy(arr.view(np.int32 if self.BITS == 32 else np.int64)).cuda()
            dev = _device_array(keep, self.BITS)
        ptr, n, dv, stream = dev
        ctx = ctx or get_context(dv)
        stop_idx = C.c_uint64(n)
        while True:
            hits = (C.c_uint64 * max(cap, 1))()
            nh = C.c_size_t()
            args = (ctx.handle, carr, d, ptr, n, int(stop_value is not None), int(stop_value or 0), hits, cap,
                    C.byref(nh))
            if shard:
                rc = self._f("root_test_shard_device")(*args, C.byref(stop_idx), stream)
            else:
                rc = self._f("root_test_device")(*args, stream)
            if rc == QK_E_CAPACITY:
                cap = nh.value
                continue
            check(rc, "root_test_device")
            return [int(h) for h in hits[: nh.value]], int(stop_idx.value)

    def decode_host(self, log, stop_at_last: bool = False) -> list:
        """Positions of the missing entries of a HOST log (numpy / sequence),
        tested on the CPU (qk_*_decode_host): to_coeffs, then the root test,
        cut at the first entry equal to last_value() when stop_at_last
        (media_client.rs:304-313).  For the short logs a receiver holds."""
        arr = _host_array(log, self.BITS)
        ptr = arr.ctypes.data_as(C.POINTER(self._ELEM))
        cap = max(self._t, 1)
        while True:
            hits = (C.c_uint64 * cap)()
            nh = C.c_size_t()
            rc = self._f("decode_host")(self._buf, ptr, arr.size, int(stop_at_last), hits, cap, C.byref(nh))
            if rc == QK_E_CAPACITY:
                cap = nh.value
                continue
            check(rc, "decode_host")
            return [int(h) for h in hits[: nh.value]]

    def decode_with_log(self, log, ctx: Context | None = None) -> list:
        """quack's decode_with_log: the ids of `log` that are missing (every
        log entry congruent to a root, in log order)."""
        if self.count() == 0:
            return []
        coeffs = self.to_coeffs()
        pos = self.root_test(coeffs, log, ctx=ctx)
        dev = _device_array(log, self.BITS)
        if dev is not None:
            import torch
            idx = torch.tensor(pos, dtype=torch.int64, device=log.device)
            vals = log[idx].cpu().numpy()
        else:
            vals = _host_array(log, self.BITS)[pos]
        mask = 0xFFFFFFFF if self.BITS == 32 else 0xFFFFFFFFFFFFFFFF
        return [int(v) & mask for v in vals]


class PowerSumQuackU32(_PowerSumQuack):
    """quack::PowerSumQuackU32 — u32 ids over GF(2^32 - 5)."""
    BITS = 32
    _ELEM = C.c_uint32
    _P = P32
    _pre = "qk_u32_"


class PowerSumQuackU64(_PowerSumQuack):
    """quack::PowerSumQuackU64 — u64 ids over GF(2^64 - 59)."""
    BITS = 64
    _ELEM = C.c_uint64
    _P = P64
    _pre = "qk_u64_"


# --------------------------------------------------------------------------
# Low-level async encode (bench / multi-GPU): partial vectors on the device
# --------------------------------------------------------------------------
class PktMeta(C.Structure):
    _fields_ = [("pkttype", C.c_uint8), ("reserved", C.c_uint8), ("protocol_be", C.c_uint16), ("len", C.c_uint32)]


class PktStats(C.Structure):
    _fields_ = [("inserted", C.c_uint64), ("discarded", C.c_uint64), ("resets", C.c_uint64),
                ("filtered", C.c_uint64), ("last_reset_index", C.c_int64)]


def encode_packets(q: "PowerSumQuackU32", bufs, stride: int = 67, meta=None, my_ipv4=None,
                   ctx: Context | None = None) -> dict:
    """Sniff-loop batch (sidekick.rs:76-124) on the GPU: `bufs` is a CUDA
    uint8 tensor of n*stride bytes (records), `meta` an optional CUDA tensor
    of n 8-byte qk_pkt_meta records (int64 view), `my_ipv4` 4 ints or None.
    Updates q in place (reset if a packet to my_ipv4 is seen); returns stats."""
    import torch
    if not (isinstance(bufs, torch.Tensor) and bufs.is_cuda and bufs.dtype == torch.uint8 and bufs.is_contiguous()):
        raise TypeError("bufs must be a contiguous CUDA uint8 tensor")
    n = bufs.numel() // stride
    dev = bufs.device.index if bufs.device.index is not None else torch.cuda.current_device()
    ctx = ctx or get_context(dev)
    mptr = None
    if meta is not None:
        if not (meta.is_cuda and meta.is_contiguous() and meta.numel() * meta.element_size() == 8 * n):
            raise ValueError("meta must be a contiguous CUDA tensor of n 8-byte records")
        mptr = meta.data_ptr()
    ip = (C.c_uint8 * 4)(*my_ipv4) if my_ipv4 is not None else None
    st = PktStats()
    check(lib().qk_u32_encode_packets_device(ctx.handle, bufs.data_ptr(), n, stride, mptr, ip, q._buf,
                                              C.byref(st), torch.cuda.current_stream(dev).cuda_stream),
          "encode_packets")
    return {k: getattr(st, k) for k, _ in PktStats._fields_}


class FlowKey(C.Structure):
    _fields_ = [("addr", C.c_uint8 * 12)]


def encode_segments(ids, offsets, threshold: int, ctx: Context | None = None) -> list:
    """Segmented encode: `ids` a CUDA u32 tensor grouped by flow, `offsets`
    nseg+1 ints (CSR).  Returns one PowerSumQuackU32 per segment."""
    ptr, n, dev, stream = _device_array(ids, 32)
    ctx = ctx or get_context(dev)
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
    nseg = len(offs) - 1
    rec = lib().qk_u32_size(threshold)
    out = C.create_string_buffer(max(nseg, 1) * rec)
    check(lib().qk_u32_encode_segments_device(ctx.handle, ptr, offs.ctypes.data_as(C.POINTER(C.c_uint64)), nseg,
                                               threshold, out, stream), "encode_segments")
    res = []
    raw = out.raw                     # one copy (ctypes .raw copies the whole buffer per access)
    for i in range(nseg):
        q = PowerSumQuackU32.__new__(PowerSumQuackU32)
        q._t = threshold
        q._buf = C.create_string_buffer(raw[i * rec:(i + 1) * rec], rec)
        res.append(q)
    return res


def encode_flows(bufs, threshold: int, stride: int = 67, meta=None, my_addr=None, ctx: Context | None = None,
                 device_out: bool = False):
    """One SidekickMulti batch (sidekick_multi.rs:65-90,101-143) without the
    table merge: returns (keys, sketches, stats) for the batch's flows in
    ascending AddrKey order.  device_out=False: keys is a list of 12-byte
    AddrKeys and sketches a list of PowerSumQuackU32.  device_out=True: both
    stay in HBM as CUDA tensors (uint8 [nf, 12] and int32 [nf, 4 + t], the
    qk_u32 records), written in place by the finalize kernel."""
    import torch
    if not (isinstance(bufs, torch.Tensor) and bufs.is_cuda and bufs.dtype == torch.uint8 and bufs.is_contiguous()):
        raise TypeError("bufs must be a contiguous CUDA uint8 tensor")
    n = bufs.numel() // stride
    dev = bufs.device.index if bufs.device.index is not None else torch.cuda.current_device()
    ctx = ctx or get_context(dev)
    mptr = None
    if meta is not None:
        if not (meta.is_cuda and meta.is_contiguous() and meta.numel() * meta.element_size() == 8 * n):
            raise ValueError("meta must be a contiguous CUDA tensor of n 8-byte records")
        mptr = meta.data_ptr()
    addr = (C.c_uint8 * 6)(*my_addr) if my_addr is not None else None
    rec = lib().qk_u32_size(threshold)
    stream = torch.cuda.current_stream(dev).cuda_stream
    cap = 1024
    while True:
        nf, st = C.c_size_t(), PktStats()
        if device_out:
            keys = torch.empty((cap, 12), dtype=torch.uint8, device=bufs.device)
            sk = torch.empty((cap, rec // 4), dtype=torch.int32, device=bufs.device)
            kp, sp = keys.data_ptr(), sk.data_ptr()
        else:
            keys = (FlowKey * cap)()
            sk = C.create_string_buffer(cap * rec)
            kp, sp = keys, sk
        rc = lib().qk_u32_encode_flows_device(ctx.handle, bufs.data_ptr(), n, stride, mptr, addr, threshold, kp, sp,
                                              cap, C.byref(nf), C.byref(st), stream)
        if rc == QK_E_CAPACITY:
            cap = nf.value
            continue
        check(rc, "encode_flows")
        break
    stats = {k: getattr(st, k) for k, _ in PktStats._fields_}
    m = nf.value
    if device_out:
        return keys[:m], sk[:m], stats
    out_k, out_q = [], []
    raw = sk.raw                      # one copy of the records (ctypes .raw copies the whole buffer per access)
    for i in range(m):
        out_k.append(bytes(keys[i].addr))
        q = PowerSumQuackU32.__new__(PowerSumQuackU32)
        q._t = threshold
        q._buf = C.create_string_buffer(raw[i * rec:(i + 1) * rec], rec)
        out_q.append(q)
    return out_k, out_q, stats


class FlowQuacks:
    """SidekickMulti's flow table, HashMap<AddrKey, PowerSumQuackU32>
    (sidekick_multi.rs:22-37,57-90), with a GPU batch entry point.
    Keys are the 12-byte AddrKey (bytes)."""

    def __init__(self, threshold: int):
        self.threshold = int(threshold)
        self._senders: dict = {}

    # per-packet host path (sidekick_multi.rs:65-90)
    def insert(self, addr_key: bytes, sidekick_id: int) -> "PowerSumQuackU32":
        q = self._senders.get(bytes(addr_key))
        if q is None:
            q = self._senders[bytes(addr_key)] = PowerSumQuackU32(self.threshold)
        q.insert(sidekick_id)
        return q

    # SidekickMulti::reset (sidekick_multi.rs:59-63): only an existing entry is
    # reset.  The sniff loops never call it — a Reset packet replaces the whole
    # map (:205, :265), which insert_packets does.
    def reset(self, addr_key: bytes) -> None:
        if bytes(addr_key) in self._senders:
            self._senders[bytes(addr_key)] = PowerSumQuackU32(self.threshold)

    def quack(self, addr_key: bytes):
        q = self._senders.get(bytes(addr_key))
        return q.clone() if q is not None else None

    def senders(self) -> dict:
        return self._senders

    def insert_packets(self, bufs, stride: int = 67, meta=None, my_addr=None, ctx: Context | None = None) -> dict:
        """Batch of captured records (CUDA uint8 tensor) through the GPU:
        extract, group by AddrKey, encode per flow, merge into the table."""
        keys, quacks, stats = encode_flows(bufs, self.threshold, stride, meta, my_addr, ctx)
        if stats["resets"]:
            # a Reset wipes every flow (`senders = HashMap::new()`,
            # sidekick_multi.rs:205,265); the batch output is what follows it
            self._senders = {}
        for key, q in zip(keys, quacks):
            old = self._senders.get(key)
            if old is None:
                self._senders[key] = q
            else:
                old.merge(q)
        return stats


def partial_words(threshold: int, bits: int = 32) -> int:
    return int(getattr(lib(), f"qk_u{bits}_partial_words")(threshold))


def encode_device_async(ctx: Context, ids, threshold: int, partial, bits: int = 32, stream=None) -> None:
    """Enqueue encode of a CUDA id tensor into a CUDA int64 `partial` tensor
    of partial_words(threshold, bits) words (layout: include/quack_hip.h)."""
    ptr, n, _, s = _device_array(ids, bits)
    if stream is None:
        stream = s
    check(getattr(lib(), f"qk_u{bits}_encode_device_async")(ctx.handle, ptr, n, threshold,
                                                              partial.data_ptr(), stream), "encode_device_async")


def merge_partial(q: _PowerSumQuack, partial_host, has_last: bool, last: int) -> None:
    arr = np.ascontiguousarray(np.asarray(partial_host).astype(np.uint64))
    check(q._f("merge_partial")(q._buf, arr.ctypes.data_as(C.POINTER(C.c_uint64)), int(has_last), int(last)),
          "merge_partial")


def fill_splitmix(ctx: Context, out, seed: int, start: int = 0, bits: int = 32, stream=None) -> None:
    """Fill a CUDA tensor with the synthetic splitmix64 id stream (device-side)."""
    ptr, n, _, s = _device_array(out, bits)
    check(getattr(lib(), f"qk_fill_splitmix_u{bits}")(ctx.handle, ptr, n, seed & 0xFFFFFFFFFFFFFFFF, start,
                                                        s if stream is None else stream), "fill_splitmix")
