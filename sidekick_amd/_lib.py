"""ctypes binding of libquack_hip.so (include/quack_hip.h).

The shared library is built in-tree (``sidekick_amd/libquack_hip.so``) by
``__graft_entry__.build()`` / ``make -C sidekick_amd/csrc``.  There is no
fallback: if the library is missing, importing the device API raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# QK_LIB_PATH selects another build of the same library: the host-sanitized
# libquack_hip_asan.so in tests/test_sanitizers.py
LIB_PATH = os.environ.get("QK_LIB_PATH") or os.path.join(HERE, "libquack_hip.so")

QK_OK = 0
QK_E_INVAL = -1
QK_E_THRESHOLD = -2
QK_E_MISMATCH = -3
QK_E_UNDECODABLE = -4
QK_E_CAPACITY = -5
QK_E_HIP = -6
QK_E_NO_DEVICE = -7
QK_E_NOMEM = -8
QK_E_FORMAT = -9
QK_E_COMM = -10
QK_E_PEER = -11

P32 = 4294967291
P64 = 18446744073709551557
MAX_THRESHOLD = 1024

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p
vpp = C.POINTER(C.c_void_p)
sz = C.c_size_t
szp = C.POINTER(C.c_size_t)

# name -> (restype, argtypes).  Every symbol declared in include/quack_hip.h.
SIGNATURES = {
    "qk_strerror": (C.c_char_p, [C.c_int]),
    "qk_version": (C.c_char_p, []),
    "qk_u32_size": (sz, [C.c_uint32]),
    "qk_u64_size": (sz, [C.c_uint32]),
    "qk_u32_init": (C.c_int, [vp, C.c_uint32]),
    "qk_u64_init": (C.c_int, [vp, C.c_uint32]),
    "qk_u32_insert": (C.c_int, [vp, C.c_uint32]),
    "qk_u64_insert": (C.c_int, [vp, C.c_uint64]),
    "qk_u32_remove": (C.c_int, [vp, C.c_uint32]),
    "qk_u64_remove": (C.c_int, [vp, C.c_uint64]),
    "qk_u32_sub_assign": (C.c_int, [vp, vp]),
    "qk_u64_sub_assign": (C.c_int, [vp, vp]),
    "qk_u32_merge": (C.c_int, [vp, vp]),
    "qk_u64_merge": (C.c_int, [vp, vp]),
    "qk_u32_to_coeffs": (C.c_int, [vp, u32p, C.c_uint32, u32p]),
    "qk_u64_to_coeffs": (C.c_int, [vp, u64p, C.c_uint32, u32p]),
    "qk_u32_eval": (C.c_uint32, [u32p, C.c_uint32, C.c_uint32]),
    "qk_u64_eval": (C.c_uint64, [u64p, C.c_uint32, C.c_uint64]),
    "qk_u32_decode_host": (C.c_int, [vp, u32p, sz, C.c_int, u64p, sz, szp]),
    "qk_u64_decode_host": (C.c_int, [vp, u64p, sz, C.c_int, u64p, sz, szp]),
    "qk_u32_serialized_size": (sz, [vp]),
    "qk_u32_serialize": (C.c_int, [vp, u8p, sz, szp]),
    "qk_u32_deserialize": (C.c_int, [u8p, sz, vp, u32p]),
    "qk_u64_serialized_size": (sz, [vp]),
    "qk_u64_serialize": (C.c_int, [vp, u8p, sz, szp]),
    "qk_u64_deserialize": (C.c_int, [u8p, sz, vp, u32p]),
    "qk_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "qk_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "qk_ctx_destroy": (None, [vp]),
    "qk_ctx_synchronize": (C.c_int, [vp, vp]),
    "qk_ctx_set_profiling": (C.c_int, [vp, C.c_int]),
    "qk_ctx_kernel_stats": (C.c_int, [vp, C.POINTER(C.c_double), u64p]),
    "qk_ctx_set_grid": (C.c_int, [vp, C.c_uint32]),
    "qk_ctx_set_knob": (C.c_int, [vp, C.c_char_p, C.c_int64]),
    "qk_clock_probe": (C.c_int, [vp, C.c_uint32, vp, vp]),
    "qk_ctx_trim": (C.c_int, [vp]),
    "qk_host_alloc": (C.c_int, [sz, C.POINTER(vp)]),
    "qk_host_free": (C.c_int, [vp]),
    "qk_u32_partial_words": (sz, [C.c_uint32]),
    "qk_u64_partial_words": (sz, [C.c_uint32]),
    "qk_u32_encode_device_async": (C.c_int, [vp, vp, sz, C.c_uint32, vp, vp]),
    "qk_u64_encode_device_async": (C.c_int, [vp, vp, sz, C.c_uint32, vp, vp]),
    "qk_u32_merge_partial": (C.c_int, [vp, u64p, C.c_int, C.c_uint32]),
    "qk_u64_merge_partial": (C.c_int, [vp, u64p, C.c_int, C.c_uint64]),
    "qk_u32_encode_device": (C.c_int, [vp, vp, sz, vp, vp]),
    "qk_u64_encode_device": (C.c_int, [vp, vp, sz, vp, vp]),
    "qk_u32_encode_host": (C.c_int, [vp, vp, sz, vp]),
    "qk_u64_encode_host": (C.c_int, [vp, vp, sz, vp]),
    "qk_u32_root_test_device": (C.c_int, [vp, u32p, C.c_uint32, vp, sz, C.c_int, C.c_uint32, u64p, sz, szp, vp]),
    "qk_u64_root_test_device": (C.c_int, [vp, u64p, C.c_uint32, vp, sz, C.c_int, C.c_uint64, u64p, sz, szp, vp]),
    "qk_u32_root_test_shard_device": (C.c_int, [vp, u32p, C.c_uint32, vp, sz, C.c_int, C.c_uint32, u64p, sz, szp,
                                                u64p, vp]),
    "qk_u64_root_test_shard_device": (C.c_int, [vp, u64p, C.c_uint32, vp, sz, C.c_int, C.c_uint64, u64p, sz, szp,
                                                u64p, vp]),
    "qk_u32_roots": (C.c_int, [u32p, C.c_uint32, u32p, C.c_uint32, u32p]),
    "qk_u64_roots": (C.c_int, [u64p, C.c_uint32, u64p, C.c_uint32, u32p]),
    "qk_u32_decode_device": (C.c_int, [vp, vp, vp, sz, C.c_int, u64p, sz, szp, vp]),
    "qk_u64_decode_device": (C.c_int, [vp, vp, vp, sz, C.c_int, u64p, sz, szp, vp]),
    "qk_u32_encode_packets_device": (C.c_int, [vp, vp, sz, sz, vp, vp, vp, vp, vp]),
    "qk_u32_encode_flows_device": (C.c_int, [vp, vp, sz, sz, vp, vp, C.c_uint32, vp, vp, sz, szp, vp, vp]),
    "qk_u32_encode_segments_device": (C.c_int, [vp, vp, u64p, sz, C.c_uint32, vp, vp]),
    "qk_comm_unique_id": (C.c_int, [u8p]),
    "qk_comm_create": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(vp)]),
    "qk_comm_init_rank": (C.c_int, [u8p, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
    "qk_comm_init_host": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
    "qk_comm_destroy": (None, [vp]),
    "qk_comm_info": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "qk_comm_context": (C.c_int, [vp, C.c_int, C.POINTER(vp)]),
    "qk_comm_barrier": (C.c_int, [vp]),
    "qk_comm_set_timeout": (C.c_int, [vp, C.c_int64]),
    "qk_comm_rccl_info": (C.c_int, [vp, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "qk_u32_encode_sharded_async": (C.c_int, [vp, vpp, szp, C.c_uint32, C.c_int, vpp]),
    "qk_u64_encode_sharded_async": (C.c_int, [vp, vpp, szp, C.c_uint32, C.c_int, vpp]),
    "qk_u32_encode_sharded_wait": (C.c_int, [vp, vp]),
    "qk_u64_encode_sharded_wait": (C.c_int, [vp, vp]),
    "qk_u32_encode_sharded": (C.c_int, [vp, vpp, szp, vp, C.c_int, vpp]),
    "qk_u64_encode_sharded": (C.c_int, [vp, vpp, szp, vp, C.c_int, vpp]),
    "qk_u32_decode_sharded": (C.c_int, [vp, vp, C.c_int, vpp, szp, C.c_int, u64p, sz, szp, vpp]),
    "qk_u64_decode_sharded": (C.c_int, [vp, vp, C.c_int, vpp, szp, C.c_int, u64p, sz, szp, vpp]),
    "qk_fill_splitmix_u32": (C.c_int, [vp, vp, sz, C.c_uint64, C.c_uint64, vp]),
    "qk_fill_splitmix_u64": (C.c_int, [vp, vp, sz, C.c_uint64, C.c_uint64, vp]),
}


class QuackError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().qk_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class UndecodableError(QuackError):
    """count > threshold: the caller must reset (media_client.rs:258-278)."""


_lib = None


def lib():
    """Load libquack_hip.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        # torch first when it is installed: it brings its own HIP runtime
        # (libamdhip64.so.7), and the library must bind to that same copy —
        # loaded the other way round, torch finds the /opt/rocm runtime
        # already mapped under its soname and reports no GPU
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C sidekick_amd/csrc` (there is no CPU fallback for the device path)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != QK_OK:
        if rc == QK_E_UNDECODABLE:
            raise UndecodableError(rc, what)
        raise QuackError(rc, what)
