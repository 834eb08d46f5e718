"""ctypes loader for oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this.  See quack_oracle.c for what it restates (parity unpinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(HERE, "quack_oracle.c")
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            build()
        L = C.CDLL(LIB_PATH)
        u32p, u64p, i64p = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_int64)
        sig = {
            "qo_splitmix_u32": (None, [C.c_uint64, C.c_uint64, C.c_uint64, u32p]),
            "qo_splitmix_u64": (None, [C.c_uint64, C.c_uint64, C.c_uint64, u64p]),
            "qo_encode_u32": (None, [u32p, C.c_uint64, C.c_uint32, u32p]),
            "qo_encode_u32_seed": (None, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, u32p]),
            "qo_encode_u64": (None, [u64p, C.c_uint64, C.c_uint32, u64p]),
            "qo_encode_u64_seed": (None, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, u64p]),
            "qo_encode_seed_mt": (C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                            C.c_void_p]),
            "qo_encode_mt": (C.c_int, [C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]),
            "qo_to_coeffs_u32": (None, [u32p, C.c_uint32, u32p]),
            "qo_to_coeffs_u64": (None, [u64p, C.c_uint32, u64p]),
            "qo_eval_u32": (C.c_uint32, [u32p, C.c_uint32, C.c_uint32]),
            "qo_eval_u64": (C.c_uint64, [u64p, C.c_uint32, C.c_uint64]),
            "qo_root_test_u32": (C.c_uint64, [u32p, C.c_uint32, u32p, C.c_uint64, i64p, C.c_uint64]),
            "qo_root_test_u64": (C.c_uint64, [u64p, C.c_uint32, u64p, C.c_uint64, i64p, C.c_uint64]),
            "qo_bench_construct": (C.c_uint64, [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, u64p]),
            "qo_bench_decode": (C.c_uint64, [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, u64p]),
            "qo_encode_timed": (None, [C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, u64p, u64p]),
            "qo_encode_cycles": (None, [C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, u64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def splitmix_u32(seed, n, start=0):
    out = np.empty(n, dtype=np.uint32)
    lib().qo_splitmix_u32(seed, start, n, _p(out, C.c_uint32))
    return out


def splitmix_u64(seed, n, start=0):
    out = np.empty(n, dtype=np.uint64)
    lib().qo_splitmix_u64(seed, start, n, _p(out, C.c_uint64))
    return out


def encode_u32(ids, t):
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    S = np.zeros(t, dtype=np.uint32)
    lib().qo_encode_u32(_p(ids, C.c_uint32), len(ids), t, _p(S, C.c_uint32))
    return [int(v) for v in S]


def encode_u32_seed(seed, n, t, start=0):
    S = np.zeros(t, dtype=np.uint32)
    lib().qo_encode_u32_seed(seed, start, n, t, _p(S, C.c_uint32))
    return [int(v) for v in S]


def encode_seed_mt(bits, seed, n, t, threads, start=0):
    """All-cores restatement (one partial per thread, merged): bench.py's
    cpu_baseline_all_cores leg."""
    S = np.zeros(t, dtype=np.uint32 if bits == 32 else np.uint64)
    rc = lib().qo_encode_seed_mt(bits, seed, start, n, t, threads, S.ctypes.data)
    if rc:
        raise RuntimeError(f"qo_encode_seed_mt rc={rc}")
    return [int(v) for v in S]


def encode_timed(ids, t):
    """The scalar insert loop over pre-generated ids timed as the crate's
    benchmark_construct does (rdtsc) and by CLOCK_MONOTONIC over the same
    region: (power sums, TSC ticks, nanoseconds)."""
    bits = 32 if ids.dtype == np.uint32 else 64
    ids = np.ascontiguousarray(ids)
    S = np.zeros(t, dtype=np.uint32 if bits == 32 else np.uint64)
    tsc, ns = C.c_uint64(), C.c_uint64()
    lib().qo_encode_timed(bits, ids.ctypes.data, len(ids), t, S.ctypes.data, C.byref(tsc), C.byref(ns))
    return [int(v) for v in S], tsc.value, ns.value


def encode_cycles(ids, t):
    """encode_timed with the core's view of the same region (quack_oracle.c
    qo_encode_cycles): (power sums, dict of core cycles and instructions
    from perf_event_open (None where refused, with its errno), TSC ticks, ns,
    and the core clock read by a dependent-add chain around the loop)."""
    bits = 32 if ids.dtype == np.uint32 else 64
    ids = np.ascontiguousarray(ids)
    S = np.zeros(t, dtype=np.uint32 if bits == 32 else np.uint64)
    out = (C.c_uint64 * 6)()
    lib().qo_encode_cycles(bits, ids.ctypes.data, len(ids), t, S.ctypes.data, C.cast(out, C.POINTER(C.c_uint64)))
    return [int(v) for v in S], {"core_cycles": out[0] or None, "instructions": out[1] or None, "tsc": out[2],
                                 "ns": out[3], "clock_probe_ghz": out[4] / 1e6 if out[4] else None,
                                 "perf_errno": out[5] or None}


def encode_mt(ids, t, threads):
    """All-cores restatement over a pre-generated id array (one partial per
    thread over a contiguous slice, merged)."""
    bits = 32 if ids.dtype == np.uint32 else 64
    ids = np.ascontiguousarray(ids)
    S = np.zeros(t, dtype=np.uint32 if bits == 32 else np.uint64)
    rc = lib().qo_encode_mt(bits, ids.ctypes.data, len(ids), t, threads, S.ctypes.data)
    if rc:
        raise RuntimeError(f"qo_encode_mt rc={rc}")
    return [int(v) for v in S]


def bench_construct(bits, seed, n, t, trials):
    """Reference-shape CPU microbenchmark: mean ns per id over `trials`
    construct-and-insert-n-ids runs (BASELINE.md's `-e 1000` rows)."""
    sink = C.c_uint64()
    ns = lib().qo_bench_construct(bits, seed, n, t, trials, C.byref(sink))
    return ns / max(1, n * trials)


def bench_decode(bits, n, d, trials):
    """Reference-shape CPU decode microbenchmark (benchmark_decode -n N -d D
    -t D): mean microseconds per subtract + to_coeffs + root test over n,
    and the hits found."""
    found = C.c_uint64()
    ns = lib().qo_bench_decode(bits, n, d, trials, C.byref(found))
    return ns / max(1, trials) / 1e3, found.value


def encode_u64(ids, t):
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    S = np.zeros(t, dtype=np.uint64)
    lib().qo_encode_u64(_p(ids, C.c_uint64), len(ids), t, _p(S, C.c_uint64))
    return [int(v) for v in S]


def encode_u64_seed(seed, n, t, start=0):
    S = np.zeros(t, dtype=np.uint64)
    lib().qo_encode_u64_seed(seed, start, n, t, _p(S, C.c_uint64))
    return [int(v) for v in S]


def to_coeffs_u32(S):
    S = np.ascontiguousarray(S, dtype=np.uint32)
    c = np.zeros(len(S), dtype=np.uint32)
    lib().qo_to_coeffs_u32(_p(S, C.c_uint32), len(S), _p(c, C.c_uint32))
    return [int(v) for v in c]


def to_coeffs_u64(S):
    S = np.ascontiguousarray(np.array([int(v) for v in S], dtype=np.uint64))
    c = np.zeros(len(S), dtype=np.uint64)
    lib().qo_to_coeffs_u64(_p(S, C.c_uint64), len(S), _p(c, C.c_uint64))
    return [int(v) for v in c]


def root_test_u32(coeffs, log, cap=1 << 20):
    c = np.ascontiguousarray(coeffs, dtype=np.uint32)
    log = np.ascontiguousarray(log, dtype=np.uint32)
    hits = np.zeros(cap, dtype=np.int64)
    nh = lib().qo_root_test_u32(_p(c, C.c_uint32), len(c), _p(log, C.c_uint32), len(log), _p(hits, C.c_int64), cap)
    return hits[:min(nh, cap)].copy(), int(nh)


def root_test_u64(coeffs, log, cap=1 << 20):
    c = np.ascontiguousarray(np.array([int(v) for v in coeffs], dtype=np.uint64))
    log = np.ascontiguousarray(log, dtype=np.uint64)
    hits = np.zeros(cap, dtype=np.int64)
    nh = lib().qo_root_test_u64(_p(c, C.c_uint64), len(c), _p(log, C.c_uint64), len(log), _p(hits, C.c_int64), cap)
    return hits[:min(nh, cap)].copy(), int(nh)
