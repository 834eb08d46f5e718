#!/usr/bin/env python3
"""Where configs[4]'s decode wall goes: the pieces of qk_u*_decode_device
timed one by one through the C ABI (medians over --reps calls each):

  coeffs    qk_u*_to_coeffs (host Newton identities)
  roots     qk_u*_roots on those coefficients (host root finding)
  rt        qk_u*_root_test_device with the coefficients (roots + scan + hand-back)
  rt_tiny   the same on a 64-entry log (the fixed cost: roots, launch, wait)
  decode    qk_u*_decode_device (everything)
  scan      the scan kernel alone (HIP events, profiled calls)

    python tools/decode_parts.py [--bits 32,64] [--reps 200]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", default="32,64")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import sidekick_amd as sk
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import fill_splitmix
    L = lib()
    ctx = sk.get_context(0)
    for bits in (int(x) for x in a.bits.split(",")):
        n, t = bench.DECODE_N, bench.DECODE_T
        seed = bench.DECODE_SEED + (bits == 64)
        T = C.c_uint32 if bits == 32 else C.c_uint64
        log_ = torch.empty(n, dtype=torch.int32 if bits == 32 else torch.int64, device="cuda:0")
        fill_splitmix(ctx, log_, seed, bits=bits)
        drops = np.sort(np.random.default_rng(seed).choice(n, bench.DECODE_DROPS, replace=False))
        keep = torch.ones(n, dtype=torch.bool, device="cuda:0")
        keep[torch.from_numpy(drops).to("cuda:0")] = False
        Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
        A, B = Q(t), Q(t)
        A.insert_batch(log_, ctx=ctx)
        B.insert_batch(log_[keep].contiguous(), ctx=ctx)
        diff = A.clone()
        diff.sub_assign(B)
        del keep
        torch.cuda.synchronize()
        f_coeffs = getattr(L, f"qk_u{bits}_to_coeffs")
        f_roots = getattr(L, f"qk_u{bits}_roots")
        f_rt = getattr(L, f"qk_u{bits}_root_test_device")
        f_dec = getattr(L, f"qk_u{bits}_decode_device")
        coeffs = (T * t)()
        d = C.c_uint32()
        roots = (T * t)()
        k = C.c_uint32()
        cap = 1 << 12
        hits = (C.c_uint64 * cap)()
        nh = C.c_size_t()
        tiny = log_[:64].contiguous()
        torch.cuda.synchronize()
        res = {}

        def timeit(name, fn, reps=a.reps):
            ts = []
            for r in range(reps + 5):
                t0 = time.perf_counter()
                rc = fn()
                dt = time.perf_counter() - t0
                assert rc == 0, (name, rc)
                if r >= 5:
                    ts.append(dt * 1e6)
            res[name] = {"median_us": med(ts), "min_us": min(ts)}

        timeit("coeffs", lambda: f_coeffs(diff._buf, coeffs, t, C.byref(d)))
        timeit("roots", lambda: f_roots(coeffs, d.value, roots, t, C.byref(k)))
        timeit("rt", lambda: f_rt(ctx.handle, coeffs, d.value, log_.data_ptr(), n, 1, diff.last_value(), hits, cap,
                                  C.byref(nh), None))
        timeit("rt_tiny", lambda: f_rt(ctx.handle, coeffs, d.value, tiny.data_ptr(), 64, 0, 0, hits, cap,
                                       C.byref(nh), None))
        timeit("decode", lambda: f_dec(ctx.handle, diff._buf, log_.data_ptr(), n, 1, hits, cap, C.byref(nh), None))
        ctx.kernel_stats()
        ctx.set_profiling(True)
        for _ in range(30):
            f_dec(ctx.handle, diff._buf, log_.data_ptr(), n, 1, hits, cap, C.byref(nh), None)
        ctx.set_profiling(False)
        kms, kc = ctx.kernel_stats()
        res["scan_kernel_us_mean"] = kms * 1e3 / max(kc, 1)
        res["bits"] = bits
        res["d"] = d.value
        res["roots_found"] = k.value
        print(json.dumps(res), flush=True)
        del log_, tiny


if __name__ == "__main__":
    main()
