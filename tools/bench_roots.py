#!/usr/bin/env python3
"""Host root finding (roots.cpp, qk_u32_roots / qk_u64_roots) on the decode
case: the coefficients of a product of d distinct linear factors (random
GF(p) roots), the call timed directly through ctypes (prebuilt arrays),
min and median over many calls — the min is robust to a shared host — for
each of --sets root sets (the time depends on how the roots fall into the
splitting classes); min_us / median_us are the first set's (the round-4
figures), mean_min_us the mean of the sets' minima.

    python tools/bench_roots.py [--d 8,16,32,64] [--reps 200] [--sets 8]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def coeffs_of(roots, p):
    """z^d + c_1 z^(d-1) + ... + c_d = prod (z - r), as to_coeffs writes them."""
    poly = [1]
    for r in roots:
        nxt = [0] * (len(poly) + 1)
        for i, c in enumerate(poly):
            nxt[i] = (nxt[i] + c) % p
            nxt[i + 1] = (nxt[i + 1] - c * r) % p
        poly = nxt
    return poly[1:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", default="8,16,32,64")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--sets", type=int, default=8)
    a = ap.parse_args()
    from sidekick_amd._lib import P32, P64, lib
    rng = np.random.default_rng(7)
    for bits, p, f, T in ((32, P32, lib().qk_u32_roots, C.c_uint32), (64, P64, lib().qk_u64_roots, C.c_uint64)):
        for d in (int(x) for x in a.d.split(",")):
            mins, med0 = [], None
            for _ in range(a.sets):
                roots = sorted(set(int(x) % p for x in rng.integers(1, 2**63, size=d)))
                c = coeffs_of(roots, p)
                carr = (T * len(c))(*c)
                out = (T * (d + 1))()
                k = C.c_uint32()
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    rc = f(carr, len(c), out, d + 1, C.byref(k))
                    ts.append(time.perf_counter() - t0)
                assert rc == 0 and sorted(out[: k.value]) == roots
                mins.append(min(ts) * 1e6)
                if med0 is None:
                    med0 = float(np.median(ts)) * 1e6
            print(json.dumps({"bits": bits, "d": d, "min_us": mins[0], "median_us": med0, "reps": a.reps,
                              "sets": a.sets, "mean_min_us": float(np.mean(mins)), "set_min_us": mins}), flush=True)


if __name__ == "__main__":
    main()
