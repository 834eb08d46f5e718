#!/usr/bin/env python3
"""A process's first flow batch against its steady state.

One fresh process per flow count: torch generates the records in HBM, then
the FIRST qk_ctx_create of the process and its first
qk_u32_encode_flows_device call are timed (context creation apart), then
--steady further calls.  Prints one JSON line.

    python tools/flows_cold.py --flows 16 [--npkts 1e8 --steady 8]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=float, default=16)
    ap.add_argument("--npkts", type=float, default=1e8)
    ap.add_argument("--steady", type=int, default=8)
    ap.add_argument("--t", type=int, default=32)
    a = ap.parse_args()
    import torch
    from bench import make_records
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import Context, PktStats
    dev = "cuda:0"
    n, nflows, t = int(a.npkts), int(a.flows), a.t
    raw, rec, g = make_records(dev, n, 11)
    f = torch.randint(0, nflows, (n,), device=dev, generator=g, dtype=torch.int64)
    for k in range(4):
        rec[:, 26 + k] = ((f >> (8 * k)) & 255).to(torch.uint8)
    del f
    rsz = lib().qk_u32_size(t)
    keys = torch.empty((nflows, 12), dtype=torch.uint8, device=dev)
    sks = torch.empty((nflows, rsz // 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx = Context(0)
    create_ms = (time.perf_counter() - t0) * 1e3
    times = []
    nf, st = C.c_size_t(), PktStats()
    for _ in range(a.steady + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib().qk_u32_encode_flows_device(ctx.handle, raw.data_ptr(), n, 67, None, None, t, keys.data_ptr(),
                                              sks.data_ptr(), nflows, C.byref(nf), C.byref(st), None)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        if rc:
            raise SystemExit(f"rc={rc}")
    steady = float(np.median(times[1:]))
    print(json.dumps({"flows": nflows, "npkts": n, "ctx_create_ms": create_ms, "first_ms": times[0],
                      "steady_ms_median": steady, "first_over_steady": times[0] / steady,
                      "all_ms": times, "flows_out": int(nf.value), "inserted": int(st.inserted)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
