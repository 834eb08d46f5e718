#!/usr/bin/env python3
"""Same-process A/B of a flow-batch knob (default flow_hist: the few-flow
histogram grouping against the radix sort): per flow count, the modes alternate,
every mode's output (keys + sketches, device-resident) must equal mode 0's
byte for byte, and the median wall time of the synchronous call is reported.

    python tools/ab_flows.py [--knob flow_hist] [--modes 32,0] [--flows 10000,1000000] [--rounds 4]
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
    ap.add_argument("--knob", default="flow_hist")
    ap.add_argument("--modes", default="32,0")
    ap.add_argument("--flows", default="10000,1000000")
    ap.add_argument("--npkts", type=float, default=1e8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--host-check", type=int, default=0,
                    help="1: compare outputs on the host (pageable copies between calls), 0: on the device")
    ap.add_argument("--cold", type=int, default=0,
                    help="1: every call on a fresh context (no flow-count hint: the table starts small and regrows)")
    ap.add_argument("--default", type=int, default=None, help="knob value restored afterwards (default: the first mode)")
    a = ap.parse_args()
    import torch
    import sidekick_amd as sk
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import Context, PktStats
    ctx = sk.get_context(0)
    dev = "cuda:0"
    n, stride, t = int(a.npkts), 67, a.t
    raw = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    raw.random_(0, 256, generator=g)
    rec = raw.view(n, stride)
    rec[:, 23] = 17
    modes = [int(m) for m in a.modes.split(",")]
    rsz = lib().qk_u32_size(t)
    for nflows in (int(float(f)) for f in a.flows.split(",")):
        f = torch.randint(0, nflows, (n,), device=dev, generator=g, dtype=torch.int64)
        for k in range(4):
            rec[:, 26 + k] = ((f >> (8 * k)) & 255).to(torch.uint8)
        rec[:, 30:38] = torch.tensor([192, 168, 0, 9, 0x11, 0x5C, 0x1F, 0x90], dtype=torch.uint8, device=dev)
        del f
        keys = torch.empty((nflows, 12), dtype=torch.uint8, device=dev)
        sks = torch.empty((nflows, rsz // 4), dtype=torch.int32, device=dev)
        times = {m: [] for m in modes}
        ref = None
        same = {m: True for m in modes}
        for r in range(a.rounds + 1):
            for m in modes:
                if a.cold:
                    ctx = Context(0)
                ctx.set_knob(a.knob, m)
                nf, st = C.c_size_t(), PktStats()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = lib().qk_u32_encode_flows_device(ctx.handle, raw.data_ptr(), n, stride, None, None, t,
                                                      keys.data_ptr(), sks.data_ptr(), nflows, C.byref(nf),
                                                      C.byref(st), 0)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                if rc != 0:
                    raise SystemExit(f"rc={rc} at {a.knob}={m}")
                if a.cold:
                    torch.cuda.synchronize()
                if r:
                    times[m].append(dt)
                if a.host_check:
                    out = (keys[: nf.value].cpu().numpy().tobytes(), sks[: nf.value].cpu().numpy().tobytes())
                    if ref is None:
                        ref = out
                    elif out != ref:
                        same[m] = False
                elif ref is None:
                    ref = (keys[: nf.value].clone(), sks[: nf.value].clone())
                elif not (torch.equal(keys[: nf.value], ref[0]) and torch.equal(sks[: nf.value], ref[1])):
                    same[m] = False
                if a.cold:
                    ctx.close()
        if not a.cold:
            ctx.set_knob(a.knob, modes[0] if a.default is None else a.default)
        print(json.dumps({"flows": nflows, "n_packets": n, "t": t, "knob": a.knob,
                          "median_ms": {str(m): float(np.median(times[m])) * 1e3 for m in modes},
                          "min_ms": {str(m): float(np.min(times[m])) * 1e3 for m in modes},
                          "identical_to_first_mode": same}), flush=True)


if __name__ == "__main__":
    main()
