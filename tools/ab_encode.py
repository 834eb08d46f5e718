#!/usr/bin/env python3
"""Same-process A/B of an encode knob (default grid_mult): per threshold the
knob values alternate for several rounds over the same device-resident ids,
each value's partial sums must equal the first value's, and the median
kernel time per encode (the context's profiled launches) is reported.

    python tools/ab_encode.py [--knob grid_mult] [--values 3,1] [--bits 32]
                              [--t 8,16,20,32,40,64,80] [--n 2.5e8] [--rounds 6]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="grid_mult")
    ap.add_argument("--values", default="3,1")
    ap.add_argument("--bits", type=int, default=32)
    ap.add_argument("--t", default="8,12,16,20,24,28,30,32,36,40,42,48,56,64,72,80")
    ap.add_argument("--n", type=float, default=2.5e8)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--default", type=int, default=None, help="value restored afterwards (default: the first)")
    a = ap.parse_args()
    import torch
    import sidekick_amd as sk
    from bench_configs import DEV, fill_splitmix, partial_words, time_encode
    ctx = sk.get_context(0)
    n = int(a.n)
    dt = torch.int32 if a.bits == 32 else torch.int64
    ids = torch.empty(n, dtype=dt, device=DEV)
    fill_splitmix(ctx, ids, 0x5EED0002 if a.bits == 32 else 0x5EED0003, bits=a.bits)
    values = [int(v) for v in a.values.split(",")]
    from sidekick_amd.quack import encode_device_async
    for t in (int(x) for x in a.t.split(",")):
        times = {v: [] for v in values}
        ref, same = None, {v: True for v in values}
        for r in range(a.rounds):
            for v in values:
                ctx.set_knob(a.knob, v)
                _, kern = time_encode(ctx, ids, t, a.bits, a.steps)
                times[v].append(kern)
                part = torch.zeros(partial_words(t, a.bits), dtype=torch.int64, device=DEV)
                encode_device_async(ctx, ids, t, part, bits=a.bits)
                out = part.cpu().numpy().tobytes()
                if ref is None:
                    ref = out
                elif out != ref:
                    same[v] = False
        ctx.set_knob(a.knob, values[0] if a.default is None else a.default)
        med = {str(v): float(np.median(times[v])) * 1e3 for v in values}
        print(json.dumps({"bits": a.bits, "t": t, "n": n, "knob": a.knob, "median_ms": med,
                          "min_ms": {str(v): float(np.min(times[v])) * 1e3 for v in values},
                          "ids_per_s": {str(v): n / (med[str(v)] * 1e-3) for v in values},
                          "gain_first_vs_last": med[str(values[-1])] / med[str(values[0])] - 1,
                          "identical_to_first_value": same}), flush=True)


if __name__ == "__main__":
    main()
