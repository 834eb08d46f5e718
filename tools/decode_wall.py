#!/usr/bin/env python3
"""configs[4]'s decode call alone (bench.py cfg_decode): the timed
qk_u*_decode_device over the 1e8-id log with 32 drops, u32 and/or u64, one
JSON line each — for tracing the call (rocprofv3 --kernel-trace
--hip-runtime-trace) and for decode A/Bs.

    python tools/decode_wall.py [--bits 32,64] [--reps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", default="32,64")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--knob", action="append", default=[], help="NAME=V1,V2: alternate the values (A/B)")
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    import bench
    import sidekick_amd as sk
    ctx = sk.get_context(0)
    ab = [(k, [int(v) for v in vs.split(",")]) for k, vs in (kv.split("=") for kv in a.knob)] or [(None, [None])]
    for _ in range(a.rounds):
        for k, vals in ab:
            for v in vals:
                if k:
                    ctx.set_knob(k, v)
                for b in (int(x) for x in a.bits.split(",")):
                    r = bench.cfg_decode(ctx, 0, b, reps=a.reps)
                    r["knob"] = {k: v} if k else None
                    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
