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
    a = ap.parse_args()
    import bench
    import sidekick_amd as sk
    ctx = sk.get_context(0)
    for b in (int(x) for x in a.bits.split(",")):
        print(json.dumps(bench.cfg_decode(ctx, 0, b, reps=a.reps)), flush=True)


if __name__ == "__main__":
    main()
