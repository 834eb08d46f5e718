#!/usr/bin/env python3
"""configs[4]'s decode call (bench.cfg_decode) in a fresh process, then after
the configs block's u64 encode (bench.cfg_u64), then again: whether the
bench line's decode wall depends on what ran before it in the process."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import sidekick_amd as sk
    ctx = sk.get_context(0)
    keys = ("wall_us_median", "wall_us_min", "scan_kernel_us_median")
    for warm in (8, 60):
        r = bench.cfg_decode(ctx, 0, 32, warm=warm) if warm == 8 else bench.cfg_decode(ctx, 0, 32, reps=60, warm=warm)
        print(json.dumps({"when": f"fresh warm={warm}", **{k: r[k] for k in keys}}), flush=True)
    u = bench.cfg_u64(ctx, 0)
    print(json.dumps({"u64_kernel_ms": u["kernel_ms"]}), flush=True)
    for i in range(3):
        r = bench.cfg_decode(ctx, 0, 32)
        print(json.dumps({"when": f"after u64 #{i}", **{k: r[k] for k in keys}}), flush=True)


if __name__ == "__main__":
    main()
