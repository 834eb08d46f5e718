#!/usr/bin/env python3
"""The reference's decode microbenchmark shapes, beside its published logs.

Runs tools/bench_decode (C against include/quack_hip.h: the product's host
path qk_*_decode_host and device path qk_*_decode_device) and the oracle's
CPU port (oracle/quack_oracle.c qo_bench_decode) over the two sweeps of
figures/fig2_microbenchmarks.py:
  num_missing_vs_decode_time     -n 300 -d D -t D   (D = 5..300)      :175-183
  num_candidates_vs_decode_time  -d 10 -t 10 -n N   (N = 10..300)     :134-141
for u32 and u64 ids, and prints one JSON row per point with the published
avg (profiles/published/quack_logs.json, Xeon E5, the quack crate).  Not
part of the product.

    python tools/bench_decode.py [--trials 100] [--quick] > rows.jsonl
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_c(bits, mode, trials, points):
    out = subprocess.run([os.path.join(ROOT, "tools", "bench_decode"), str(bits), mode, str(trials)]
                         + [f"{n}:{d}" for n, d in points], capture_output=True, text=True, check=True)
    return {(r["n"], r["d"]): r for r in (json.loads(l) for l in out.stdout.splitlines() if l.startswith("{"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--quick", action="store_true", help="every 4th point only")
    ap.add_argument("--no-device", action="store_true")
    args = ap.parse_args()
    from oracle import coracle
    with open(os.path.join(ROOT, "profiles", "published", "quack_logs.json")) as f:
        pub = json.load(f)
    step = 20 if args.quick else 5
    sweeps = {"num_missing_vs_decode_time": [(300, d) for d in range(5, 301, step)],
              "num_candidates_vs_decode_time": [(n, 10) for n in range(10, 301, step)]}
    for bits in (32, 64):
        for sweep, points in sweeps.items():
            host = run_c(bits, "host", args.trials, points)
            dev = {} if args.no_device else run_c(bits, "device", args.trials, points)
            for n, d in points:
                key = str(d) if sweep.startswith("num_missing") else str(n)
                p = pub[sweep][str(bits)].get(key, {})
                port_us, found = coracle.bench_decode(bits, n, d, max(5, args.trials // 4))
                row = {"config": f"decode u{bits} n={n} d=t={d}", "sweep": sweep, "bits": bits, "n": n, "d": d,
                       "published_us": p.get("avg_us"), "cpu_port_us": round(port_us, 3),
                       "host_us": host[(n, d)]["avg_us"], "gpu_us": dev[(n, d)]["avg_us"] if dev else None,
                       "hits": host[(n, d)]["hits"], "port_hits": found}
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
