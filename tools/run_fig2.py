#!/usr/bin/env python3
"""Run the reference's figure-2 microbenchmark command lines against the
drop-in programs (target/release/examples/benchmark_{construct,decode}) and
write logs in the reference's log format — the command line, then the
program's SUMMARY lines — to OUT/{threshold_vs_encode_time,
num_missing_vs_decode_time,num_candidates_vs_decode_time}/{32,64}.txt, the
layout figures/fig2_microbenchmarks.py reads (its parsers at :25-69 consume
them unchanged).  Also writes OUT/summary.json: per point our avg beside the
published one (profiles/published/quack_logs.json).  Not product code.

    python tools/run_fig2.py OUT [--trials 100] [--gpu] [--quick]
"""
import argparse
import json
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "target", "release", "examples")


def us(v):
    m = re.fullmatch(r"([0-9.]+)(ns|µs|ms|s)", v)
    return float(m.group(1)) * {"ns": 1e-3, "µs": 1.0, "ms": 1e3, "s": 1e6}[m.group(2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--gpu", action="store_true", help="add --gpu (device batch paths) to every command")
    ap.add_argument("--quick", action="store_true", help="every 4th point")
    args = ap.parse_args()
    pub = json.load(open(os.path.join(ROOT, "profiles", "published", "quack_logs.json")))
    step = 4 if args.quick else 1
    sweeps = {
        "threshold_vs_encode_time": ("benchmark_construct", [(t, ["-e", "1000", "--trials", str(args.trials),
                                                                  "-t", str(t)]) for t in range(10, 310, 10)]),
        "num_missing_vs_decode_time": ("benchmark_decode", [(d, ["-n", "300", "--trials", str(args.trials),
                                                                 "-d", str(d), "-t", str(d)])
                                                            for d in range(5, 301, 5)]),
        "num_candidates_vs_decode_time": ("benchmark_decode", [(n, ["-d", "10", "-t", "10", "--trials",
                                                                    str(args.trials), "-n", str(n)])
                                                               for n in range(10, 301, 5)]),
    }
    summary = []
    for kind, (prog, points) in sweeps.items():
        os.makedirs(os.path.join(args.out, kind), exist_ok=True)
        for bits in (32, 64):
            lines = []
            for x, a in points[::step]:
                cmd = [f"./target/release/examples/{prog}", "power-sum", *a, "-b", str(bits)]
                if bits == 64:
                    cmd.append("--montgomery")
                if args.gpu:
                    cmd.append("--gpu")
                r = subprocess.run([os.path.join(BIN, prog), *cmd[1:]], capture_output=True, text=True,
                                   timeout=600, cwd=ROOT)
                lines.append(" ".join(cmd))
                lines += [l for l in (r.stdout + r.stderr).splitlines() if l.strip()]
                m = re.search(r"avg = (\S+)", r.stderr)
                p = pub[kind][str(bits)].get(str(x), {})
                summary.append({"sweep": kind, "bits": bits, "x": x, "avg_us": us(m.group(1)) if m else None,
                                "published_avg_us": p.get("avg_us"), "rc": r.returncode})
            with open(os.path.join(args.out, kind, f"{bits}.txt"), "w") as f:
                f.write("\n".join(lines) + "\n")
    with open(os.path.join(args.out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=0)
    ok = [s for s in summary if s["avg_us"] and s["published_avg_us"]]
    faster = sum(s["avg_us"] < s["published_avg_us"] for s in ok)
    print(json.dumps({"points": len(summary), "with_published": len(ok), "faster_than_published": faster}))


if __name__ == "__main__":
    main()
