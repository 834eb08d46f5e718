#!/usr/bin/env python3
"""Extract the reference's published quack microbenchmark numbers (the raw
logs in /root/reference/nsdi24_raw_data.zip, nsdi24/quack/*) into a small
JSON fixture, profiles/published/quack_logs.json, so that benchmarks on the
GPU box (where /root/reference does not exist) can print them beside their
own rows.  Data only: (command shape, avg time) pairs parsed the same way as
the reference's figures/fig2_microbenchmarks.py:25-69.  Run in this
container; the output is committed.

    python tools/extract_published.py
"""
import json
import os
import re
import zipfile

ZIP = "/root/reference/nsdi24_raw_data.zip"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "published",
                   "quack_logs.json")


def us(v):
    if v.endswith("ms"):
        return float(v[:-2]) * 1000
    if v.endswith("µs"):
        return float(v[:-2])
    if v.endswith("ns"):
        return float(v[:-2]) / 1000
    raise ValueError(v)


def parse(text, x_regex):
    """x -> {avg_us, avg_cycles, per_packet_ns} from a benchmark log."""
    out, x = {}, None
    for line in text.split("\n"):
        m = re.match(x_regex, line)
        if m:
            x = int(m.group(1))
            continue
        m = re.match(r".*SUMMARY: num_trials = (\d+), avg_cycles = (\d+), avg = (\S+)", line)
        if m and x is not None:
            out.setdefault(x, {})["avg_us"] = us(m.group(3))
            out[x]["avg_cycles"] = int(m.group(2))
            out[x]["trials"] = int(m.group(1))
            continue
        m = re.match(r".*SUMMARY \(per-packet\): (\S+)/packet", line)
        if m and x is not None:
            out.setdefault(x, {})["per_packet_ns"] = us(m.group(1)) * 1000
    return out


def main():
    z = zipfile.ZipFile(ZIP)
    res = {"source": "nsdi24_raw_data.zip: nsdi24/quack/{threshold_vs_encode_time,num_missing_vs_decode_time,"
                     "num_candidates_vs_decode_time}/{16,32,64}.txt (logged 2024-02-13, Intel Xeon E5, 1 core, "
                     "quack crate examples benchmark_construct / benchmark_decode)",
           "parser": "figures/fig2_microbenchmarks.py:25-69 (avg = per-trial time; per-packet = avg / n)"}
    for kind, rx, cmd in (("threshold_vs_encode_time", r".*-t (\d+)", "benchmark_construct power-sum -e 1000 "
                                                                       "--trials 100 -t T -b B"),
                          ("num_missing_vs_decode_time", r".*-d (\d+).*", "benchmark_decode power-sum -n 300 "
                                                                          "--trials 100 -d D -t D -b B"),
                          ("num_candidates_vs_decode_time", r".*-n (\d+)", "benchmark_decode power-sum -d 10 -t 10 "
                                                                           "--trials 100 -b B -n N")):
        res[kind] = {"command": cmd}
        for bits in (16, 32, 64):
            res[kind][str(bits)] = {str(k): v for k, v in sorted(parse(z.read(f"nsdi24/quack/{kind}/{bits}.txt")
                                                                         .decode(), rx).items())}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(OUT, {k: {b: len(v) for b, v in res[k].items() if b.isdigit()} for k in res if k.endswith("time")})


if __name__ == "__main__":
    main()
