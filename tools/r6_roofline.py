#!/usr/bin/env python3
"""Roofline rows of the bench run's kernels (round 6: bench.py's N = 1 run
now carries every single-GPU config, so one kernel trace and one FETCH_SIZE
pass of `python bench.py` cover them all; not product code):

  <dir>/prof/run_kernel_trace.csv     rocprofv3 --kernel-trace (per dispatch)
  <dir>/pmc/run_counter_collection.csv rocprofv3 --pmc FETCH_SIZE

Per kernel, the dispatches over the config's full array are the ones that
take at least half the kernel's longest duration (the same kernels also run
on the configs' smaller arrays: the CPU-baseline prefix, the packet check's
reference encode); average duration and FETCH_SIZE x 1024 x 2 bytes (the
gfx950 correction, MI355X_MICROARCH.md) over those.  Algorithmic bytes per
launch: SURVEY.md §8(d)'s per-unit bytes x the config's units.

    python tools/r6_roofline.py profiles/r06/final > profiles/r06/final/roofline.json
"""
import csv
import json
import os
import sys

PEAK_GBPS = 8000.0
ROWS = [("void qk::k_encode_u32_bsgs<8, 4, 8, 1>", 4.0e9, "configs[1] (the bench line): encode 1e9 u32 ids, t=32"),
        ("void qk::k_encode_u64_bsgs<10, 14, 1>", 8.0e9, "configs[2]: encode 1e9 u64 ids, t=80"),
        ("void qk::k_root_scan_k<unsigned int, 1>", 4.0e8, "configs[4]: root-set scan of 1e8 u32 candidates, d=32"),
        ("void qk::k_root_scan_k<unsigned long, 1>", 8.0e8, "configs[4] u64 twin: root-set scan of 1e8 u64 candidates"),
        ("qk::k_flow_extract", 6.7e9, "f1: per-flow extract of 1e8 x 67-byte records, 1e6 flows (record bytes)"),
        ("void qk::k_pkt_kernel<qk::NoEncode, true>", 6.7e9, "f2: packet extract of 1e8 x 67-byte records (record bytes)")]


def main(d):
    trace = list(csv.DictReader(open(os.path.join(d, "prof", "run_kernel_trace.csv"))))
    pmc_path = os.path.join(d, "pmc", "run_counter_collection.csv")
    pmc = list(csv.DictReader(open(pmc_path))) if os.path.exists(pmc_path) else []
    out = []
    for prefix, alg, cfg in ROWS:
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in trace
              if r["Kernel_Name"].startswith(prefix)]
        if not ds:
            out.append({"config": cfg, "kernel": prefix, "missing": True})
            continue
        big = [x for x in ds if x >= 0.5 * max(ds)]
        avg = sum(big) / len(big)
        fs = [float(r["Counter_Value"]) for r in pmc if r["Kernel_Name"].startswith(prefix)
              and r["Counter_Name"] == "FETCH_SIZE"]
        fbig = [x for x in fs if x >= 0.5 * max(fs)] if fs else []
        traffic = sum(fbig) / len(fbig) * 1024 * 2 if fbig else None
        ach = alg / avg / 1e9
        out.append({"config": cfg, "kernel": prefix, "launches": len(big), "avg_ms": avg * 1e3,
                    "algorithmic_bytes": alg, "achieved_GBps": ach, "peak_GBps": PEAK_GBPS, "frac": ach / PEAK_GBPS,
                    "traffic_bytes": traffic, "traffic_over_algorithmic": traffic / alg if traffic else None})
    print(json.dumps({"source": d, "rows": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
