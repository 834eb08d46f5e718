#!/usr/bin/env python3
"""Roofline rows for the secondary BASELINE configs' kernels, recomputed from
the committed rocprofv3 CSVs of one round (not part of the product):

  <round>/configs_kernel_stats.csv   --kernel-trace --stats (average duration)
  <round>/configs_pmc_fetch_size.csv --pmc FETCH_SIZE
  <round>/configs_pmc_sq.csv         --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE

all three collected on `tools/bench_configs.py u64 decode decode64`, plus
the integer-issue roofline of each kernel from <round>/issue_roofline.json
(tools/issue_roofline.py: VALU instructions per unit x the mean issue cost
of the kernel's hot-loop mix, against the SIMD-cycles per unit of the
profiled launch at its GRBM_GUI_ACTIVE clock).
Algorithmic bytes: 8 B per u64 id (encode), 4 / 8 B per u32 / u64 candidate
(root test), one launch = the whole array.  HBM traffic =
FETCH_SIZE KiB x 1024 x 2 (the gfx950 correction of MI355X_MICROARCH.md, as
tools/update_profiles.py).  Instruction counts are wave-instructions; x64 =
lane operations.

    python tools/config_roofline.py profiles/r03 > profiles/r03/configs_roofline.json
"""
import collections
import csv
import json
import os
import sys

PEAK_GBPS = 8000.0
# (kernel name prefix, units, bytes per unit, config, issue_roofline.json key):
# the first profiled kernel whose name starts with the prefix (the template
# arguments change between rounds), its most frequent grid in the PMC files
ROWS = [("void qk::k_encode_u64_bsgs<10,", 1_000_000_000, 8,
         "configs[2]: encode 1e9 u64 ids, t=80", "encode_u64_t80"),
        ("void qk::k_root_scan<unsigned int, 1", 100_000_000, 4,
         "configs[4]: root test of 1e8 u32 candidates, d=32 — root-set scan (the default)", "root_scan_u32_d32"),
        ("void qk::k_root_test_u32<32>", 100_000_000, 4,
         "configs[4]: root test of 1e8 u32 candidates, d=32 — Horner", "root_test_u32_d32"),
        ("void qk::k_root_scan<unsigned long, 1", 100_000_000, 8,
         "root test of 1e8 u64 candidates, d=32 — root-set scan (the default)", "root_scan_u64_d32"),
        ("void qk::k_root_test_u64_bsgs<0>", 100_000_000, 8,
         "root test of 1e8 u64 candidates, d=32 — baby-step/giant-step Horner", "root_test_u64_d32")]


def main(d):
    stats = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(os.path.join(d, "configs_kernel_stats.csv")))}
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in ("configs_pmc_fetch_size.csv", "configs_pmc_sq.csv"):
        for r in csv.DictReader(open(os.path.join(d, f))):
            ctr[(r["Kernel_Name"].split("(")[0], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    issue = {}
    ip = os.path.join(d, "issue_roofline.json")
    if os.path.exists(ip):
        issue = json.load(open(ip))["kernels"]
    out = []
    for prefix, units, bpu, cfg, ikey in ROWS:
        name = next(n for n in stats if n.startswith(prefix))
        s = stats[name]
        key = max((k for k in ctr if k[0] == name), key=lambda k: len(ctr[k]["FETCH_SIZE"]))
        c = {k: sum(v) / len(v) for k, v in ctr[key].items()}
        avg_s = float(s["AverageNs"]) * 1e-9
        alg = units * bpu
        traffic = c["FETCH_SIZE"] * 1024 * 2
        gbps = alg / avg_s / 1e9
        out.append({"config": cfg, "kernel": name.replace("void ", ""), "launches": int(s["Calls"]),
                    "avg_ms": round(avg_s * 1e3, 4), "units_per_s": units / avg_s,
                    "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": PEAK_GBPS, "unit": "GB/s",
                                 "frac": round(gbps / PEAK_GBPS, 4), "traffic": traffic,
                                 "traffic_over_algorithmic": round(traffic / alg, 4)},
                    "valu_wave_insts_per_unit": round(c["SQ_INSTS_VALU"] / units, 3),
                    "valu_lane_ops_per_unit": round(c["SQ_INSTS_VALU"] / units * 64, 1),
                    "salu_wave_insts_per_unit": round(c["SQ_INSTS_SALU"] / units, 3),
                    "lds_wave_insts_per_unit": round(c["SQ_INSTS_LDS"] / units, 3)})
        if ikey in issue:
            k = issue[ikey]
            out[-1]["valu"] = {"bound": "valu-issue", "unit": "SIMD-cycles/unit",
                               "peak": k["issue_cycles_per_unit_peak"],
                               "achieved": k["issue_cycles_per_unit_achieved"], "frac": k["frac"],
                               "mean_issue_cycles_per_valu": k["mean_issue_cycles_per_valu"],
                               "clock_ghz": k["clock_ghz"], "salu_busy": k["salu_busy"]}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
