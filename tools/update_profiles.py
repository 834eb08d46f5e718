#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of a gpu_check.sh run (gpurun_out/) into
profiles/<round>/ and refresh profiles/pmc_encode.json (the per-launch HBM
traffic bench.py reports).  FETCH_SIZE is KiB and, on gfx950, half the bytes
of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM): bytes = 2 *
FETCH_SIZE * 1024."""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(rnd: str, src: str = "gpurun_out", key: str = "u32_t32", n_ids: int = 1_000_000_000):
    src = os.path.join(ROOT, src)
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    copies = {"prof/run_kernel_stats.csv": "encode_kernel_stats.csv",
              "pmc/run_counter_collection.csv": "encode_pmc_fetch_size.csv",
              "pmcsq/run_counter_collection.csv": "encode_pmc_sq.csv",
              "ubench.log": "ubench_int.json", "tune.log": "tune_encode.json", "ubdep.log": "ubench_dep.json",
              "tunebsgs.log": "tune_bsgs.json", "ubissue.log": "ubench_issue.json",
              "proflows/run_kernel_stats.csv": "flows_packets_kernel_stats.csv",
              "pytest.log": "pytest_gpu.log", "smoke.log": "smoke.log"}
    for a, b in copies.items():
        if os.path.exists(os.path.join(src, a)):
            shutil.copy(os.path.join(src, a), os.path.join(dst, b))
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        lines = [l for l in open(bench) if l.startswith("{")]
        if lines:
            open(os.path.join(dst, "bench_n1.json"), "w").write(lines[-1])

    # tools/bench_configs.py rows (configs*.log): one JSON object per line
    rows = []
    for name in sorted(os.listdir(src)):
        if name.startswith("configs") and name.endswith(".log"):
            rows += [l for l in open(os.path.join(src, name)) if l.startswith("{")]
    if rows:   # merged by "config": a partial run refreshes its own rows only
        path = os.path.join(dst, "configs.jsonl")
        merged = collections.OrderedDict()
        if os.path.exists(path):
            for l in open(path):
                if l.startswith("{"):
                    merged[json.loads(l)["config"]] = l
        for l in rows:
            merged[json.loads(l)["config"]] = l
        open(path, "w").write("".join(merged.values()))

    out = {}
    pmc = os.path.join(src, "pmc/run_counter_collection.csv")
    if os.path.exists(pmc):
        rows = [r for r in csv.DictReader(open(pmc)) if "k_encode_u32" in r["Kernel_Name"]]
        fs = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "FETCH_SIZE"]
        if fs:
            avg = sum(fs) / len(fs)
            out = {"kernel": rows[0]["Kernel_Name"].split("(")[0], "n_ids": n_ids, "launches": len(fs),
                   "fetch_size_kib_avg": avg, "hbm_read_bytes_corrected": 2 * avg * 1024,
                   "algorithmic_bytes": 4 * n_ids, "ratio_to_algorithmic": 2 * avg * 1024 / (4 * n_ids)}
    sq = os.path.join(src, "pmcsq/run_counter_collection.csv")
    if os.path.exists(sq):
        agg = collections.defaultdict(dict)
        for r in csv.DictReader(open(sq)):
            if "k_encode_u32" in r["Kernel_Name"]:
                agg[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        if agg:
            last = list(agg.values())[-1]
            out["sq_counters_last_launch"] = last
            if "SQ_INSTS_VALU" in last:
                out["valu_wave_insts_per_id"] = last["SQ_INSTS_VALU"] / n_ids
    if out:
        path = os.path.join(ROOT, "profiles", "pmc_encode.json")
        d = json.load(open(path)) if os.path.exists(path) else {}
        d["source"] = f"tools/gpu_check.sh pmc/pmcsq steps ({rnd}): rocprofv3 --pmc over bench.py --steps 3"
        d["note"] = ("FETCH_SIZE is in KiB; on gfx950 it reports half the bytes of a wide coalesced streaming "
                     "read (MI355X_MICROARCH.md §HBM), so bytes = 2 * FETCH_SIZE * 1024")
        d.setdefault("encode", {})[key] = out
        json.dump(d, open(path, "w"), indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
