#!/usr/bin/env python3
"""Integer-issue roofline of the hot kernels (BASELINE.md:61).

Every kernel of this path reads its bytes once (FETCH_SIZE = 1.000x the
algorithmic bytes) and is bound by instruction issue, not HBM.  This tool
turns the committed rocprofv3 SQ counters into that second roofline:

  per unit (id / candidate)   VALU and SALU wave-instructions (SQ_INSTS_VALU,
                              SQ_INSTS_SALU) / units per launch
  effective clock             GRBM_GUI_ACTIVE / 8 (the counter sums the 8
                              XCDs, MI355X_MICROARCH.md "DVFS give-back") /
                              the profiled dispatch's duration
  achieved issue cycles       SIMD-cycles the launch spent per unit:
                              clock * duration * 1024 SIMDs / units
  peak issue cycles           the fewest SIMD-cycles that issue the measured
                              VALU stream: VALU wave-instructions per unit x
                              the mean issue cost of the kernel's hot-loop
                              instruction mix, each instruction priced by the
                              measured per-class costs (profiles/r01/
                              ubench_issue.json, 8 waves/SIMD: a 2-source VALU
                              op 2.25 cycles, a 3-source op or one with an
                              SGPR/VCC result — v_mad_u64_u32, v_min3,
                              v_cmp, v_cndmask, v_addc — 4.19)
  frac                        peak / achieved: the fraction of the VALU issue
                              roofline the kernel reaches
  salu_busy                   SALU instructions per CU per cycle (one scalar
                              unit per CU, shared by its 4 SIMDs)

The hot-loop mix comes from the kernel's gfx950 assembly (`make -C
sidekick_amd/csrc asm`): the loop whose static VALU count per iteration
matches the measured VALU per unit (for a loop nest, the inner loop is
weighted by the trip count that makes the two agree).

    python tools/issue_roofline.py [--asm-dir sidekick_amd/csrc/_build/asm] [--out profiles/r03/issue_roofline.json]
    python tools/issue_roofline.py --bench profiles/r04/bench_n1.json

The second form is the bench line's figure (round 4 on): the peak is the
algorithmic anchor of tools/issue_model.py — the decomposition's VALU work,
fixed per t — not the measured instruction count, and the clock is the one
bench.py read in the same run (qk_clock_probe).  The counter-based analysis
above stays as the per-kernel diagnostic (how close the emitted instruction
stream is to the anchor, and how busy the scalar unit is).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
CUS = 256

# measured issue costs, SIMD cycles per wave64 instruction at 8 waves/SIMD
# (profiles/r01/ubench_issue.json: vadd8 17.97/8, vmad8 33.52/8)
COST_SIMPLE = 17.97 / 8
COST_HEAVY = 33.52 / 8

# kernel -> (asm file, symbol prefix, pmc csv, kernel-name substring, grid of the
#            measured launch, units per launch, units per hot-loop iteration per
#            wave, config label)
KERNELS = {
    "encode_u32_t32": ("encode.s", "_ZN2qk17k_encode_u32_bsgsILi8ELi4ELi8E", "profiles/r03/encode_pmc_sq.csv",
                       "k_encode_u32_bsgs<8, 4, 8>", "327680", 1e9, 256,
                       "configs[1]: encode 1e9 u32 ids, t=32 (the bench line)"),
    "encode_u64_t80": ("encode.s", "_ZN2qk17k_encode_u64_bsgsILi10ELi16E", "profiles/r03/configs_pmc_sq.csv",
                       "k_encode_u64_bsgs<10, 16>", "262144", 1e9, 64,
                       "configs[2]: encode 1e9 u64 ids, t=80"),
    "root_scan_u32_d32": ("decode.s", "_ZN2qk11k_root_scanIjLi1E", "profiles/r03/configs_pmc_sq.csv",
                          "k_root_scan<unsigned int, 1>", "524288", 1e8, 512,
                          "configs[4]: root test of 1e8 u32 candidates, d=32 (root-set scan, the default)"),
    "root_test_u32_d32": ("decode.s", "_ZN2qk15k_root_test_u32ILi32E", "profiles/r03/configs_pmc_sq.csv",
                          "k_root_test_u32<32>", "458752", 1e8, 256,
                          "configs[4]: root test of 1e8 u32 candidates, d=32 (Horner)"),
    "root_scan_u64_d32": ("decode.s", "_ZN2qk11k_root_scanImLi1E", "profiles/r03/configs_pmc_sq.csv",
                          "k_root_scan<unsigned long, 1>", "524288", 1e8, 256,
                          "root test of 1e8 u64 candidates, d=32 (root-set scan, the default)"),
    "root_test_u64_d32": ("decode.s", "_ZN2qk20k_root_test_u64_bsgsILi0E", "profiles/r03/configs_pmc_sq.csv",
                          "k_root_test_u64_bsgs<0>", "458752", 1e8, 128,
                          "root test of 1e8 u64 candidates, d=32 (baby-step/giant-step Horner)"),
}


def classify(line: str):
    """('v', cost) / ('s', 1) / None for one assembly line."""
    m = re.match(r"\s+([vs]_[a-z0-9_]+)\s*(.*?)(?:\s*;.*)?$", line)
    if not m:
        return None
    op, args = m.group(1), m.group(2)
    if op.startswith("s_"):
        if op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_endpgm", "s_setprio", "s_barrier")):
            return None
        return ("s", 1.0)
    ops = [a.strip() for a in re.split(r",(?![^\[]*\])", args) if a.strip()]
    heavy = False
    if re.search(r"cndmask|addc|subb|_co_|v_cmp|v_mad|v_mul_lo|v_mul_hi|3_|lshl_add|add_lshl|lshl_or|and_or|"
                 r"bfe|bfi|alignbit|perm|_u64|_i64|_b64", op):
        heavy = True
    if len(ops) >= 4:                                   # dst + 3 sources
        heavy = True
    if ops and re.match(r"(s\[|s\d|vcc)", ops[0]):     # SGPR / VCC result
        heavy = True
    return ("v", COST_HEAVY if heavy else COST_SIMPLE)


def loops(asm_lines, sym):
    start = next(i for i, l in enumerate(asm_lines) if re.match(r"^" + sym + r"\w*:", l))
    end = next(i for i in range(start, len(asm_lines)) if asm_lines[i].startswith(".Lfunc_end"))
    body = asm_lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\w+):", l))}
    out = []
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and labels.get(m.group(1), 1 << 30) < i:
            seg = body[labels[m.group(1)]:i + 1]
            cls = [c for c in (classify(x) for x in seg) if c]
            v = [c for k, c in cls if k == "v"]
            out.append({"label": m.group(1), "lo": labels[m.group(1)], "hi": i, "valu": len(v),
                        "valu_cost": sum(v), "salu": sum(1 for k, _ in cls if k == "s"),
                        "mix": collections.Counter(re.match(r"\s+(\S+)", x).group(1) for x in seg
                                                   if re.match(r"\s+v_", x))})
    return out


def pick_loop(ls, dyn_valu_per_iter):
    """The loop (or loop nest: outer + (k-1) x inner) whose VALU count per
    iteration matches the measured one."""
    best = None
    for o in ls:
        inner = [x for x in ls if o["lo"] < x["lo"] and x["hi"] < o["hi"] and x["valu"] > 8]
        cands = [(o["valu"], o["valu_cost"], o["label"], 1)]
        for x in inner:
            k = max(1, round((dyn_valu_per_iter - o["valu"]) / x["valu"]) + 1)
            cands.append((o["valu"] + (k - 1) * x["valu"], o["valu_cost"] + (k - 1) * x["valu_cost"],
                          f"{o['label']} + {k - 1} x {x['label']}", k))
        for n, cost, name, _ in cands:
            err = abs(n - dyn_valu_per_iter) / dyn_valu_per_iter
            if best is None or err < best[0]:
                best = (err, n, cost, name)
    return best


def pmc_row(path, kname, grid):
    """Counters and duration (ns) of the last profiled dispatch of kname at grid."""
    disp = collections.defaultdict(dict)
    with open(os.path.join(ROOT, path)) as f:
        for r in csv.DictReader(f):
            if kname in r["Kernel_Name"] and r["Grid_Size"] == grid:
                d = disp[r["Dispatch_Id"]]
                d[r["Counter_Name"]] = float(r["Counter_Value"])
                d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if not disp:
        raise KeyError(f"{kname} not in {path}")
    full = [d for d in disp.values() if "GRBM_GUI_ACTIVE" in d and "SQ_INSTS_VALU" in d]
    return full[-1]


def analyse(name, asm_dir):
    asm, sym, csvp, kname, grid, units, per_iter, label = KERNELS[name]
    lines = open(os.path.join(asm_dir, asm)).read().split("\n")
    c = pmc_row(csvp, kname, grid)
    valu_pu = c["SQ_INSTS_VALU"] / units
    salu_pu = c["SQ_INSTS_SALU"] / units
    err, n_static, cost_static, loop_name = pick_loop(loops(lines, sym), valu_pu * per_iter)
    mean_cost = cost_static / n_static
    cycles = c["GRBM_GUI_ACTIVE"] / 8
    clock = cycles / (c["_ns"] * 1e-9)
    achieved = cycles * SIMDS / units
    peak = valu_pu * mean_cost
    return {
        "config": label, "kernel": kname, "units_per_launch": units,
        "valu_insts_per_unit": round(valu_pu, 4), "salu_insts_per_unit": round(salu_pu, 4),
        "hot_loop": loop_name, "hot_loop_valu_per_iteration": n_static,
        "hot_loop_match_error": round(err, 4),
        "mean_issue_cycles_per_valu": round(mean_cost, 3),
        "clock_ghz": round(clock / 1e9, 3), "profiled_dispatch_ms": round(c["_ns"] * 1e-6, 4),
        "issue_cycles_per_unit_peak": round(peak, 3),
        "issue_cycles_per_unit_achieved": round(achieved, 3),
        "frac": round(peak / achieved, 4),
        "salu_busy": round(salu_pu * units / CUS / cycles, 4),
        "source": f"{csvp} (SQ_INSTS_VALU, SQ_INSTS_SALU, GRBM_GUI_ACTIVE); gfx950 assembly of {asm}",
    }


def recompute_bench(path):
    """The bench line's roofline.valu recomputed from the line's own fields
    (this run's kernel time and shader clock) and the algorithmic anchor of
    tools/issue_model.py — the anchor is fixed per t, so a kernel that issued
    more instructions would take longer and report a lower fraction."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import issue_model
    with open(path) as f:
        line = json.loads(next(l for l in f if l.startswith("{")))
    cfg, rf = line["config"], line["roofline"]
    got = issue_model.roofline(cfg["bits"], cfg["threshold"], cfg["ids_per_gpu"], rf["kernel_avg_ms"],
                               line["clock_ghz"])
    want = rf["valu"]
    return {"bench": os.path.relpath(path, ROOT), "anchor_cycles_per_id": got["peak"],
            "achieved_cycles_per_id": got["achieved"], "frac": got["frac"], "frac_on_line": want["frac"],
            "agree": abs(got["frac"] - want["frac"]) < 1e-9, "clock_ghz": line["clock_ghz"],
            "kernel_avg_ms": rf["kernel_avg_ms"], "ops_per_id": got["anchor"]["ops_per_id"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm-dir", default=os.path.join(ROOT, "sidekick_amd", "csrc", "_build", "asm"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03", "issue_roofline.json"))
    ap.add_argument("--bench", help="recompute a bench line's roofline.valu (tools/issue_model.py) and exit")
    a = ap.parse_args()
    if a.bench:
        json.dump(recompute_bench(a.bench), sys.stdout, indent=1)
        print()
        return
    res = {"method": __doc__.split("\n\n")[1], "costs": {"simple": COST_SIMPLE, "heavy": COST_HEAVY,
                                                         "source": "profiles/r01/ubench_issue.json"},
           "kernels": {k: analyse(k, a.asm_dir) for k in KERNELS}}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    json.dump(res["kernels"], sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
