#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the last one in a log)."""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print(f"value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.3f}  kernel {r['kernel_avg_ms']:.3f} ms  "
      f"hbm frac {r['frac']:.3f}  valu frac {(r.get('valu') or {}).get('frac')}  clock {d.get('clock_ghz')}  "
      f"digest ok {d['result'].get('equals_recorded')}")
for k, v in (d.get("configs") or {}).items():
    keep = {a: b for a, b in v.items() if a not in ("workload", "valu")}
    if "valu" in v and v["valu"]:
        keep["valu_frac"] = v["valu"]["frac"]
    print(k, json.dumps(keep))
cb = d.get("cpu_baseline") or {}
print("cpu_baseline", {a: cb.get(a) for a in ("value", "ns_per_id", "tsc_cycles_per_id", "core_cycles_per_id",
                                              "parity_with_gpu")})
