"""Compact summary of a gpu_check.sh session in gpurun_out/ (dev helper)."""
import glob
import json
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
if os.path.exists(f"{out}/steps.log"):
    print("".join(l for l in open(f"{out}/steps.log") if " rc=" in l), end="")
for f in sorted(glob.glob(f"{out}/*.log")):
    name = os.path.basename(f)[:-4]
    lines = open(f, errors="replace").read().strip().splitlines()
    if not lines or name == "steps":
        continue
    last = lines[-1]
    try:
        d = json.loads(last)
        if "metric" in d:
            print(f"{name}: value={d['value']:.4g} kernel_ms={d['roofline']['kernel_avg_ms']:.4f} "
                  f"frac={d['roofline']['frac']:.4f} digest={d['result']['digest']}")
        else:
            print(f"{name}: {last[:300]}")
    except Exception:
        print(f"{name}: {last[:200]}")
