#!/usr/bin/env python3
"""Per-call kernel breakdown of flow batches from a rocprofv3 kernel trace
(tools/ab_flows.py under rocprofv3 --kernel-trace): calls are cut at each
k_flow_extract not directly after another (a table regrow); prints, per call, the wall
span from the first to the last flow kernel and each kernel's duration.

    python tools/flow_trace.py gpurun_out/profflows/run_kernel_trace.csv [--timeline]

--timeline: per call, also each stream's busy span and the main stream's
idle gaps (where it waits for the side stream or for launches)
"""
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "").replace("qk::", "").replace("rsort::", "")
    return n[:60]


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"]))
    rows.sort()
    flow_k = ("k_flow", "k_rs", "k_row_scan", "k_used", "k_slot", "k_key_rank", "k_rank", "k_hist", "k_seg",
              "k_list_big", "k_flow_finalize")
    calls, cur = [], None
    for s, e, n, st in rows:
        if n.startswith("k_flow_extract") and (cur is None or not cur[-1][2].startswith("k_flow_extract")):
            cur = []
            calls.append(cur)
        if cur is not None and n.startswith(flow_k):
            cur.append((s, e, n, st))
    for i, c in enumerate(calls):
        span = (max(e for _, e, _, _ in c) - c[0][0]) / 1e6
        print(f"call {i}: {len(c)} kernels, span {span:.3f} ms")
        agg = {}
        for s, e, n, st in c:
            a = agg.setdefault((n, st), [0, 0.0])
            a[0] += 1
            a[1] += (e - s) / 1e6
        for (n, st), (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"   {t:8.3f} ms  x{k:<3d} stream {st}  {n}")
        if "--timeline" in sys.argv:
            t0 = c[0][0]
            streams = sorted(set(st for _, _, _, st in c))
            for st in streams:
                ks = [(s, e, n) for s, e, n, x in c if x == st]
                print(f"   stream {st}: first start {(ks[0][0] - t0) / 1e6:.3f}, last end "
                      f"{(max(e for _, e, _ in ks) - t0) / 1e6:.3f} ms")
            main = [(s, e, n) for s, e, n, x in c if x == c[0][3]]
            for (s1, e1, n1), (s2, e2, n2) in zip(main, main[1:]):
                if s2 - e1 > 20_000:   # > 20 us idle
                    print(f"   main idle {(s2 - e1) / 1e6:.3f} ms at {(e1 - t0) / 1e6:.3f} before {n2}")


if __name__ == "__main__":
    main()
