#!/usr/bin/env python3
"""Secondary measurements for DESIGN.md (not the driver's bench line):

  u64      configs[2]: encode 1e9 u64 ids at t=80, device-resident
  decode   configs[4]: subtract two quACKs built from 1e8 u32 ids, 32 missing,
           root test over the 1e8-entry candidate log (device-resident)
  host     encode 1e9 u32 ids at t=32 starting from HOST memory (pinned and
           pageable): the PCIe-inclusive rate the sniffer-fed path sees
  sweep    encode rate vs threshold t (u32)
  packets  sniff-loop batch: 67-byte records in HBM -> one quACK
  flows    per-flow batch: records of 16 / 1e4 / 1e6 flows -> one quACK each
  micro    reference-shape rows (1000 ids x 100 trials) and configs[0]

Each prints one JSON line per measurement.  Kernel times come from HIP events
on the launch stream (qk_ctx_set_profiling); wall times from perf_counter
around synchronised loops.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sidekick_amd as sk  # noqa: E402
from sidekick_amd.quack import encode_device_async, fill_splitmix, partial_words  # noqa: E402

DEV = "cuda:0"


def emit(d):
    print(json.dumps(d), flush=True)


def time_encode(ctx, ids, t, bits, steps, warmup=2):
    part = torch.zeros(partial_words(t, bits), dtype=torch.int64, device=DEV)
    for _ in range(warmup):
        encode_device_async(ctx, ids, t, part, bits=bits)
    torch.cuda.synchronize()
    ctx.kernel_stats()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        encode_device_async(ctx, ids, t, part, bits=bits)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ctx.set_profiling(False)
    ms, n = ctx.kernel_stats()
    # kernel time per step: a multi-pass encode (u32 t > 80) launches one
    # profiled kernel per pass
    return wall / steps, ms / steps / 1e3


def run_u64(args, ctx):
    n, t = int(args.n64), 80
    ids = torch.empty(n, dtype=torch.int64, device=DEV)
    fill_splitmix(ctx, ids, 0x5EED0003, bits=64)
    wall, kern = time_encode(ctx, ids, t, 64, args.steps)
    emit({"config": "encode u64 t=80 device-resident", "n": n, "ids_per_s": n / wall, "kernel_s": kern,
          "hbm_GBps_algorithmic": 8 * n / kern / 1e9, "frac_hbm_8TBs": 8 * n / kern / 8e12})
    if args.cpu:
        from oracle import coracle
        m = int(args.cpu_sample64)
        tc = time.perf_counter()
        S = coracle.encode_u64_seed(0x5EED0003, m, t)
        cs = time.perf_counter() - tc
        q = sk.PowerSumQuackU64(t)
        q.insert_batch(ids[:m])
        emit({"config": "cpu baseline u64 t=80 (oracle C, 1 core)", "n": m, "ids_per_s": m / cs,
              "parity_with_gpu": q.power_sums() == S})


def run_decode(args, ctx, bits=32):
    n, t, seed = int(args.ndec), 32, 0x5EED0005 + (bits == 64)
    log = torch.empty(n, dtype=torch.int32 if bits == 32 else torch.int64, device=DEV)
    fill_splitmix(ctx, log, seed, bits=bits)
    cls = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    rng = np.random.default_rng(seed)
    drops = np.sort(rng.choice(n, size=32, replace=False))
    keep = torch.ones(n, dtype=torch.bool, device=DEV)
    keep[torch.from_numpy(drops).to(DEV)] = False
    kept = log[keep].contiguous()
    torch.cuda.synchronize()
    # host root finding alone (the root-set scan's host step, roots.cpp)
    sent, recv = cls(t), cls(t)
    sent.insert_batch(log)
    recv.insert_batch(kept)
    diff = sent.clone()
    diff.sub_assign(recv)
    c = diff.to_coeffs()
    rt = []
    for _ in range(max(5, args.steps)):
        t0 = time.perf_counter()
        r = sk.roots(c, bits)
        rt.append(time.perf_counter() - t0)
    emit({"config": f"host root finding u{bits} d={len(c)} (roots.cpp)", "roots": len(r),
          "median_s": float(np.median(rt)), "min_s": min(rt)})
    # the timed decode step: encode both sides, subtract, to_coeffs, root test
    # (mode 1: Horner per candidate; 2: host roots + root-set scan; 0: automatic)
    results = {}
    for mode in args.rt_modes:
        ctx.set_knob("root_test", mode)
        reps = []
        for r in range(args.steps + 1):
            t0 = time.perf_counter()
            sent, recv = cls(t), cls(t)
            sent.insert_batch(log)
            recv.insert_batch(kept)
            diff = sent.clone()
            diff.sub_assign(recv)
            t1 = time.perf_counter()
            c = diff.to_coeffs()
            t2 = time.perf_counter()
            ctx.set_profiling(True)
            hits = diff.root_test(c, log)
            ctx.set_profiling(False)
            t3 = time.perf_counter()
            ms, k = ctx.kernel_stats()
            if r:
                reps.append((t1 - t0, t2 - t1, t3 - t2, ms / 1e3))
        ctx.set_knob("root_test", 0)
        results[mode] = hits
        a = np.median(np.array(reps), axis=0)
        ok = set(drops.tolist()) <= set(hits)
        b = bits // 8
        name = {0: "auto", 1: "horner", 2: "root-set scan"}[mode]
        emit({"config": f"decode-missing u{bits} n=1e8 d=32" + (" (configs[4])" if bits == 32 else "")
                        + f", root test: {name}", "n": n,
              "hits": len(hits), "drops_recovered": ok, "same_hits_as_first_mode": hits == results[args.rt_modes[0]],
              "encode_both_s": a[0], "to_coeffs_s": a[1], "root_test_wall_s": a[2], "root_test_kernel_s": a[3],
              "root_test_candidates_per_s": n / a[3], "root_test_GBps": b * n / a[3] / 1e9,
              "frac_hbm_8TBs": b * n / a[3] / 8e12, "total_s": a[0] + a[1] + a[2]})
    if args.cpu:
        from oracle import coracle
        m = int(args.cpu_sample_dec)
        h = log[:m].cpu().numpy().view(np.uint32 if bits == 32 else np.uint64)
        tc = time.perf_counter()
        if bits == 32:
            w, nh = coracle.root_test_u32(list(c), h)
        else:
            w, nh = coracle.root_test_u64(list(c), h)
        cs = time.perf_counter() - tc
        emit({"config": f"cpu baseline root test u{bits} d=32 (oracle C, 1 core)", "n": m,
              "candidates_per_s": m / cs, "extrapolated_1e8_s": cs * n / m,
              "hits_match_gpu_prefix": w.tolist() == [x for x in hits if x < m]})


def run_decode64(args, ctx):
    run_decode(args, ctx, bits=64)


def run_host(args, ctx):
    n, t = int(args.nhost), 32
    d = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, d, 0x5EED0002)
    pinned = torch.empty(n, dtype=torch.int32, pin_memory=True)
    pinned.copy_(d)
    pageable = d.cpu().numpy()
    ref = sk.PowerSumQuackU32(t)
    ref.insert_batch(d)
    for name, arr in (("pinned", pinned.numpy()), ("pageable", pageable)):
        times = []
        for r in range(3):
            q = sk.PowerSumQuackU32(t)
            t0 = time.perf_counter()
            q.insert_batch(arr.view(np.uint32))
            times.append(time.perf_counter() - t0)
        assert q == ref
        tm = min(times)
        emit({"config": f"encode u32 t=32 from {name} host memory (H2D + kernel, pipelined)", "n": n,
              "ids_per_s": n / tm, "GBps_h2d_equiv": 4 * n / tm / 1e9, "seconds": tm})
    # raw H2D copy rate for reference
    tmp = torch.empty(n, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tmp.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    emit({"config": "raw H2D copy, pinned (torch)", "GBps": 4 * n / (time.perf_counter() - t0) / 1e9})


def run_packets(args, ctx):
    """Sniff-loop batch: n 67-byte captured records in HBM -> quACK (t=32)."""
    from sidekick_amd.quack import encode_packets
    n, stride = int(args.npkts), 67
    raw = torch.empty(n * stride, dtype=torch.uint8, device=DEV)
    # synthetic records: random bytes, UDP at byte 23, foreign dst ip, no resets
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    raw.random_(0, 256, generator=g)
    rec = raw.view(n, stride)
    rec[:, 23] = 17
    rec[:, 30] = 192
    for t in [int(x) for x in args.pkt_t.split(",")]:
        q = sk.PowerSumQuackU32(t)
        encode_packets(q, raw, stride=stride, my_ipv4=(10, 0, 2, 1))   # warm
        torch.cuda.synchronize()
        times = []
        for _ in range(args.steps):
            q = sk.PowerSumQuackU32(t)
            t0 = time.perf_counter()
            st = encode_packets(q, raw, stride=stride, my_ipv4=(10, 0, 2, 1))
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        tm = float(np.median(times))
        emit({"config": f"sniff-loop batch: 67-byte records in HBM -> extract + encode u32 t={t}", "n_packets": n,
              "packets_per_s": n / tm, "record_GBps": n * stride / tm / 1e9, "frac_hbm_8TBs": n * stride / tm / 8e12,
              "inserted": st["inserted"], "seconds": tm})


def run_flows(args, ctx):
    """SidekickMulti batch (sidekick_multi.rs:101-143): n 67-byte records of F
    flows in HBM -> one quACK per AddrKey (extract, radix-sort grouping,
    segmented encode, keys + sketches copied to the host)."""
    import ctypes as C
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import FlowKey, PktStats
    n, stride, t = int(args.npkts), 67, 32
    raw = torch.empty(n * stride, dtype=torch.uint8, device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    raw.random_(0, 256, generator=g)
    rec = raw.view(n, stride)
    rec[:, 23] = 17
    for nflows in (16, 10_000, 1_000_000):
        f = torch.randint(0, nflows, (n,), device=DEV, generator=g, dtype=torch.int64)
        for k in range(4):                       # src ip = flow id (LE bytes), fixed ports / dst
            rec[:, 26 + k] = ((f >> (8 * k)) & 255).to(torch.uint8)
        rec[:, 30:38] = torch.tensor([192, 168, 0, 9, 0x11, 0x5C, 0x1F, 0x90], dtype=torch.uint8, device=DEV)
        cap = nflows
        rsz = lib().qk_u32_size(t)
        outs = {"host output (pageable)": ((FlowKey * cap)(), C.create_string_buffer(cap * rsz)),
                "device-resident output": (torch.empty((cap, 12), dtype=torch.uint8, device=DEV),
                                           torch.empty((cap, rsz // 4), dtype=torch.int32, device=DEV))}
        for where, (keys, sk_buf) in outs.items():
            kp = keys.data_ptr() if isinstance(keys, torch.Tensor) else keys
            sp = sk_buf.data_ptr() if isinstance(sk_buf, torch.Tensor) else sk_buf
            times = []
            for it in range(max(3, args.steps // 2) + 1):
                nf, st = C.c_size_t(), PktStats()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = lib().qk_u32_encode_flows_device(ctx.handle, raw.data_ptr(), n, stride, None, None, t, kp, sp,
                                                      cap, C.byref(nf), C.byref(st), 0)
                torch.cuda.synchronize()
                if rc != 0:
                    raise RuntimeError(f"encode_flows rc={rc}")
                if it:
                    times.append(time.perf_counter() - t0)
            tm = float(np.median(times))
            emit({"config": f"per-flow batch: {n} records of {nflows} flows -> one quACK per AddrKey, t={t}, {where}",
                  "n_packets": n, "flows": int(nf.value), "packets_per_s": n / tm,
                  "record_GBps": n * stride / tm / 1e9, "seconds": tm, "inserted": int(st.inserted)})
        del f


# published quack-crate encode ns/id, 1000 ids per trial, 1 Xeon core
# (zip:nsdi24/quack/threshold_vs_encode_time/{32,64}.txt)
PUBLISHED_NS = {(32, 10): 34, (32, 20): 75, (32, 30): 117, (32, 40): 161, (32, 80): 327,
                (64, 30): 167, (64, 40): 227, (64, 80): 461}


def run_micro(args, ctx):
    """Reference-shape rows: 1000 ids x 100 trials per
    threshold, CPU restatement beside the published crate numbers and the GPU
    doing the same tiny job (launch-latency bound at this size), then
    configs[0] (1e6 u32 ids, t=16) on both."""
    from oracle import coracle
    n, trials = 1000, 100
    rows = [(32, t) for t in (10, 16, 20, 30, 32, 40, 80)] + [(64, t) for t in (30, 40, 80)]
    for bits, t in rows:
        seed = 0xB0 + t + bits
        cpu_ns = coracle.bench_construct(bits, seed, n, t, trials)
        dt = torch.int32 if bits == 32 else torch.int64
        ids = torch.empty(n * trials, dtype=dt, device=DEV)
        fill_splitmix(ctx, ids, seed, bits=bits)
        cls = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
        q = cls(t)
        q.insert_batch(ids[:n])                          # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(trials):
            q = cls(t)
            q.insert_batch(ids[r * n:(r + 1) * n])        # returns after the sketch is on the host
        gpu_ns = (time.perf_counter() - t0) / (n * trials) * 1e9
        last = ids[(trials - 1) * n:].cpu().numpy()
        want = (coracle.encode_u32(last.view(np.uint32), t) if bits == 32
                else coracle.encode_u64(last.view(np.uint64), t))
        emit({"config": f"reference-shape construct u{bits} t={t}: {n} ids x {trials} trials",
              "published_crate_ns_per_id": PUBLISHED_NS.get((bits, t)), "cpu_port_ns_per_id": round(cpu_ns, 2),
              "gpu_ns_per_id": round(gpu_ns, 2), "parity": q.power_sums() == want})
    # configs[0]: 1e6 u32 ids, t = 16
    m, t, seed = 1_000_000, 16, 0x5EED0001
    d = torch.empty(m, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, d, seed)
    wall, kern = time_encode(ctx, d, t, 32, max(10, args.steps))
    h = d.cpu().numpy().view(np.uint32)
    times = []
    for _ in range(5):
        q = sk.PowerSumQuackU32(t)
        t0 = time.perf_counter()
        q.insert_batch(h)
        times.append(time.perf_counter() - t0)
    tc = time.perf_counter()
    S = coracle.encode_u32_seed(seed, m, t)
    cs = time.perf_counter() - tc
    emit({"config": "configs[0]: encode 1e6 u32 ids t=16", "n": m, "gpu_device_resident_ids_per_s": m / wall,
          "gpu_kernel_ids_per_s": m / kern, "gpu_from_pageable_host_ids_per_s": m / min(times),
          "cpu_port_1core_ids_per_s": m / cs, "parity": q.power_sums() == S})


def sweep_ts(args, default):
    return tuple(int(x) for x in args.sweep_t.split(",")) if args.sweep_t else default


def run_sweep(args, ctx):
    n = int(args.nsweep)
    ids = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, ids, 0x5EED0002)
    for t in sweep_ts(args, (1, 4, 8, 10, 16, 17, 20, 24, 25, 28, 30, 32, 33, 36, 40, 42, 48, 50, 56, 60, 64, 70, 72, 80,
                             96, 128, 176, 256, 300, 512, 1024)):
        wall, kern = time_encode(ctx, ids, t, 32, max(3, args.steps // 2))
        emit({"config": f"encode u32 t={t}", "n": n, "ids_per_s": n / kern, "ns_per_id_per_power": kern / n / t * 1e9 * 1})


def run_sweep64(args, ctx):
    n = int(args.nsweep)
    ids = torch.empty(n, dtype=torch.int64, device=DEV)
    fill_splitmix(ctx, ids, 0x5EED0003, bits=64)
    path = "default"
    for t in sweep_ts(args, (8, 9, 12, 16, 17, 20, 24, 32, 40, 48, 56, 64, 72, 80, 81, 128, 160, 256, 512, 1024)):
        wall, kern = time_encode(ctx, ids, t, 64, max(3, args.steps // 2))
        emit({"config": f"encode u64 t={t} ({path})", "n": n, "ids_per_s": n / kern,
              "ns_per_id_per_power": kern / n / t * 1e9})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pkt-t", default="32", help="packets: thresholds (comma list)")
    ap.add_argument("what", nargs="+", choices=["u64", "decode", "decode64", "host", "sweep", "sweep64", "packets", "flows", "micro"])
    ap.add_argument("--npkts", type=float, default=1e8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n64", type=float, default=1e9)
    ap.add_argument("--ndec", type=float, default=1e8)
    ap.add_argument("--nhost", type=float, default=1e9)
    ap.add_argument("--nsweep", type=float, default=2.5e8)
    ap.add_argument("--sweep-t", default="", help="sweep / sweep64: thresholds (comma list) instead of the default set")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--cpu-sample64", type=float, default=5e6)
    ap.add_argument("--cpu-sample-dec", type=float, default=2e7)
    ap.add_argument("--rt-modes", default="1,2", help="decode: root-test modes to time (0 auto, 1 Horner, 2 scan)")
    ap.add_argument("--knob", action="append", default=[],
                    help="NAME=VALUE measurement knob (qk_ctx_set_knob; grid=N: qk_ctx_set_grid)")
    args = ap.parse_args()
    args.rt_modes = [int(x) for x in args.rt_modes.split(",")]
    ctx = sk.get_context(0)
    for kv in args.knob:
        k, v = kv.split("=")
        if k == "grid":   # workgroups per launch for every kernel (qk_ctx_set_grid), measurements
            ctx.set_grid(int(v))
        else:
            ctx.set_knob(k, int(v))
    for w in args.what:
        {"u64": run_u64, "decode": run_decode, "decode64": run_decode64, "host": run_host, "sweep": run_sweep, "sweep64": run_sweep64,
         "packets": run_packets, "flows": run_flows, "micro": run_micro}[w](args, ctx)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
