#!/usr/bin/env python3
"""Benchmark: device-resident quACK encode throughput (identifiers/s).

Metric (BASELINE.json): "quACK encode identifiers/s (device-resident), u32
ids, threshold t=32".  Workload at N=1 is configs[1]: encode 1e9 u32 ids at
t=32 on one MI355X, ids already resident in HBM.  One step = one pass of the
encode path over the GPU's batch: the encode kernel + finalize kernel, and,
for N > 1, the single RCCL sum-reduce of the partial power-sum vectors to
rank 0 (weak scaling: every GPU owns a fixed 1e9-id shard of one global
stream).  For N > 1 the data path is the library's native communicator
(qk_u32_encode_sharded_async: encode + ONE ncclReduce over xGMI, comm.hip);
torch.distributed (gloo) only carries the control plane — the RCCL unique
id, the barriers around the timed region and the max-over-ranks time.  On a
node with fewer GPUs than ranks (a one-GPU rehearsal: RCCL refuses two ranks
on one device) the same native protocol runs with its collectives over gloo
(qk_comm_init_host), and the line says so; with enough GPUs a communicator
that cannot be built is an error, never a silent fallback.

    python bench.py [--gpus N --steps K --warmup W --n IDS_PER_GPU --t 32 --bits 32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  Alongside the metric it reports
  roofline      the encode kernel's achieved algorithmic HBM bytes/s (4 B per
                u32 id) over its average launch duration, measured with HIP
                events on the launch stream, against the 8 TB/s HBM3E peak;
                and `valu`, the integer-issue roofline that actually binds
                (tools/issue_model.py: the decomposition's VALU work per id
                at the measured issue costs, against the SIMD cycles the
                launch spent per id at this run's shader clock, read by
                qk_clock_probe beside the running kernel after the timed
                region);
  parity        N > 1: after the timed region, the N = 1 stream cut into N
                shards and encoded through the same communicator; its digest
                against rank 0's single-GPU encode and the recorded N = 1
                digest; `rccl` / `ranks`: what RCCL reports on every rank
                (ncclCommCount, ncclCommCuDevice, ncclCommUserRank);
  decode_parity N > 1: configs[4]'s decode through the same communicator
                (two sharded encodes, the difference, decode_sharded's
                broadcast and all-gathers) against rank 0's single-GPU root
                test: equal hit lists, every drop recovered;
  configs       N = 1, untimed, after the headline: configs[2] (u64 t=80),
                configs[4] (decode-missing, and its u64 twin) and SURVEY §8f's
                flow and packet batches, each with its kernel / wall times,
                roofline fractions and an independent check of its result
                (secondary_configs; --configs 0 skips it);
  cpu_baseline  the oracle's scalar C restatement of the reference insert
                loop on ONE host core over a bounded prefix of the same
                stream (rank 0, N = 1 only), timed in the crate's own unit
                (rdtsc around the loop) and in ns, with a GPU/CPU parity
                check on that prefix.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_traffic(bits: int, t: int, n: int):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (FETCH_SIZE
    corrected x2 per MI355X_MICROARCH.md §HBM), scaled to n ids."""
    path = os.path.join(ROOT, "profiles", "pmc_encode.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d["encode"][f"u{bits}_t{t}"]
        return e["hbm_read_bytes_corrected"] / e["n_ids"] * n, os.path.relpath(path, ROOT)
    except Exception:
        return None, None


def valu_roofline(bits: int, t: int, n: int, kern_avg_ms: float, clock_ghz):
    """The integer-issue roofline (tools/issue_model.py): the decomposition's
    VALU work per id at the measured per-class issue costs — fixed per t, so
    instruction bloat lowers the fraction — against the SIMD-cycles per id of
    THIS run's kernel time at THIS run's shader clock (measure_clock)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import issue_model
    return issue_model.roofline(bits, t, n, kern_avg_ms, clock_ghz)


def measure_clock(ctx, step, dev_index, kern_avg_ms, steps=10):
    """The shader clock the chip holds under this kernel, in this run: after
    the timed region, qk_clock_probe's one wave spins on a side stream for
    ~90 % of `steps` further (untimed) steps and reads s_memtime against
    s_memrealtime (100 MHz).  Returns GHz or None.  For N > 1 every step is a
    collective, so every rank runs all of them whatever happens to its probe
    (a probe failure only nulls the clock); a failing step raises."""
    import torch
    out = torch.zeros(2, dtype=torch.int64, device=f"cuda:{dev_index}")
    side = torch.cuda.Stream(device=dev_index)
    for _ in range(2):
        step()                                       # the chip busy before the probe lands
    probe_ok = True
    try:
        us = max(1000, int(kern_avg_ms * steps * 0.9 * 1e3))
        ctx.clock_probe_async(us, out, side.cuda_stream)
    except Exception as e:  # noqa: BLE001 — a measurement aid, never fatal
        log(f"clock probe failed: {e!r}")
        probe_ok = False
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if not probe_ok:
        return None
    c, r = (int(v) for v in out.cpu().tolist())
    return c / r * 0.1 if r > 0 else None


# Digests of the folded power sums of the global stream (u32 ids, t = 32,
# seed 0x5EED0002): N = 1 (configs[1], 1e9 ids) unchanged since round 1
# (BENCH_r01..r04); N = 2, 4, 8 (2e9 / 4e9 / 8e9 ids, configs[3] at N = 8)
# recorded by tests/test_gpu_comm.py::test_configs3_full_size_world8_host_channel
# (whole-stream single-GPU encodes, equal to the world-8 sharded encode;
# profiles/r05/check1/pytest.txt), so the driver's scaling runs check their
# result too.
RECORDED_DIGESTS = {(32, 32, 1_000_000_000, 0x5EED0002): "523499db79543cdf",
                    (32, 32, 2_000_000_000, 0x5EED0002): "bb61bb32e92b9799",
                    (32, 32, 4_000_000_000, 0x5EED0002): "37d66ecb59b3a758",
                    (32, 32, 8_000_000_000, 0x5EED0002): "032bc2155ec17f4a"}


def digest_of(S, count) -> str:
    import hashlib
    return hashlib.sha256((",".join(str(v) for v in S) + f"|{count}").encode()).hexdigest()[:16]


def strong_scaling_check(args, comm, ctx, ids, rank, world, dev_index, bits, t):
    """N > 1, untimed: the N = 1 stream (--ids-per-gpu ids, the same seed) cut
    into `world` contiguous shards, each filled on its own GPU and encoded
    through the same communicator (one reduce to rank 0); rank 0 then encodes
    the whole stream alone on its GPU.  Returns (on rank 0) the sharded digest,
    the single-GPU digest and the recorded N = 1 digest."""
    import torch
    import sidekick_amd as sk
    from sidekick_amd import dist as skd
    from sidekick_amd.quack import fill_splitmix
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    n1 = int(args.ids_per_gpu)
    s, c = skd.shard(n1, rank, world)
    view = ids[:c]
    fill_splitmix(ctx, view, args.seed, s, bits=bits)
    torch.cuda.synchronize()
    q = Q(t)
    comm.encode_sharded([view], q)
    if rank != 0:
        return None
    sharded = digest_of(q.power_sums(), q.count())
    fill_splitmix(ctx, ids[:n1], args.seed, 0, bits=bits)
    q1 = Q(t)
    q1.insert_batch(ids[:n1], ctx=ctx)
    single = digest_of(q1.power_sums(), q1.count())
    rec = RECORDED_DIGESTS.get((bits, t, n1, args.seed))
    return {"workload": f"strong scaling, untimed: the N=1 stream ({n1:.0e} u{bits} ids, seed {hex(args.seed)}) in "
                        f"{world} contiguous shards, one per rank, encoded through the same communicator",
            "digest": sharded, "digest_single_gpu": single, "equals_n1": sharded == single,
            "recorded_n1_digest": rec, "equals_recorded": (sharded == rec) if rec else None,
            "last_value_equal": q.last_value() == q1.last_value()}


# configs[4]: decode-missing over a 1e8-id candidate log with 32 drops
DECODE_SEED, DECODE_N, DECODE_DROPS, DECODE_T = 0x5EED0005, 100_000_000, 32, 32


def decode_check(comm, ctx, ids, n_per_gpu, rank, world, bits):
    """N > 1, untimed: configs[4]'s decode through the same communicator.  The
    1e8-id log (seed 0x5EED0005) is cut into `world` contiguous shards, one
    per rank, filled on its own GPU; 32 seeded drops (the same on every rank)
    are removed from the receiver's copy of each shard.  quack_A = the sharded
    encode of the log, quack_B = the sharded encode of the log without the
    drops (one reduce each), diff = A - B on the root, then decode_sharded
    (ncclBroadcast of the coefficients, every rank root-tests its shard, two
    all-gathers).  Rank 0 then fills the whole log on its own GPU and runs
    the single-GPU root test with the same difference; the two hit lists
    must be equal and contain every drop.  Returns the record on rank 0."""
    import numpy as np
    import torch
    import sidekick_amd as sk
    from sidekick_amd import dist as skd
    from sidekick_amd.quack import fill_splitmix
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    n_log = min(DECODE_N, n_per_gpu)           # alike on every rank; rank 0's id buffer then holds the whole log
    drops = np.sort(np.random.default_rng(DECODE_SEED).choice(n_log, DECODE_DROPS, replace=False))
    s, c = skd.shard(n_log, rank, world)
    log_view = ids[:c]
    fill_splitmix(ctx, log_view, DECODE_SEED, s, bits=bits)
    keep = torch.ones(c, dtype=torch.bool, device=ids.device)
    mine = drops[(drops >= s) & (drops < s + c)] - s
    if len(mine):
        keep[torch.from_numpy(mine).to(ids.device)] = False
    recv_view = log_view[keep]
    torch.cuda.synchronize()
    A, B = Q(DECODE_T), Q(DECODE_T)
    comm.encode_sharded([log_view], A)
    comm.encode_sharded([recv_view], B)
    diff = None
    if rank == 0:
        diff = A.clone()
        diff.sub_assign(B)
    t0 = time.perf_counter()
    hits = comm.decode_sharded(diff, [log_view], bits=bits, stop_at_last=True)
    dec_ms = (time.perf_counter() - t0) * 1e3
    del recv_view, keep
    if rank != 0:
        return None
    fill_splitmix(ctx, ids[:n_log], DECODE_SEED, 0, bits=bits)
    want = diff.root_test(diff.to_coeffs(), ids[:n_log], stop_value=diff.last_value())
    torch.cuda.synchronize()
    return {"workload": f"configs[4], untimed: decode-missing over a {n_log:.0e}-id u{bits} log (seed "
                        f"{hex(DECODE_SEED)}) in {world} contiguous shards with {DECODE_DROPS} seeded drops: two "
                        f"sharded encodes (A = log, B = log without the drops), diff = A - B on rank 0, "
                        f"decode_sharded (broadcast + all-gathers) against rank 0's single-GPU root test",
            "d": diff.count(), "hits": len(hits), "equals_single_gpu": hits == want,
            "drops_recovered": bool(set(drops.tolist()) <= set(hits)), "decode_sharded_ms": dec_ms}


# ---------------------------------------------------------------------------
# N = 1, untimed, after the headline: every other single-GPU config of
# BASELINE.json (and SURVEY §8f's two batch paths) measured and checked in the
# same run, so the driver's record carries them (reported under "configs").
# Kernel times come from HIP events on the launch stream (qk_ctx profiling);
# wall times from perf_counter around synchronised calls; each block checks
# its own result independently of the kernel it times.
# ---------------------------------------------------------------------------
# configs[2]: digest of the folded power sums of 1e9 u64 ids (seed
# 0x5EED0003) at t = 80, recorded by this block's first run (BENCH line of
# profiles/r06/), equal across every u64 kernel change since.
RECORDED_U64_DIGEST = {(64, 80, 1_000_000_000, 0x5EED0003): "9d86f76bad8351be"}


def cfg_u64(ctx, dev_index, steps=10):
    """configs[2]: encode 1e9 u64 ids at t = 80, device-resident: kernel ms,
    ids/s, algorithmic HBM fraction, the issue-anchor fraction on the same
    method as the headline's roofline.valu, the digest against the recorded
    one, and the first 1e6 ids against the oracle's scalar C encode of the
    same stream generated on the host."""
    import numpy as np
    import torch
    import sidekick_amd as sk
    from oracle import coracle
    from sidekick_amd import dist as skd
    from sidekick_amd.quack import encode_device_async, fill_splitmix, partial_words
    n, t, seed, m = 1_000_000_000, 80, 0x5EED0003, 1_000_000
    dev = f"cuda:{dev_index}"
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    fill_splitmix(ctx, ids, seed, bits=64)
    part = torch.zeros(partial_words(t, 64), dtype=torch.int64, device=dev)

    def step():
        encode_device_async(ctx, ids, t, part, bits=64)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    ctx.kernel_stats()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ctx.set_profiling(False)
    kms, launches = ctx.kernel_stats()
    kern = kms / max(launches, 1)
    S, count = skd.fold_partial_sum(part.cpu().numpy().view(np.uint64), t, 64)
    digest = digest_of(S, count)
    clock = measure_clock(ctx, step, dev_index, kern)
    torch.cuda.synchronize()
    q = sk.PowerSumQuackU64(t)
    q.insert_batch(ids[:m], ctx=ctx)
    want = coracle.encode_u64(coracle.splitmix_u64(seed, m), t)
    rec = RECORDED_U64_DIGEST.get((64, t, n, seed))
    del ids
    return {"workload": f"configs[2]: encode {n:.0e} u64 ids at t={t}, device-resident (seed {hex(seed)})",
            "kernel_ms": kern, "launches": launches, "ms_per_step": wall * 1e3, "ids_per_s": n / wall,
            "hbm_frac": 8 * n / (kern * 1e-3) / (HBM_PEAK_GBS * 1e9),
            "valu": valu_roofline(64, t, n, kern, clock), "clock_ghz": clock,
            "digest": digest, "recorded_digest": rec, "equals_recorded": (digest == rec) if rec else None,
            "oracle_prefix": {"ids": m, "equal": q.power_sums() == want}}


def cfg_decode(ctx, dev_index, bits=32, reps=200, warm=8):
    """configs[4] (u32; its u64 twin with bits = 64): a 1e8-id candidate log,
    32 seeded drops; quack_A = encode(log), quack_B = encode(log without the
    drops), diff = A - B; the timed call is qk_u*_decode_device(diff, log,
    stop_at_last) — to_coeffs, the host root finding, the root-set scan and
    the hand-back — by perf_counter around the C call, the scan kernel by HIP
    events.  Check: the hits equal the positions whose id is one of the
    dropped ids (torch.isin on the device, no polynomial involved)."""
    import ctypes as C
    import numpy as np
    import torch
    import sidekick_amd as sk
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import fill_splitmix
    n, t = DECODE_N, DECODE_T
    seed = DECODE_SEED + (bits == 64)
    dev = f"cuda:{dev_index}"
    log_ = torch.empty(n, dtype=torch.int32 if bits == 32 else torch.int64, device=dev)
    fill_splitmix(ctx, log_, seed, bits=bits)
    drops = np.sort(np.random.default_rng(seed).choice(n, DECODE_DROPS, replace=False))
    d_drops = torch.from_numpy(drops).to(dev)
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    keep[d_drops] = False
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    A, B = Q(t), Q(t)
    A.insert_batch(log_, ctx=ctx)
    B.insert_batch(log_[keep].contiguous(), ctx=ctx)
    diff = A.clone()
    diff.sub_assign(B)
    expected = torch.isin(log_, log_[d_drops]).nonzero().flatten().cpu().tolist()
    del keep
    torch.cuda.synchronize()
    fn = getattr(lib(), f"qk_u{bits}_decode_device")
    cap = 1 << 12
    hits = (C.c_uint64 * cap)()
    nh = C.c_size_t()
    walls, kerns, ok = [], [], True
    # the call's arguments built once (the C caller's view: the timed region
    # is the call, not the Python marshalling of its arguments)
    args = (ctx.handle, diff._buf, C.c_void_p(log_.data_ptr()), C.c_size_t(n), C.c_int(1), hits, C.c_size_t(cap),
            C.byref(nh), None)
    # wall times without the profiling events (two event records per call);
    # the scan kernel's time from separate profiled calls
    for prof in (False, True):
        for r in range(reps + warm):
            if prof:
                ctx.kernel_stats()
                ctx.set_profiling(True)
            t0 = time.perf_counter()
            rc = fn(*args)
            wall = time.perf_counter() - t0
            got = [int(h) for h in hits[:nh.value]] if rc == 0 else None
            ok = ok and got == expected
            if prof:
                ctx.set_profiling(False)
                kms, k = ctx.kernel_stats()
                if r >= warm:
                    kerns.append(kms * 1e3 / max(k, 1))
            elif r >= warm:
                walls.append(wall * 1e6)
    b = bits // 8
    scan = float(np.median(kerns))
    del log_
    return {"workload": f"configs[4]{'' if bits == 32 else ' (u64 twin)'}: decode-missing over a {n:.0e}-id u{bits} "
                        f"log (seed {hex(seed)}), {DECODE_DROPS} drops, t={t}: qk_u{bits}_decode_device with "
                        f"stop_at_last (to_coeffs + host roots + root-set scan + hand-back)",
            "wall_us_median": float(np.median(walls)), "wall_us_min": float(np.min(walls)),
            "scan_kernel_us_median": scan, "scan_hbm_frac": b * n / (scan * 1e-6) / (HBM_PEAK_GBS * 1e9),
            "d": diff.count(), "hits": len(expected), "hits_equal_expected": ok,
            "drops_recovered": bool(set(drops.tolist()) <= set(expected)) and ok, "reps": reps}


def make_records(dev, n, seed, stride=67):
    """n synthetic 67-byte captured records in HBM: random bytes, UDP, a
    foreign destination (192.168.0.9:8080, src port 0x115C), id at byte 63."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    raw = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    raw.random_(0, 256, generator=g)
    rec = raw.view(n, stride)
    rec[:, 23] = 17
    rec[:, 30:38] = torch.tensor([192, 168, 0, 9, 0x11, 0x5C, 0x1F, 0x90], dtype=torch.uint8, device=dev)
    return raw, rec, g


def record_ids(rec_rows):
    """The big-endian u32 identifiers (buffer.rs:99-106) of CUDA record rows,
    as a host uint32 array."""
    import numpy as np
    import torch
    b = rec_rows[:, 63:67].to(torch.int64)
    v = (b[:, 0] << 24) | (b[:, 1] << 16) | (b[:, 2] << 8) | b[:, 3]
    return v.cpu().numpy().astype(np.uint32)


def cfg_flows(dev_index, n=100_000_000, nflows=1_000_000, t=32, steps=10):
    """one SidekickMulti batch of n records over nflows
    flows (src ip = flow number), device-resident output, on a FRESH context
    (its first batch sizes the flow table from nothing).  First-batch and
    steady (median) wall ms.  Check: flow count and inserts, and 8 sampled
    flows' records against the oracle's scalar encode of their ids gathered
    by torch in packet order."""
    import ctypes as C
    import numpy as np
    import torch
    import sidekick_amd as sk
    from oracle import coracle
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import Context, PktStats
    dev = f"cuda:{dev_index}"
    raw, rec, g = make_records(dev, n, 11)
    f = torch.randint(0, nflows, (n,), device=dev, generator=g, dtype=torch.int64)
    for k in range(4):
        rec[:, 26 + k] = ((f >> (8 * k)) & 255).to(torch.uint8)
    distinct = int(torch.unique(f).numel())
    rsz = lib().qk_u32_size(t)
    keys = torch.empty((nflows, 12), dtype=torch.uint8, device=dev)
    sks = torch.empty((nflows, rsz // 4), dtype=torch.int32, device=dev)
    ctx = Context(dev_index)
    times, nf, st = [], C.c_size_t(), PktStats()
    for _ in range(steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib().qk_u32_encode_flows_device(ctx.handle, raw.data_ptr(), n, 67, None, None, t, keys.data_ptr(),
                                              sks.data_ptr(), nflows, C.byref(nf), C.byref(st), None)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        if rc != 0:
            raise RuntimeError(f"qk_u32_encode_flows_device rc={rc}")
    m = int(nf.value)
    kh = keys[:m].cpu().numpy()
    rng = np.random.default_rng(0xF1)
    sample = sorted({0, 1, nflows // 2, nflows - 1, *rng.integers(0, nflows, 4).tolist()})
    ok = True
    for fid in sample:
        key = np.array([*(fid >> (8 * k) & 255 for k in range(4)), 0x11, 0x5C, 192, 168, 0, 9, 0x1F, 0x90], np.uint8)
        row = np.nonzero(np.all(kh == key, axis=1))[0]
        want_ids = record_ids(rec[f == fid])
        if len(want_ids) == 0:
            ok = ok and len(row) == 0
            continue
        if len(row) != 1:
            ok = False
            continue
        q = sk.PowerSumQuackU32.__new__(sk.PowerSumQuackU32)
        q._t = t
        q._buf = C.create_string_buffer(sks[int(row[0])].cpu().numpy().tobytes(), rsz)
        ok = ok and (q.power_sums() == coracle.encode_u32(want_ids, t) and q.count() == len(want_ids)
                     and q.last_value() == int(want_ids[-1]))
    ctx.close()
    del raw, rec, f, keys, sks
    steady = float(np.median(times[1:]))
    return {"workload": f"SURVEY 8f row 1: per-flow batch, {n:.0e} 67-byte records of {nflows:.0e} flows -> one "
                        f"quACK per AddrKey, t={t}, device-resident output, fresh context",
            "first_batch_ms": times[0], "steady_ms_median": steady, "steady_ms_min": float(np.min(times[1:])),
            "first_over_steady": times[0] / steady, "record_hbm_frac": n * 67 / (steady * 1e-3) / (HBM_PEAK_GBS * 1e9),
            "flows": m, "flows_expected": distinct, "inserted": int(st.inserted),
            "check": {"flows_equal": m == distinct, "inserted_equal": int(st.inserted) == n,
                      "sampled_flows": len(sample), "sampled_flows_equal_oracle": ok}}


def cfg_packets(ctx, dev_index, n=100_000_000, t=32, steps=10):
    """one sniff-loop batch (sidekick.rs:76-124) of n
    records -> one quACK.  Median wall ms.  Check: the batch's quACK equals
    the GPU encode of the ids torch extracts from the same records, and a
    1e6-record prefix batch equals the oracle's scalar encode."""
    import numpy as np
    import torch
    import sidekick_amd as sk
    from oracle import coracle
    from sidekick_amd.quack import encode_packets
    dev = f"cuda:{dev_index}"
    raw, rec, _ = make_records(dev, n, 7)
    ip = (10, 0, 2, 1)
    times = []
    for _ in range(steps + 1):
        q = sk.PowerSumQuackU32(t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = encode_packets(q, raw, stride=67, my_ipv4=ip, ctx=ctx)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    b = rec[:, 63:67].to(torch.int64)
    ids = ((b[:, 0] << 24) | (b[:, 1] << 16) | (b[:, 2] << 8) | b[:, 3]).to(torch.int32)
    del b
    ref = sk.PowerSumQuackU32(t)
    ref.insert_batch(ids, ctx=ctx)
    m = 1_000_000
    qp = sk.PowerSumQuackU32(t)
    encode_packets(qp, raw[:m * 67], stride=67, my_ipv4=ip, ctx=ctx)
    want = coracle.encode_u32(ids[:m].cpu().numpy().view(np.uint32), t)
    del raw, rec, ids
    tm = float(np.median(times[1:]))
    return {"workload": f"SURVEY 8f row 2: sniff-loop batch, {n:.0e} 67-byte records in HBM -> extract + encode "
                        f"u32 t={t}",
            "ms_median": tm, "ms_min": float(np.min(times[1:])), "packets_per_s": n / (tm * 1e-3),
            "record_hbm_frac": n * 67 / (tm * 1e-3) / (HBM_PEAK_GBS * 1e9), "inserted": st["inserted"],
            "check": {"inserted_equal": st["inserted"] == n, "equals_gpu_encode_of_extracted_ids": q == ref,
                      "prefix_ids": m, "prefix_equals_oracle": qp.power_sums() == want}}


def secondary_configs(ctx, dev_index):
    """The N = 1 configs block: each entry is its own record or an error
    string (a failure here never voids the measured headline)."""
    import torch
    out = {}
    for name, fn in (("configs2_u64_t80", lambda: cfg_u64(ctx, dev_index)),
                     ("configs4_decode_u32", lambda: cfg_decode(ctx, dev_index, 32)),
                     ("configs4_decode_u64_twin", lambda: cfg_decode(ctx, dev_index, 64)),
                     ("f1_flows_1e6", lambda: cfg_flows(dev_index)),
                     ("f2_packets", lambda: cfg_packets(ctx, dev_index))):
        tc = time.perf_counter()
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001 — reported in the line
            log(f"config {name} failed: {e!r}")
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        out[name]["block_s"] = time.perf_counter() - tc
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


# The published crate at the metric's threshold: benchmark_construct on one
# core of a Xeon E5, `-e 1000 --trials 100`, in its own units — avg_cycles
# (rdtsc around the insert loop) / 1000 ids and avg_us / 1000 ids; t = 32 and
# t = 16 interpolated between the neighbouring rows
# (zip:nsdi24/quack/threshold_vs_encode_time/32.txt:3,6,9,12, 64.txt:24;
# profiles/published/quack_logs.json).
PUBLISHED = {  # (bits, t): (ns per id, TSC cycles per id)
    (32, 32): (117.159 + 0.2 * (161.618 - 117.159), (268165 + 0.2 * (370345 - 268165)) / 1000),
    (32, 16): (34.676 + 0.6 * (75.334 - 34.676), (78220 + 0.6 * (171639 - 78220)) / 1000),
    (64, 80): (461.745, 1060.493),
}


def host_cpu():
    """(model name, logical CPUs) of this host."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def usable_cpus():
    """(CPUs this process may run on, how that was derived): its CPU affinity,
    capped by the cgroup CPU quota when one is set (a GPU box's share of a
    256-CPU host is 16 CPUs; os.cpu_count() shows the whole host)."""
    aff = len(os.sched_getaffinity(0))
    n, how = aff, f"sched_getaffinity: {aff}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            how += f", cgroup cpu.max quota {int(quota) / int(period):g} CPUs"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, how


def cgroup_throttling():
    """nr_periods / nr_throttled / throttled_usec of this process's cgroup
    (cgroup v2 cpu.stat), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            d = dict(line.split() for line in f if line.strip())
        return {k: int(d[k]) for k in ("nr_periods", "nr_throttled", "throttled_usec") if k in d}
    except (OSError, ValueError):
        return None


def cpu_baselines(args, bits, t, start, cnt, ids):
    """The oracle's scalar restatement of the reference insert loop, timed on
    this host over a bounded prefix of the same stream, with the ids
    pre-generated (the crate's benchmark_construct times inserts of
    pre-generated ids): one core, then every core of this process's share."""
    import numpy as np
    import sidekick_amd as sk
    from oracle import coracle
    m = int(min(args.cpu_sample, cnt))
    host_ids = (coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64)(args.seed, m, start)
    # the insert loop timed in the crate's own unit (rdtsc, as its
    # benchmark_construct's avg_cycles) and by the monotonic clock over the
    # same region (the TSC rate comes from this run, not from /proc/cpuinfo),
    # and in core cycles: perf_event_open's user-mode cycle count where the
    # kernel allows it, and the core clock read by a dependent-add chain just
    # before and after the loop; the cgroup's CPU throttling over the region
    thr0 = cgroup_throttling()
    cpu_S, cyc = coracle.encode_cycles(host_ids, t)
    thr1 = cgroup_throttling()
    tsc, ns = cyc["tsc"], cyc["ns"]
    cpu_s = ns * 1e-9
    q = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
    q.insert_batch(ids[:m])                    # GPU on the same prefix: bit-exact parity check
    parity = q.power_sums() == cpu_S
    if not parity:
        log("PARITY FAILURE: GPU power sums differ from the CPU oracle on the sample prefix")
    model, ncpu = host_cpu()
    pub_ns, pub_cyc = PUBLISHED.get((bits, t), (None, None))
    host = f"host {model}, {ncpu} logical CPUs"
    ns_id = cpu_s / m * 1e9
    tsc_id = tsc / m if tsc else None
    tsc_ghz = tsc / ns if tsc else None
    clk = cyc["clock_probe_ghz"]
    if cyc["core_cycles"]:
        core_id, core_how = cyc["core_cycles"] / m, "perf_event_open user-mode cycles"
    elif clk:
        core_id, core_how = ns_id * clk, (f"ns x the core clock of a dependent-add chain ({clk:.2f} GHz; "
                                          f"perf_event_open refused, errno {cyc['perf_errno']})")
    else:
        core_id, core_how = None, "unavailable"
    throttled = None
    if thr0 and thr1:
        throttled = {k: thr1[k] - thr0.get(k, 0) for k in thr1}
    one = {
        "value": m / cpu_s, "unit": "identifiers/s", "cores": 1, "kind": "port",
        "ns_per_id": ns_id, "tsc_cycles_per_id": tsc_id, "tsc_cycles_per_power": tsc_id / t if tsc_id else None,
        "tsc_ghz": tsc_ghz,
        "core_cycles_per_id": core_id, "core_cycles_per_power": core_id / t if core_id else None,
        "core_cycles_source": core_how, "core_clock_probe_ghz": clk,
        "instructions_per_id": cyc["instructions"] / m if cyc["instructions"] else None,
        "cgroup_throttling_during_loop": throttled,
        "sample": f"first {m} ids of the same stream (seed {hex(args.seed)}), pre-generated, inserted by the "
                  f"scalar C restatement of the reference insert loop (oracle/quack_oracle.c qo_encode_cycles: "
                  f"t - 1 dependent mul + mod-by-constant steps per id, the sums' conditional subtract as a "
                  f"mask), 1 core, {cpu_s:.1f} s = {ns_id:.1f} ns/id"
                  + (f" = {tsc_id:.1f} TSC cycles/id (rdtsc around the loop, TSC at {tsc_ghz:.3f} GHz from the "
                     f"same region)" if tsc_id else "")
                  + (f" = {core_id:.1f} core cycles/id, {core_id / t:.1f} per power ({core_how})" if core_id else "")
                  + (f"; cgroup throttling over the loop: {throttled}" if throttled is not None else "")
                  + f"; {host}"
                  + (f"; the published crate in the same units: {pub_cyc:.1f} TSC cycles/id = {pub_ns:.1f} ns/id "
                     f"at u{bits} t={t} on one Xeon E5 core (benchmark_construct avg_cycles / 1000 ids; "
                     f"BASELINE.md): this port takes {tsc_id / pub_cyc:.2f}x the crate's TSC cycles per id. "
                     f"A power step is one dependent chain of a 64-bit multiply and the modulo by the constant "
                     f"prime (multiply-high, shifts, subtracts), so the loop is latency-bound: "
                     + (f"{core_id / (t - 1):.1f} core cycles per step here" if core_id and t > 1 else "")
                     + f"; the TSC ratio to the crate follows the two hosts' core-clock / TSC ratios. (Until round "
                     f"5 the port's modular add compiled to a branch that mispredicted every other power: 1.77x "
                     f"the crate.)"
                     if pub_cyc and tsc_id else ""),
        "published_crate_ns_per_id": pub_ns,
        "published_crate_tsc_cycles_per_id": pub_cyc,
        "parity_with_gpu": parity,
    }
    thr, how = usable_cpus()
    thr = max(1, min(thr, 256))
    mm = int(min(m * thr // 3, cnt))           # ~1/3 of the 1-core sample per thread
    host_mm = (coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64)(args.seed, mm, start)
    tc = time.perf_counter()
    mt_S = coracle.encode_mt(host_mm, t, thr)
    mt_s = time.perf_counter() - tc
    del host_mm
    q = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
    q.insert_batch(ids[:mm])
    allc = {
        "value": mm / mt_s, "unit": "identifiers/s", "cores": thr, "kind": "port",
        "sample": f"first {mm} ids of the same stream, pre-generated, {thr} threads x {mm // thr} ids, one partial "
                  f"sketch per thread merged (oracle/quack_oracle.c qo_encode_mt), {mt_s:.1f} s; threads = the "
                  f"CPUs this process may use ({how}); {host}",
        "parity_with_gpu": q.power_sums() == mt_S,
    }
    return one, allc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ids-per-gpu", type=float, default=1e9, help="ids per GPU (weak scaling)")
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--bits", type=int, default=32, choices=(32, 64))
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    ap.add_argument("--cpu-sample", type=float, default=1e8, help="ids for the CPU baseline (0 disables)")
    ap.add_argument("--configs", type=int, default=1,
                    help="N = 1: after the headline, the untimed self-checked block of the other single-GPU configs "
                         "(configs[2], configs[4] and its u64 twin, SURVEY 8f flows / packets); 0 skips it")
    ap.add_argument("--grid", type=int, default=0, help="override workgroups per launch")
    ap.add_argument("--knob", action="append", default=[], help="NAME=VALUE measurement knob (qk_ctx_set_knob)")
    ap.add_argument("--comm", action="store_true",
                    help="at N = 1 too, run each step through the native communicator (a world-1 ncclReduce)")
    ap.add_argument("--dist-backend", default="auto", choices=("auto", "rccl", "host"),
                    help="rccl: the native communicator over RCCL/xGMI (one GPU per rank); host: the same native "
                         "protocol with its collectives over gloo (qk_comm_init_host), to rehearse more ranks than "
                         "GPUs; auto: rccl when the node has a GPU per rank, else host")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import sidekick_amd as sk
    from sidekick_amd import dist as skd
    from sidekick_amd.quack import encode_device_async, fill_splitmix, merge_partial, partial_words

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    ndev = torch.cuda.device_count()
    dev_index = local % ndev  # == local on a real node (one process per GPU)
    torch.cuda.set_device(dev_index)
    comm = None
    data_path = "single"
    if world > 1:
        dist.init_process_group("gloo")          # control plane only
        backend = args.dist_backend
        if backend == "auto":
            backend = "rccl" if ndev >= world else "host"
        if backend == "rccl":
            if ndev < world:
                raise SystemExit(f"--dist-backend rccl needs a GPU per rank ({world} ranks, {ndev} GPUs)")
            # a failure here is an error (torch.distributed.run then stops every rank)
            comm = skd.Comm.from_process_group(dev_index)
            data_path = "rccl"
        else:
            comm = skd.Comm.init_host(skd.ProcessGroupChannel(), rank, world, dev_index)
            data_path = "host"
    elif args.comm:
        comm = skd.Comm.create([dev_index])
        data_path = "rccl"

    n = int(args.ids_per_gpu)
    t, bits = args.t, args.bits
    n_total = n * world
    start, cnt = skd.shard(n_total, rank, world)
    # the context that runs the encode: the communicator's own for the native
    # multi-GPU path (profiling and the grid knob must reach that one)
    ctx = comm.context(0) if comm is not None else sk.get_context(dev_index)
    if args.grid:
        ctx.set_grid(args.grid)
    for kv in args.knob:                       # measurements only (tools/gpu_check.sh sweeps)
        k, v = kv.split("=")
        ctx.set_knob(k, int(v))

    idt = torch.int32 if bits == 32 else torch.int64
    ids = torch.empty(cnt, dtype=idt, device=f"cuda:{dev_index}")
    fill_splitmix(ctx, ids, args.seed, start, bits=bits)
    partial = torch.zeros(partial_words(t, bits), dtype=torch.int64, device=f"cuda:{dev_index}")
    torch.cuda.synchronize()

    def step():
        if comm is not None:
            comm.encode_sharded_async([ids], t, bits=bits, root=0)   # encode + one reduce (comm.hip)
            return
        encode_device_async(ctx, ids, t, partial, bits=bits)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.kernel_stats()  # drop warmup events
    ctx.set_profiling(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    kern_ms, launches = ctx.kernel_stats()
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
    ms_per_step = elapsed / args.steps * 1e3
    kern_avg_ms = kern_ms / max(launches, 1)

    # result of the last step (rank 0 holds the reduced sum)
    if comm is not None:
        qres = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
        comm.encode_sharded_wait(qres)
    part_host = partial.cpu().numpy().view(np.uint64)
    if rank == 0:
        if comm is not None:
            S, count = qres.power_sums(), qres.count()
        else:
            S, count = skd.fold_partial_sum(part_host, t, bits)
        log(f"encode result: count={count} S[0..3]={S[:3]}")
        digest = digest_of(S, count)

    # untimed, after the timed region: this run's shader clock under the
    # kernel (roofline.valu), and for N > 1 the strong-scaling parity pass and
    # what RCCL itself reports on every rank
    clock_ghz = measure_clock(ctx, step, dev_index, kern_avg_ms)
    if comm is not None:   # drain the probe's steps (the root merges into a throwaway sketch)
        comm.encode_sharded_wait((sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t))
    strong = dec = None
    ranks = None
    if world > 1:
        # untimed checks after the measurement: a failure is reported in the
        # line, not raised (the measured value stands).  The native
        # communicator makes a collective's failure the same status on every
        # rank; the ranks also agree over gloo before the next check starts,
        # so none enters a collective its peers have left.
        def agreed(fn, *a):
            err = None
            try:
                res = fn(*a)
            except Exception as e:  # noqa: BLE001
                res, err = None, f"{type(e).__name__}: {e}"
                log(f"rank {rank}: {fn.__name__} failed: {err}")
            bad = torch.tensor([1 if err else 0], dtype=torch.int64)
            dist.all_reduce(bad, op=dist.ReduceOp.SUM)
            if int(bad.item()):
                return {"error": err or f"failed on {int(bad.item())} other rank(s)"}, False
            return res, True
        strong, ok = agreed(strong_scaling_check, args, comm, ctx, ids, rank, world, dev_index, bits, t)
        dec = agreed(decode_check, comm, ctx, ids, n, rank, world, bits)[0] if ok else {"error": "skipped"}
        info = comm.rccl_info()
        props = torch.cuda.get_device_properties(dev_index)
        mine = {"rank": rank, "local_rank": local, "device": dev_index,
                "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")),
                "rccl_count": info[0] if info else None, "rccl_device": info[1] if info else None,
                "rccl_rank": info[2] if info else None}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)

    if rank != 0:
        if world > 1:
            dist.barrier()
            if comm is not None:
                comm.close()
            dist.destroy_process_group()
        return

    bytes_per_id = 4 if bits == 32 else 8
    value = n_total * args.steps / elapsed
    achieved_gbs = bytes_per_id * cnt / (kern_avg_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(bits, t, cnt)
    valu = valu_roofline(bits, t, cnt, kern_avg_ms, clock_ghz)

    out = {
        "metric": f"quACK encode identifiers/s (device-resident), u{bits} ids, threshold t={t}",
        "value": value,
        "unit": "identifiers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32" if bits == 32 else "u64",
        "data": "synthetic: splitmix64 uniform ids generated in HBM (seeded), no host copies in the timed region",
        "config": {
            "workload": f"encode {n:.0e} u{bits} ids per GPU at t={t}, device-resident"
                        + {"single": "",
                           "rccl": f", {world} contiguous shards + one RCCL reduce over xGMI (native qk_comm)",
                           "host": f", {world} contiguous shards on {ndev} GPU(s) + one reduce of the native "
                                   f"protocol over gloo (qk_comm_init_host): a rehearsal, not a scaling result"
                           }[data_path],
            "ids_per_gpu": cnt, "global_ids": n_total, "threshold": t, "bits": bits,
            "seed": hex(args.seed), "parallelism": f"shard{world}", "collectives": data_path,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": f"k_encode_u{bits} (avg of {launches} launches, HIP events on the launch stream)",
            "kernel_avg_ms": kern_avg_ms,
            "algorithmic_bytes_per_launch": bytes_per_id * cnt,
            "valu": valu,
        },
        "cpu_baseline": None,
        "clock_ghz": clock_ghz,
        "result": {"count": count, "power_sums_head": S[:4], "digest": digest,
                   "note": "sha256 of the folded power sums of the whole global stream of this run "
                           "(N x ids-per-gpu ids)"},
    }
    rec = RECORDED_DIGESTS.get((bits, t, n_total, args.seed))
    if rec:
        out["result"]["equals_recorded"] = digest == rec
    if world > 1:
        out["parity"] = strong
        out["decode_parity"] = dec
        out["ranks"] = ranks
        if data_path == "rccl":
            out["rccl"] = {"ranks_reported": sorted({r["rccl_count"] for r in ranks}),
                           "all_ranks_joined": all(r["rccl_count"] == world for r in ranks),
                           "devices": [r["rccl_device"] for r in ranks],
                           "user_ranks": [r["rccl_rank"] for r in ranks]}

    if world == 1 and args.configs and bits == 32 and t == 32:
        out["configs"] = secondary_configs(ctx, dev_index)
    if world == 1 and args.cpu_sample > 0:
        out["cpu_baseline"], out["cpu_baseline_all_cores"] = cpu_baselines(args, bits, t, start, cnt, ids)
    print(json.dumps(out), flush=True)
    if comm is not None and world == 1:
        comm.close()
    if world > 1:
        dist.barrier()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
