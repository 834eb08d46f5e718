"""GPU parity of the batch encode path (gfx950 kernels through the C ABI)
against the oracle and the golden fixtures; bit-exact (integer arithmetic).
Full-size (1e9) behaviour is checked through size-independent properties:
additivity under arbitrary splits and grid-shape independence."""
import ctypes as C

import numpy as np
import pytest
import torch

import sidekick_amd as sk
from sidekick_amd._lib import lib
from sidekick_amd.quack import encode_device_async, fill_splitmix, merge_partial, partial_words
from oracle import coracle, quack_oracle as qo

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev_u32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)


def dev_u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def gpu_state(ids, t, bits=32, ctx=None):
    q = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
    q.insert_batch(ids if isinstance(ids, torch.Tensor) else (dev_u32(ids) if bits == 32 else dev_u64(ids)), ctx=ctx)
    return q


def test_kats_and_empty(golden):
    for k in golden["kats"]:
        q = gpu_state(np.array(k["ids"], dtype=np.uint32 if k["bits"] == 32 else np.uint64), k["t"], k["bits"])
        assert q.power_sums() == k["expect"]["power_sums"], k["name"]
        assert q.count() == k["expect"]["count"]
        assert q.last_value() == k["expect"]["last_value"]


def test_edges(golden):
    for e in golden["edges"]:
        ids = np.array([int(v) for v in e["ids"]], dtype=np.uint32 if e["bits"] == 32 else np.uint64)
        q = gpu_state(ids, e["t"], e["bits"])
        assert q.power_sums() == [int(v) for v in e["expect"]["power_sums"]], (e["bits"], e["t"])
        assert q.last_value() == int(e["expect"]["last_value"])


def test_golden_streams(golden):
    for s in golden["streams"]:
        if s["bits"] == 32:
            q = gpu_state(qo.ids_u32(s["seed"], s["n"]), s["t"], 32)
        else:
            q = gpu_state(qo.ids_u64(s["seed"], s["n"]), s["t"], 64)
        assert q.power_sums() == [int(v) for v in s["expect"]["power_sums"]], (s["bits"], s["n"], s["t"])
        assert q.count() == s["n"]


U32_TS = list(range(1, 34)) + [36, 40, 41, 47, 48, 49, 55, 56, 57, 63, 64, 65, 80, 81, 88, 100, 120, 128, 129, 168,
                               169, 256, 300, 513, 1023, 1024]
U64_TS = [1, 2, 3, 5, 8, 12, 16, 19, 20, 21, 32, 40, 64, 65, 72, 73, 74, 79, 80, 81, 88, 96, 97, 120, 160, 161, 176,
          240, 300, 513, 1024]


@pytest.mark.parametrize("t", U32_TS)
def test_u32_threshold_sweep(t):
    ids = coracle.splitmix_u32(0xABC0 + t, 20011)
    assert gpu_state(ids, t).power_sums() == coracle.encode_u32(ids, t)


@pytest.mark.parametrize("t", U64_TS)
def test_u64_threshold_sweep(t):
    ids = coracle.splitmix_u64(0xDEF0 + t, 3001)
    assert gpu_state(ids, t, 64).power_sums() == coracle.encode_u64(ids, t)


@pytest.mark.parametrize("t", [81, 90, 160, 300, 1024])
def test_u64_multipass_edges(t):
    """u64 thresholds above 80 run as baby-step/giant-step passes (powers
    1..80, then offset passes of <= 80 with giants x^(base + 8a) and x^base by
    square-and-multiply): field-edge ids, misaligned starts, ragged tails,
    incremental batches."""
    P64 = 18446744073709551557
    ids = coracle.splitmix_u64(0x64 + t, 20_011)
    edge = np.array([0, 1, P64 - 1, P64, P64 + 1, 2**64 - 1, 2**63], dtype=np.uint64)
    ids[::991] = np.resize(edge, len(ids[::991]))
    d = dev_u64(ids)
    for off in (0, 1, 3):
        assert gpu_state(d[off:], t, 64).power_sums() == coracle.encode_u64(ids[off:], t), (t, off)
    q = sk.PowerSumQuackU64(t)
    for a, b in ((0, 5), (5, 10_000), (10_000, len(ids))):
        q.insert_batch(d[a:b])
    assert q.power_sums() == coracle.encode_u64(ids, t)
    assert q.count() == len(ids) and q.last_value() == int(ids[-1])


@pytest.mark.parametrize("t", [81, 128, 300, 1024])
def test_u32_multipass_edges(golden, t):
    """Thresholds above 80 run as baby-step/giant-step passes (80 powers, then
    offset passes of <= 48 with giants from x^base): ids at the field edges,
    the lazy-fold wrap ids of the shared baby chain, misaligned starts, and
    equality with the power chain (the oracle here; knob u32_passes = 0
    selects the chain on the device)."""
    P32 = 4294967291
    ids = coracle.splitmix_u32(0x77 + t, 30_011)
    edge = np.array([0, 1, P32 - 1, P32, P32 + 1, 2**32 - 1, 2**31], dtype=np.uint32)
    ids[::997] = np.resize(edge, len(ids[::997]))
    wraps = np.array(golden["bsgs_wrap_ids"]["8x10"], dtype=np.uint32)
    ids[5000:5000 + 64 * len(wraps):64] = wraps
    d = dev_u32(ids)
    for off in (0, 1, 3):
        assert gpu_state(d[off:], t).power_sums() == coracle.encode_u32(ids[off:], t), (t, off)


@pytest.mark.parametrize("t", [80, 73, 96, 160, 250])
def test_u64_max_ids_carry_storm(t):
    """ids at the top of the u64 range (2^64-1, p, p+1, ...): the largest
    products, so the MAC accumulators of the u64 BSGS kernel wrap on almost
    every multiply-accumulate."""
    P64 = 18446744073709551557
    edge = np.array([2**64 - 1, 2**64 - 2, P64 - 1, P64, P64 + 1, 2**63, 2**64 - 60], dtype=np.uint64)
    ids = np.resize(edge, 100_003)
    ids[::7] = coracle.splitmix_u64(3, len(ids[::7]))
    assert gpu_state(ids, t, 64).power_sums() == coracle.encode_u64(ids, t)


@pytest.mark.parametrize("bits", [32, 64])
def test_misaligned_and_ragged(bits):
    base_n = 4099
    ids = coracle.splitmix_u32(5, base_n) if bits == 32 else coracle.splitmix_u64(5, base_n)
    d = dev_u32(ids) if bits == 32 else dev_u64(ids)
    enc = coracle.encode_u32 if bits == 32 else coracle.encode_u64
    for off in range(0, 5):
        for n in (0, 1, 2, 3, 4, 5, 7, 8, 9, 17, 64, 257, 1000):
            q = gpu_state(d[off:off + n], 32, bits)
            assert q.power_sums() == enc(ids[off:off + n], 32), (off, n)
            assert q.count() == n
            assert q.last_value() == (int(ids[off + n - 1]) if n else None)


@pytest.mark.parametrize("bits,t", [(32, 32), (32, 16), (32, 80), (32, 200), (64, 80), (64, 16), (64, 200)])
def test_grid_shape_independent(bits, t):
    n = 300_007
    ids = coracle.splitmix_u32(77, n) if bits == 32 else coracle.splitmix_u64(77, n)
    want = (coracle.encode_u32 if bits == 32 else coracle.encode_u64)(ids, t)
    ctx = sk.Context(0)
    try:
        for g in (0, 1, 3, 8, 255, 1024, 4096):
            ctx.set_grid(g)
            assert gpu_state(ids, t, bits, ctx=ctx).power_sums() == want, g
    finally:
        ctx.close()


def test_device_fill_matches_oracle_generator():
    ctx = sk.get_context(0)
    out = torch.empty(100_003, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, out, 0x1234, start=999, bits=32)
    assert (out.cpu().numpy().view(np.uint32) == coracle.splitmix_u32(0x1234, 100_003, start=999)).all()
    out64 = torch.empty(50_001, dtype=torch.int64, device=DEV)
    fill_splitmix(ctx, out64, 0x1234, start=5, bits=64)
    assert (out64.cpu().numpy().view(np.uint64) == coracle.splitmix_u64(0x1234, 50_001, start=5)).all()


def test_large_stream_vs_oracle():
    """1e7 ids at t = 32 against the scalar C oracle (a few seconds of CPU)."""
    n, t, seed = 10_000_000, 32, 0x5EED0002
    ctx = sk.get_context(0)
    d = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, d, seed)
    q = gpu_state(d, t)
    assert q.power_sums() == coracle.encode_u32_seed(seed, n, t)


def test_async_partial_api():
    ctx = sk.get_context(0)
    n, t = 1_000_003, 32
    ids = coracle.splitmix_u32(9, n)
    d = dev_u32(ids)
    part = torch.zeros(partial_words(t), dtype=torch.int64, device=DEV)
    encode_device_async(ctx, d, t, part)
    torch.cuda.synchronize()
    h = part.cpu().numpy().view(np.uint64)
    assert h[:t].tolist() == coracle.encode_u32(ids, t)
    assert int(h[t]) == n and int(h[t + 1]) == int(ids[-1])
    q = sk.PowerSumQuackU32(t)
    merge_partial(q, h, True, int(ids[-1]))
    assert q.power_sums() == h[:t].tolist() and q.count() == n


def test_u64_async_partial_limbs():
    ctx = sk.get_context(0)
    n, t = 100_003, 80
    ids = coracle.splitmix_u64(10, n)
    part = torch.zeros(partial_words(t, 64), dtype=torch.int64, device=DEV)
    encode_device_async(ctx, dev_u64(ids), t, part, bits=64)
    torch.cuda.synchronize()
    h = [int(v) for v in part.cpu().numpy().view(np.uint64)]
    S = [h[2 * k] + (h[2 * k + 1] << 32) for k in range(t)]
    assert S == coracle.encode_u64(ids, t)
    assert all(h[2 * k] < 2**32 and h[2 * k + 1] < 2**32 for k in range(t))


@pytest.mark.parametrize("pinned", [False, True])
def test_host_input_path_multi_chunk(pinned):
    """Host-resident ids (the sniffed-packet case): > one 64 MiB chunk."""
    n, t = 40_000_003, 32
    ids = coracle.splitmix_u32(0x77, n)
    if pinned:
        buf = torch.empty(n, dtype=torch.int32, pin_memory=True)
        buf.numpy().view(np.uint32)[:] = ids
        ids = buf.numpy().view(np.uint32)
    q = sk.PowerSumQuackU32(t)
    q.insert_batch(ids)
    ref = gpu_state(dev_u32(ids), t)
    assert q == ref
    assert q.count() == n and q.last_value() == int(ids[-1])


def test_incremental_batches_equal_single_batch():
    ids = coracle.splitmix_u32(0x99, 100_000)
    whole = gpu_state(ids, 32)
    inc = sk.PowerSumQuackU32(32)
    for a, b in ((0, 1), (1, 33_333), (33_333, 33_334), (33_334, 100_000)):
        inc.insert_batch(dev_u32(ids[a:b]))
    assert inc == whole
    # mixing the per-packet host insert and the batch path
    mix = sk.PowerSumQuackU32(32)
    for x in ids[:10].tolist():
        mix.insert(x)
    mix.insert_batch(dev_u32(ids[10:]))
    assert mix == whole


def test_rejects_host_pointer_on_device_entry():
    ctx = sk.get_context(0)
    arr = np.arange(16, dtype=np.uint32)
    q = sk.PowerSumQuackU32(4)
    rc = lib().qk_u32_encode_device(ctx.handle, arr.ctypes.data, arr.size, q._buf, None)
    assert rc == -1  # QK_E_INVAL, not a fault


def test_full_size_1e9_properties():
    """configs[1] size: 1e9 u32 ids at t = 32.  Size-independent checks: the
    whole-array encode equals the merge of uneven pieces and is independent
    of the grid shape; count / last_value are exact."""
    n, t, seed = 1_000_000_000, 32, 0x5EED0002
    ctx = sk.get_context(0)
    d = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, d, seed)
    whole = gpu_state(d, t)
    assert whole.count() == n
    assert whole.last_value() == int(coracle.splitmix_u32(seed, 1, start=n - 1)[0])
    pieces = sk.PowerSumQuackU32(t)
    for a, b in ((0, 123_456_789), (123_456_789, 123_456_790), (123_456_790, 999_999_999), (999_999_999, n)):
        pieces.insert_batch(d[a:b])
    assert pieces == whole
    c2 = sk.Context(0)
    try:
        c2.set_grid(1000)
        assert gpu_state(d, t, ctx=c2) == whole
    finally:
        c2.close()
    # the first 2e6 ids against the oracle (same stream, same kernels)
    assert gpu_state(d[:2_000_000], t).power_sums() == coracle.encode_u32_seed(seed, 2_000_000, t)
    del d
    torch.cuda.empty_cache()


def test_full_size_u64_properties():
    """configs[2] at full size: 1e9 u64 ids at t = 80 (8 GB).  Additivity over
    uneven pieces, grid-shape independence, exact count / last_value, and
    oracle agreement on a prefix of the same stream."""
    n, t, seed = 1_000_000_000, 80, 0x5EED0003
    ctx = sk.get_context(0)
    d = torch.empty(n, dtype=torch.int64, device=DEV)
    fill_splitmix(ctx, d, seed, bits=64)
    whole = gpu_state(d, t, 64)
    assert whole.count() == n
    assert whole.last_value() == int(coracle.splitmix_u64(seed, 1, start=n - 1)[0])
    pieces = sk.PowerSumQuackU64(t)
    for a, b in ((0, 77_777_777), (77_777_777, 77_777_778), (77_777_778, 999_999_999), (999_999_999, n)):
        pieces.insert_batch(d[a:b])
    assert pieces == whole
    c2 = sk.Context(0)
    try:
        c2.set_grid(1000)
        assert gpu_state(d, t, 64, ctx=c2) == whole
    finally:
        c2.close()
    assert gpu_state(d[:200_000], t, 64).power_sums() == coracle.encode_u64_seed(seed, 200_000, t)
    del d
    torch.cuda.empty_cache()


# (babies x giants) chain of the kernel each threshold runs (encode.hip enc32;
# t > 80: pass 0 is the (8,10) kernel)
def wrap_cfg(t):
    for hi, cfg in ((8, "4x2"), (12, "4x3"), (16, "4x4"), (24, "6x4"), (32, "8x4"), (40, "8x5"), (48, "8x6"),
                    (56, "8x7"), (64, "8x8")):
        if t <= hi:
            return cfg
    return "8x10"


@pytest.mark.parametrize("t", [5, 8, 9, 12, 13, 16, 17, 20, 24, 25, 31, 32, 33, 37, 40, 41, 44, 48, 49, 56, 57, 64,
                               65, 72, 80, 96])
def test_bsgs_rare_wrap_branch(golden, t):
    """Ids whose lazy folds wrap (prob ~2.6e-8 per id) force the exact
    recompute branch of the baby-step/giant-step kernel: alone in a wave,
    several in one wave, and in the unaligned head/tail (scalar path)."""
    cfg = wrap_cfg(t)
    wraps = np.array(golden["bsgs_wrap_ids"][cfg], dtype=np.uint32)
    ids = coracle.splitmix_u32(0xF00D + t, 20_003)
    ids[100] = wraps[0]                      # one lane of one wave
    ids[4096:4096 + 4] = wraps[:4]           # four chains of one lane
    ids[5000:5000 + 64 * 4:64] = wraps[:4]   # several lanes of one wave
    ids[-1] = wraps[-1]                      # tail (scalar path)
    d = dev_u32(ids)
    for off in (0, 1, 3):                    # head (scalar path) at off 1, 3
        sub = ids[off:]
        assert gpu_state(d[off:], t).power_sums() == coracle.encode_u32(sub, t), (t, off)
    only = dev_u32(np.tile(wraps, 11))
    assert gpu_state(only, t).power_sums() == coracle.encode_u32(np.tile(wraps, 11), t)


P32, P64 = 4294967291, 18446744073709551557


@pytest.mark.parametrize("bits,t,m", [(32, 32, 1_000_003), (64, 80, 500_009), (32, 100, 1_000_003),
                                      (64, 100, 500_009)])
def test_beyond_2pow32_ids(bits, t, m):
    """Maximum sizes: one encode over more than 2^32 ids (17 GB of u32, 34 GB
    of u64).  The stream is one oracle-encoded block tiled R times, so the
    expected sums are R * S_block mod p exactly; count wraps as the crate's
    u32 does; last_value is the block's last id."""
    p = P32 if bits == 32 else P64
    blk = coracle.splitmix_u32(0xB16 + t, m) if bits == 32 else coracle.splitmix_u64(0xB16 + t, m)
    want_blk = coracle.encode_u32(blk, t) if bits == 32 else coracle.encode_u64(blk, t)
    R = (1 << 32) // m + 2
    n = R * m
    assert n > (1 << 32)
    big = (dev_u32(blk) if bits == 32 else dev_u64(blk)).repeat(R)
    q = gpu_state(big, t, bits)
    assert q.count() == n & 0xFFFFFFFF
    assert q.last_value() == int(blk[-1])
    assert q.power_sums() == [(R * s) % p for s in want_blk]
    del big
    torch.cuda.empty_cache()


def test_root_test_positions_beyond_2pow32():
    """Hit positions past 2^32 in a 4.3e9-entry candidate log come back as
    exact 64-bit positions in log order (u32 log, d = 3 roots planted at the
    start, past 2^32 and at the end)."""
    m = 1_000_003
    blk = coracle.splitmix_u32(0x5106, m)
    R = (1 << 32) // m + 2
    n = R * m
    roots = [v for v in (7, 11, 13, 17, 19) if not np.isin(v, blk)][:3]
    assert len(roots) == 3
    log = dev_u32(blk).repeat(R)
    pos = [5, (1 << 32) + 7, n - 1]
    for p_, r in zip(pos, roots):
        log[p_] = int(np.uint32(r).view(np.int32))
    want = sorted(pos)
    q = sk.PowerSumQuackU32(8)
    for r in roots:
        q.insert(r)
    hits = q.root_test(q.to_coeffs(), log)
    assert hits == want
    del log
    torch.cuda.empty_cache()


def test_root_test_u64_positions_beyond_2pow32():
    """u64 log of 4.3e9 entries (34 GB): roots planted at the start, past
    2^32 and at the end come back as exact 64-bit positions (d = 3 runs the
    Horner kernel; the 17-root case the baby-step/giant-step one)."""
    m = 500_009
    blk = coracle.splitmix_u64(0x5107, m)
    R = (1 << 32) // m + 2
    n = R * m
    cands = [v for v in range(2, 200) if not np.isin(np.uint64(v), blk)]
    log = dev_u64(blk).repeat(R)
    for d in (3, 17):
        roots = cands[:d]
        pos = sorted({5 + 3 * i for i in range(d // 2)} | {(1 << 32) + 7 + 11 * i for i in range(d - d // 2 - 1)}
                     | {n - 1})
        assert len(pos) == d
        saved = [int(log[p_].item()) for p_ in pos]
        for p_, r in zip(pos, roots):
            log[p_] = int(np.uint64(r).view(np.int64))
        q = sk.PowerSumQuackU64(d)
        for r in roots:
            q.insert(r)
        assert q.root_test(q.to_coeffs(), log) == pos, d
        for p_, v in zip(pos, saved):
            log[p_] = v
    del log
    torch.cuda.empty_cache()
