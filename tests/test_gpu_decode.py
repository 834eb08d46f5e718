"""GPU parity of the decode-missing path (host Newton's identities + gfx950
root-test kernel through the C ABI) against the oracle and golden fixtures.
Mirrors media_client.rs:295-313: diff = mine - received; coeffs =
diff.to_coeffs(); every log entry with eval(coeffs, id) == 0 is missing."""
import numpy as np
import pytest
import torch

import sidekick_amd as sk
from sidekick_amd.quack import fill_splitmix
from oracle import coracle, quack_oracle as qo

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, bits=32):
    if bits == 32:
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def QT(bits):
    return sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64


@pytest.fixture(autouse=True, params=["horner", "scan", "auto"])
def root_test_mode(request):
    """Every test of this module runs three times: the root test by Horner
    per candidate (k_root_test_*), by host root finding + the root-set scan
    (roots.cpp, k_root_scan; forced for 2 <= d <= 256) handing its results
    over through pinned host slots, and as the cost model picks (the
    default): the same hit lists."""
    ctx = sk.get_context(0)
    ctx.set_knob("root_test", {"horner": 1, "scan": 2, "auto": 0}[request.param])
    yield request.param
    ctx.set_knob("root_test", 0)


def _poly_mul(a, b, p):
    A, B = [1] + list(a), [1] + list(b)
    out = [0] * (len(A) + len(B) - 1)
    for i, x in enumerate(A):
        for j, y in enumerate(B):
            out[i + j] = (out[i + j] + x * y) % p
    return out[1:]


@pytest.mark.parametrize("bits", [32, 64])
def test_root_test_non_splitting_polynomials(bits):
    """Coefficient vectors that are not a product of linear factors over
    GF(p): planted log roots times irreducible quadratics, and random
    vectors.  Hits = the oracle's evaluation, whichever path runs."""
    p = qo.MOD[bits]
    rng = np.random.default_rng(bits)
    n = 40_003
    log = coracle.splitmix_u32(77, n) if bits == 32 else coracle.splitmix_u64(77, n)
    for trial in range(4):
        planted = [int(log[i]) for i in rng.choice(n, size=3 + trial, replace=False)]
        q = QT(bits)(len(planted))
        for x in planted:
            q.insert(x)
        c = list(q.to_coeffs())
        for _ in range(1 + trial % 2):
            while True:
                nr = int(rng.integers(2, min(p, 1 << 62)))
                if pow(nr, (p - 1) // 2, p) == p - 1:
                    break
            s0 = int(rng.integers(0, min(p, 1 << 62)))
            c = _poly_mul(c, [(-2 * s0) % p, (s0 * s0 - nr) % p], p)
        want = qo.root_test_indices(c, log.tolist(), p)
        got = QT(bits)(1).root_test(c, dev(log, bits))
        assert got == want and len(got) >= len(planted)
    for d in (5, 12, 31):
        c = [int(v) for v in rng.integers(0, min(p, 1 << 62), size=d)]
        assert QT(bits)(1).root_test(c, dev(log, bits)) == qo.root_test_indices(c, log.tolist(), p)


def test_root_test_u32_aliases_and_zero():
    """Roots 0 and 1: log entries 0, p, 1, p + 1 all hit (x mod p); 2^32 - 1
    (= 4 mod p) does not unless 4 is a root."""
    p = qo.MOD[32]
    log = coracle.splitmix_u32(5, 10_007)
    specials = [0, p, 1, p + 1, 2**32 - 1, 4, p - 1]
    pos = [10, 999, 1000, 4097, 5000, 7001, 10_006]
    log[pos] = specials
    q = sk.PowerSumQuackU32(3)
    for x in (0, 1, p - 1):
        q.insert(x)
    c = q.to_coeffs()
    got = q.root_test(c, dev(log))
    assert got == qo.root_test_indices(c, log.tolist(), p)
    assert {10, 999, 1000, 4097, 10_006} <= set(got) and 5000 not in got


def test_golden_decodes(golden):
    for g in golden["decodes"]:
        bits, n, t = g["bits"], g["n"], g["t"]
        log = qo.ids_u32(g["seed"], n) if bits == 32 else qo.ids_u64(g["seed"], n)
        if g["dup_at"] is not None:
            log[g["dup_at"]] = log[g["dup_of"]]
        keep = np.ones(n, dtype=bool)
        keep[g["drops"]] = False
        sent, recv = QT(bits)(t), QT(bits)(t)
        sent.insert_batch(dev(log, bits))
        recv.insert_batch(dev(log[keep], bits))
        diff = sent.clone()
        diff.sub_assign(recv)
        assert diff.count() == g["diff_count"]
        assert diff.power_sums() == [int(v) for v in g["diff_power_sums"]], g["name"]
        coeffs = diff.to_coeffs()
        assert list(coeffs) == [int(c) for c in g["coeffs"]]
        assert diff.root_test(coeffs, dev(log, bits)) == g["hits"], g["name"]
        missing = diff.decode_with_log(dev(log, bits))
        assert missing == [int(log[i]) for i in g["hits"]]


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("d", [1, 2, 3, 7, 8, 15, 16, 17, 20, 23, 24, 25, 31, 32, 33, 40, 64, 100, 255, 256,
                               999, 1000, 1001])
def test_root_test_vs_oracle(bits, d):
    rng = np.random.default_rng(d * 7 + bits)
    n = 50_001
    log = coracle.splitmix_u32(1000 + d, n) if bits == 32 else coracle.splitmix_u64(1000 + d, n)
    roots_at = rng.choice(n, size=d, replace=False)
    q = QT(bits)(max(d, 1))
    for i in roots_at:
        q.insert(int(log[i]))
    c = q.to_coeffs()
    # plant extra copies of two roots
    log[(roots_at[0] + 17) % n] = log[roots_at[0]]
    log[n - 1] = log[roots_at[-1]]
    want, _ = (coracle.root_test_u32 if bits == 32 else coracle.root_test_u64)(c, log)
    got = q.root_test(c, dev(log, bits))
    assert got == want.tolist()
    assert set(roots_at.tolist()) <= set(got)


@pytest.mark.parametrize("bits,t", [(32, 8), (64, 8), (64, 20)])
def test_root_test_misaligned_small(bits, t):
    log = coracle.splitmix_u32(3, 300) if bits == 32 else coracle.splitmix_u64(3, 300)
    q = QT(bits)(t)
    for i in (0, 5, 6, 150, 299):
        q.insert(int(log[i]))
    c = q.to_coeffs()
    d = dev(log, bits)
    for off in range(5):
        for n in (0, 1, 2, 3, 4, 5, 6, 7, 9, 151, 295):
            sub = log[off:off + n]
            want, _ = (coracle.root_test_u32 if bits == 32 else coracle.root_test_u64)(c, sub)
            assert q.root_test(c, d[off:off + n]) == want.tolist(), (off, n)


@pytest.mark.parametrize("d", [16, 21, 32, 48])
def test_root_test_u64_edge_ids(d):
    """u64 candidates at the edges of the representation (0, p - 1, p, p + 1,
    2^64 - 1 and neighbours, ids whose 22-bit limbs are all ones) as roots
    and as non-roots: the baby-step/giant-step kernel (d >= 16) works on the
    raw 64-bit id, its limb sums and folds must stay exact."""
    P = (1 << 64) - 59
    edge = [0, 1, 2, P - 2, P - 1, P, P + 1, P + 58, (1 << 64) - 1, (1 << 64) - 2, (1 << 44) - 1, (1 << 22) - 1,
            ((1 << 64) - 1) ^ (1 << 22), (1 << 63), (1 << 63) - 1]
    log = coracle.splitmix_u64(77 + d, 20_000)
    log[::1000] = np.array(edge * 2, dtype=np.uint64)[: len(log[::1000])]
    roots = [P - 1, (1 << 64) - 1, (1 << 44) - 1, 1] + [int(v) for v in log[3:3 + d - 4]]
    q = QT(64)(d)
    for r in roots:
        q.insert(r)
    c = q.to_coeffs()
    want, _ = coracle.root_test_u64(c, log)
    got = q.root_test(c, dev(log, 64))
    assert got == want.tolist()
    assert {i for i, v in enumerate(log.tolist()) if v % P in {r % P for r in roots}} == set(got)


def test_stop_at_last_value():
    log = coracle.splitmix_u32(44, 10_000)
    q = sk.PowerSumQuackU32(8)
    for i in (10, 20, 9000):
        q.insert(int(log[i]))
    c = q.to_coeffs()
    d = dev(log)
    assert q.root_test(c, d) == [10, 20, 9000]
    assert q.root_test(c, d, stop_value=int(log[500])) == [10, 20]
    assert q.root_test(c, d, stop_value=int(log[10])) == []
    assert q.root_test(c, d, stop_value=0xFFFFFFFF if 0xFFFFFFFF not in log else 1) == [10, 20, 9000]
    want = qo.root_test_indices(list(c), log.tolist(), qo.P32, stop_value=int(log[5000]))
    assert q.root_test(c, d, stop_value=int(log[5000])) == want


def test_root_test_shard_reports_stop_index():
    """qk_*_root_test_shard_device: the shard's hits (cut at its own stop)
    plus the position of the first stop value (len when absent); d = 0 still
    reports the stop.  Duplicated stop value -> first occurrence."""
    log = coracle.splitmix_u32(45, 20_000)
    log[7000] = log[3000]
    q = sk.PowerSumQuackU32(8)
    for i in (10, 5000, 15000):
        q.insert(int(log[i]))
    c = q.to_coeffs()
    d = dev(log)
    assert q.root_test_shard(c, d) == ([10, 5000, 15000], len(log))
    assert q.root_test_shard(c, d, stop_value=int(log[3000])) == ([10], 3000)
    absent = next(v for v in range(1, 100) if v not in set(log.tolist()))
    assert q.root_test_shard(c, d, stop_value=absent) == ([10, 5000, 15000], len(log))
    assert q.root_test_shard([], d, stop_value=int(log[12345])) == ([], 12345)
    assert q.root_test_shard([], d) == ([], len(log))
    log64 = coracle.splitmix_u64(46, 5000)
    q64 = sk.PowerSumQuackU64(4)
    q64.insert(int(log64[100]))
    assert q64.root_test_shard(q64.to_coeffs(), dev(log64, 64), stop_value=int(log64[4000])) == ([100], 4000)


def test_many_hits_capacity_growth():
    # a log made mostly of roots: > the 4096 default device hit capacity
    roots = coracle.splitmix_u32(8, 4)
    log = np.tile(roots, 5000)
    log[::7] = 12345
    q = sk.PowerSumQuackU32(4)
    for r in roots.tolist():
        q.insert(r)
    c = q.to_coeffs()
    got = q.root_test(c, dev(log), cap=16)
    want, _ = coracle.root_test_u32(c, log, cap=1 << 20)
    assert got == want.tolist() and len(got) > 16000


@pytest.mark.parametrize("nhit", [1003, 1004, 1005, 1100])
def test_hit_and_stop_slot_boundaries(nhit):
    """The root-set scan writes its hits and stops straight into pinned host
    slots (1004 hit slots, 16 stop slots; a slot past either falls back to
    the device counters): hit counts around the hit slots' end, and a stop
    value occurring 40 times (its first occurrence must win), against the
    oracle."""
    rng = np.random.default_rng(nhit)
    roots = [0x1234567, 0x7654321]
    log = rng.integers(0, 1 << 32, size=200_000, dtype=np.uint64).astype(np.uint32)
    log[np.isin(log, roots)] = 5
    pos = np.sort(rng.choice(len(log), size=nhit, replace=False))
    log[pos] = np.array(roots, dtype=np.uint32)[np.arange(nhit) % 2]
    q = sk.PowerSumQuackU32(4)
    for r in roots:
        q.insert(r)
    c = q.to_coeffs()
    d = dev(log)
    got = q.root_test(c, d)
    assert got == pos.tolist()
    stop_value = 0xABCDEF
    log2 = log.copy()
    log2[log2 == stop_value] = 6
    spos = np.sort(rng.choice(np.setdiff1d(np.arange(len(log)), pos), size=40, replace=False))
    log2[spos] = stop_value
    want = qo.root_test_indices(list(c), log2.tolist(), qo.P32, stop_value=stop_value)
    assert want == [p for p in pos.tolist() if p < spos[0]]
    assert q.root_test(c, dev(log2), stop_value=stop_value) == want
    assert q.root_test_shard(c, dev(log2), stop_value=stop_value) == (want, int(spos[0]))


@pytest.mark.parametrize("bits", [32, 64])
def test_scan_completion_mark_grids(bits):
    """The kernel-argument scan's completion mark (decode.hip k_root_scan_k:
    per-group tickets, then a ticket of the groups) at grids below, at and
    above the group count, uneven groups included, and back-to-back calls
    with alternating grids (each last taker resets its ticket): every call's
    hits equal the log positions of the roots."""
    import sidekick_amd as skm
    ctx = skm.get_context(0)
    rng = np.random.default_rng(91 + bits)
    n = 1_000_003
    dt = np.uint32 if bits == 32 else np.uint64
    log = rng.integers(0, 1 << bits, size=n, dtype=np.uint64).astype(dt)
    roots = [int(r) for r in rng.integers(1, 1 << (bits - 1), size=5)]
    log[np.isin(log, np.array(roots, dtype=dt))] = 3
    pos = np.sort(rng.choice(n, size=23, replace=False))
    log[pos] = np.array(roots, dtype=dt)[np.arange(23) % 5]
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    q = Q(8)
    for r in roots:
        q.insert(r)
    c = q.to_coeffs()
    d_log = dev(log, bits)
    want = pos.tolist()
    try:
        for grid in (1, 5, 31, 32, 33, 100, 977, 0, 7, 0, 64, 1):
            ctx.set_grid(grid)
            for _ in range(2):
                assert q.root_test(c, d_log) == want, grid
    finally:
        ctx.set_grid(0)


def test_scan_completion_mark_many_calls():
    """Two hundred back-to-back kernel-argument scans over one resident log,
    each with another root set (1-40 roots drawn from the log, so the hits
    move across the whole grid every call): every hit list equals the log
    positions of its roots (numpy), i.e. no call reads its pinned slots
    before the workgroups that found hits wrote them."""
    rng = np.random.default_rng(2026)
    n = 2_000_003
    log = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    d_log = dev(log)
    for it in range(200):
        k = int(rng.integers(1, 41))
        roots = np.unique(log[rng.choice(n, size=k, replace=False)])
        q = sk.PowerSumQuackU32(len(roots))
        for r in roots.tolist():
            q.insert(int(r))
        want = np.flatnonzero(np.isin(log, roots)).tolist()
        assert q.root_test(q.to_coeffs(), d_log) == want, it

def test_scan_kernel_args_tickets_run_on(root_test_mode):
    """The root-set scan with its set in the kernel arguments keeps its hit
    and stop tickets running across calls (no reset in front of the scan):
    a sequence of decodes with different hit and stop counts, interleaved
    with encodes (which write the context's small buffer), a Horner call, a
    shard call, a call past the hit slots (the two-phase rerun, which
    invalidates the running tickets) and a stop value past the stop slots,
    every one against the oracle; knob rt_karg = 0 (the set by copy) gives
    the same lists."""
    import sidekick_amd as skm
    ctx = skm.get_context(0)
    results = {}
    for karg in (1, 0):
        rng = np.random.default_rng(77)   # the same sequence of cases for both forms
        base = rng.integers(0, 1 << 32, size=300_000, dtype=np.uint64).astype(np.uint32)
        ctx.set_knob("rt_karg", karg)
        try:
            out = []
            for it, (nhit, nstop) in enumerate(((3, 0), (40, 2), (1, 1), (1100, 0), (7, 0), (20, 30), (5, 1),
                                                 (2, 17), (9, 0))):
                roots = [int(r) for r in rng.integers(1, 1 << 31, size=3)]
                log = base.copy()
                log[np.isin(log, roots)] = 11
                pos = np.sort(rng.choice(len(log), size=nhit, replace=False))
                log[pos] = np.array(roots, dtype=np.uint32)[np.arange(nhit) % 3]
                q = sk.PowerSumQuackU32(8)
                for r in roots:
                    q.insert(r)
                c = q.to_coeffs()
                stop_value = None
                if nstop:
                    stop_value = 0xFEEDBEE
                    log[log == stop_value] = 12
                    free = np.setdiff1d(np.arange(len(log)), pos)
                    log[np.sort(rng.choice(free, size=nstop, replace=False))] = stop_value
                want = qo.root_test_indices(list(c), log.tolist(), qo.P32, stop_value=stop_value)
                got = q.root_test(c, dev(log), stop_value=stop_value)
                assert got == want, (karg, it, nhit, nstop)
                out.append(got)
                if it == 2:   # an encode through the same context (its partial goes to the small buffer)
                    e = sk.PowerSumQuackU32(16)
                    e.insert_batch(dev(log[:5000]))
                    assert e.power_sums() == coracle.encode_u32(log[:5000], 16)
                if it == 4:
                    got2, _ = q.root_test_shard(c, dev(log), stop_value=stop_value)
                    assert got2 == want
            results[karg] = out
        finally:
            ctx.set_knob("rt_karg", 1)
    assert results[1] == results[0]


@pytest.mark.parametrize("off,n", [(1, 100_007), (2, 100_000), (3, 5), (0, 17)])
def test_scan_ragged_and_misaligned(off, n, root_test_mode):
    """The root test over a log starting 0-3 entries past a 16-byte boundary
    with ragged lengths (head, body of 16-byte loads, tail), both widths,
    against the oracle."""
    for bits in (32, 64):
        log = (coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64)(90 + off + bits, n + off)
        q = QT(bits)(16)
        for i in sorted({0, 1, n // 7, n // 2, n - 1}):
            q.insert(int(log[off + i]))
        c = q.to_coeffs()
        d = dev(log, bits)[off:]
        want = qo.root_test_indices(list(c), log[off:].tolist(), qo.P32 if bits == 32 else qo.P64)
        assert q.root_test(c, d) == want


def test_undecodable_and_empty():
    q = sk.PowerSumQuackU32(4)
    assert q.decode_with_log(dev(np.arange(10, dtype=np.uint32))) == []
    for i in range(1, 6):
        q.insert(i)
    with pytest.raises(sk.UndecodableError):
        q.decode_with_log(dev(np.arange(10, dtype=np.uint32)))


def test_config5_full_size():
    """configs[4]: two quACKs built from 1e8 u32 ids, 32 dropped; recover them
    by the GPU root test against the full candidate log.  Expected hits are
    every position whose id is congruent to a dropped id (duplicates
    included), computed independently with numpy set membership."""
    n, t, seed = 100_000_000, 32, 0x5EED0005
    ctx = sk.get_context(0)
    log = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_splitmix(ctx, log, seed)
    rng = np.random.default_rng(seed)
    drops = np.sort(rng.choice(n, size=32, replace=False))
    keep = torch.ones(n, dtype=torch.bool, device=DEV)
    keep[torch.from_numpy(drops).to(DEV)] = False
    sent, recv = sk.PowerSumQuackU32(t), sk.PowerSumQuackU32(t)
    sent.insert_batch(log)
    recv.insert_batch(log[keep].contiguous())
    diff = sent.clone()
    diff.sub_assign(recv)
    assert diff.count() == 32
    hits = diff.root_test(diff.to_coeffs(), log)
    h = log.cpu().numpy().view(np.uint32).astype(np.uint64)
    p = np.uint64(qo.P32)
    dropped_vals = np.unique(h[drops] % p)
    want = np.nonzero(np.isin(h % p, dropped_vals))[0].tolist()
    assert hits == want
    assert set(drops.tolist()) <= set(hits)
