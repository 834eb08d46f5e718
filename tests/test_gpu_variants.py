"""Every encode kernel the dispatcher can select (encode.hip enc32 / enc64),
checked against the oracle.

The dispatch is fixed by (bits, t, grid): u32 baby-step/giant-step shapes for
5 <= t <= 80, offset passes with the per-id x^base cache above 80, the power
chain below 5 (and for t 33..80 on a grid too small for scalar wrap counts);
u64 four- and eight-baby shapes for 14 <= t <= 80, passes above, the chain
below 14.  (Round 6 removed the knobs that selected the measured-and-rejected
variants — the round-2 shapes, the forms without s_setprio, the passes
without the cache, other carry modes)  Inputs cover ragged
tails (lanes with fewer iterations than their wave), an unaligned head, and
streams long enough to saturate the grid cap; the knob left, grid_mult, and
the grid override are exercised too."""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def grid(blocks=0, mult=None):
    import sidekick_amd as sk
    ctx = sk.get_context(0)
    ctx.set_grid(blocks)
    if mult is not None:
        ctx.set_knob("grid_mult", mult)
    try:
        yield
    finally:
        ctx.set_grid(0)
        ctx.set_knob("grid_mult", 3)


def _run(bits, cases):
    import torch
    import sidekick_amd as sk
    from oracle import coracle
    out = {}
    for name, n, t, off in cases:
        if bits == 32:
            ids = coracle.splitmix_u32(0xA11 + n, n + off)
            q = sk.PowerSumQuackU32(t)
            q.insert_batch(torch.from_numpy(ids.view(np.int32)).cuda()[off:])
            want = coracle.encode_u32(ids[off:], t)
        else:
            ids = coracle.splitmix_u64(0xA12 + n, n + off)
            q = sk.PowerSumQuackU64(t)
            q.insert_batch(torch.from_numpy(ids.view(np.int64)).cuda()[off:])
            want = coracle.encode_u64(ids[off:], t)
        out[name] = (q.power_sums() == list(want)) and q.count() == n
    return out


def test_u32_every_bsgs_shape():
    """Both ends of every u32 shape's range — (4,2) 5..8, (4,3) 9..12, (4,4)
    13..16, (4,5..7) 17..28, (6,5) 29..30, (8,4) 31..32, (6,6) 33..36, (8,5)
    37..40, (6,7) 41..42, (8,6..8) 43..64, (8,9) 65..72, (8,10) 73..80 — and
    the chain below, ragged and misaligned."""
    ts = (1, 4, 5, 8, 9, 12, 13, 16, 17, 20, 21, 24, 25, 28, 29, 30, 31, 32, 33, 36, 37, 40, 41, 42, 43, 48, 49, 56,
          57, 64, 65, 72, 73, 80)
    res = _run(32, [(f"t{t}", 100_003 + t, t, t % 4) for t in ts])
    assert all(res.values()), res


def test_u32_headline_shapes_ragged():
    cases = [("t32_ragged", 1_000_003, 32, 1), ("t32_small", 77, 32, 3), ("t24", 500_001, 24, 2),
             ("t16", 300_007, 16, 0), ("t12", 200_003, 12, 1), ("t30", 2_000_000, 30, 0)]
    assert all(_run(32, cases).values())


def test_u32_small_grid():
    """Override grid of one workgroup: long per-wave trip counts."""
    with grid(1):
        res = _run(32, [("g1", 3_000_001, 32, 1), ("g1_t80", 400_001, 80, 2), ("g1_t12", 200_003, 12, 3)])
    assert all(res.values()), res


def test_u32_passes_xbase_cache():
    """u32 thresholds > 80 run offset passes; pass 0 writes x^80 per id, the
    middle passes read and write it, the last one reads it — against the
    oracle with an unaligned head, ragged tails, a partial last pass (t =
    129, 250, 300; one giant row at t = 81, 88, 129, 136) and the 20-pass
    maximum (t = 1024)."""
    cases = [("t129", 300_001, 129, 1), ("t81", 70_001, 81, 2), ("t88", 50_021, 88, 0), ("t136", 30_011, 136, 1),
             ("t176", 100_003, 176, 3), ("t250", 65_537, 250, 2), ("t300", 40_009, 300, 0),
             ("t1024", 20_011, 1024, 1), ("t1024_tiny", 9, 1024, 3)]
    res = _run(32, cases)
    assert all(res.values()), res


def test_u64_every_shape():
    """u64: the chain (t < 14), four babies (t 14..20, 25..28, 33..36), eight
    babies (21..24, 29..32, 37..80, the last giant row partly or fully used at
    73..80), against the oracle at both ends of each range."""
    ts = (1, 8, 9, 12, 13, 14, 16, 17, 20, 21, 24, 25, 28, 29, 32, 33, 36, 37, 40, 41, 48, 56, 64, 72, 73, 77, 79, 80)
    res = _run(64, [(f"t{t}", 40_009 + t, t, t % 2) for t in ts])
    assert all(res.values()), res


def test_u64_t80_ragged():
    cases = [("t80", 300_001, 80, 1), ("t73", 100_003, 73, 0), ("t77", 4099, 77, 1), ("t79_tiny", 37, 79, 0)]
    assert all(_run(64, cases).values())


def test_u64_passes_xbase_cache():
    """u64 thresholds > 80: offset passes of 80 powers hand x^(next base) on
    through the per-id cache: a partial last pass (t = 161, 250; one giant row
    at t = 81, 88, 161), full passes only (t = 240) and the 13-pass maximum
    (t = 1024), with ragged tails and a head offset."""
    cases = [("t161", 100_003, 161, 1), ("t81", 70_001, 81, 0), ("t88", 60_013, 88, 1), ("t89", 20_011, 89, 1),
             ("t240", 50_001, 240, 0), ("t250", 30_011, 250, 2), ("t1024", 8_009, 1024, 1),
             ("t1024_tiny", 5, 1024, 0)]
    res = _run(64, cases)
    assert all(res.values()), res


def test_knob_validation():
    """The knobs left select live product paths; the removed ones (round 6)
    and out-of-range values are rejected."""
    import sidekick_amd as sk
    from sidekick_amd._lib import QuackError
    ctx = sk.get_context(0)
    for name, bad in (("root_test", 3), ("no_such_knob", 1), ("flow_byslot", 3), ("comm_fault", -1),
                      ("grid_mult", 0), ("grid_mult", 9), ("flow_hist", -1),
                      ("flow_sort", 2), ("flow_pipe", 0), ("bsgs_prio", 1), ("bsgs64_sg", 14), ("rt_direct", 1),
                      ("rt_scan_u", 1), ("pkt_fused", 1), ("u64_kmax", 40)):
        with pytest.raises(QuackError):
            ctx.set_knob(name, bad)
    for name, good in (("grid_mult", 3), ("flow_hist", 32), ("flow_byslot", 0), ("root_test", 0), ("comm_fault", 0)):
        ctx.set_knob(name, good)


P32, P64 = 4294967291, 18446744073709551557


def _run_tiled(bits, cases):
    """Streams long enough to saturate the grid cap: one oracle-encoded block
    of m ids tiled R times on the device, so the expected sums are R * S_block
    mod p exactly (the oracle stays cheap at millions of ids)."""
    import sidekick_amd as sk
    import torch
    from oracle import coracle
    out = {}
    for name, m, R, t in cases:
        if bits == 32:
            blk = coracle.splitmix_u32(0xB1 + m + t, m)
            want = coracle.encode_u32(blk, t)
            big = torch.from_numpy(blk.view(np.int32)).cuda().repeat(R)
            q, p = sk.PowerSumQuackU32(t), P32
        else:
            blk = coracle.splitmix_u64(0xB2 + m + t, m)
            want = coracle.encode_u64(blk, t)
            big = torch.from_numpy(blk.view(np.int64)).cuda().repeat(R)
            q, p = sk.PowerSumQuackU64(t), P64
        q.insert_batch(big)
        out[name] = q.power_sums() == [(R * int(s)) % p for s in want] and q.count() == m * R \
            and q.last_value() == int(blk[-1])
        del big
    return out


def test_passes_saturated_grid():
    """Multi-pass encodes (t > 80) with the x^base cache, on streams long
    enough that every pass launches the capped grid (u32: > 256 CUs x 8 x 256
    threads x 4 ids; u64: > 256 CUs x 8 x 3 rounds of 256-id tiles): the cache
    placed after the partials (grid_cap: the device's resident workgroups per
    CU) must not overlap them."""
    res = _run_tiled(32, [("u32_t100", 100_003, 42, 100), ("u32_t200", 100_003, 42, 200)])
    res.update(_run_tiled(64, [("u64_t100", 50_021, 70, 100), ("u64_t200", 50_021, 70, 200)]))
    assert all(res.values()), res


@pytest.mark.parametrize("mult", [1, 3, 8])
def test_encode_grid_mult_saturated(mult):
    """Grid rounds 1 / 3 / 8 on streams above the resident-workgroup count at
    every multiplier (u32 t = 32: 1280 x 8 workgroups of 1024 ids; u64 t = 80
    and 100: 1024 x 8 tiles of 256 ids), so each multiplier really changes
    the grid — against the tiled oracle blocks."""
    with grid(0, mult):
        res = _run_tiled(32, [("u32_t32", 1_000_003, 12, 32), ("u32_t129", 1_000_003, 12, 129)])
        res.update(_run_tiled(64, [("u64_t80", 300_007, 10, 80), ("u64_t100", 300_007, 10, 100)]))
    assert all(res.values()), res


@pytest.mark.parametrize("mult", [1, 3, 8])
def test_encode_grid_mult(mult):
    """Encode grids of 1, 3 (the default) and 8 rounds of resident workgroups
    (knob grid_mult): shorter contiguous runs per workgroup, more partials —
    u32 and u64, single-pass and passes, against the oracle."""
    c32 = [(f"t{t}", 1_000_003 + t, t, t % 4) for t in (8, 16, 28, 32, 48, 80, 129)]
    c64 = [(f"t{t}", 200_003 + t, t, t % 2) for t in (8, 16, 32, 80, 100)]
    with grid(0, mult):
        res = _run(32, c32)
        res.update({f"u64_{k}": v for k, v in _run(64, c64).items()})
    assert all(res.values()), res
