"""Every kernel variant the dispatcher can select, checked against the oracle.

The measurement knobs of a context (qk_ctx_set_knob): bsgs_sg
— how many 4-wide BSGS accumulator groups (the a = 0 add row first, then the
multiply-accumulate rows) count their wraps on the scalar unit; u32_xcache —
the per-id x^base cache of the u32 offset passes (u64_xcache: of the u64
ones); u64_kmax —
u64 accumulators per lane; bsgs64_sg — the u64 BSGS MAC carry mode;
bsgs64_off — the u64 power chain.  Each variant runs on the shared context of
device 0 with the knob set and restored afterwards.  Inputs cover ragged
tails (lanes with fewer iterations than their wave), an unaligned head, and
ids that force the rare lazy-fold wrap branch."""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DEFAULTS = {"bsgs_sg": -1, "u64_kmax": 40, "bsgs64_sg": -1, "bsgs64_off": 0, "bsgs64_tmin": 14, "bsgs64_shapes": 1, "u32_xcache": 1, "u64_xcache": 1,
            "bsgs_shapes": 1, "bsgs_prio": 1, "bsgs64_prio": 1, "grid_mult": 3}


@contextlib.contextmanager
def knob(name, value, grid=0):
    import sidekick_amd as sk
    ctx = sk.get_context(0)
    ctx.set_knob(name, value)
    ctx.set_grid(grid)
    try:
        yield
    finally:
        ctx.set_knob(name, DEFAULTS[name])
        ctx.set_grid(0)


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


U32_CASES = [("t32_ragged", 1_000_003, 32, 1), ("t32_small", 77, 32, 3), ("t24", 500_001, 24, 2),
             ("t16", 300_007, 16, 0), ("t12", 200_003, 12, 1), ("t30", 2_000_000, 30, 0)]


@pytest.mark.parametrize("sg", [0, 1, 2, 3, 5, 8])
def test_bsgs_scalar_carry_groups(sg):
    with knob("bsgs_sg", sg):
        res = _run(32, U32_CASES)
    assert all(res.values()), res


def test_bsgs_scalar_carry_small_grid():
    """Override grid of one workgroup: long per-wave trip counts."""
    with knob("bsgs_sg", 8, grid=1):
        res = _run(32, [("g1", 3_000_001, 32, 1)])
    assert all(res.values()), res


@pytest.mark.parametrize("kmax", [20, 40])
def test_u64_lane_split(kmax):
    cases = [("t80", 300_001, 80, 1), ("t40", 200_003, 40, 0), ("t33", 100_001, 33, 1), ("t20", 100_000, 20, 0),
             ("t64", 50_001, 64, 0), ("t200", 20_001, 200, 1)]
    with knob("u64_kmax", kmax):
        res = _run(64, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("sg", [-1, 8, 12, 14, 16, 18])
def test_u64_bsgs_scalar_carry_macs(sg):
    """The u64 baby-step/giant-step kernel (bsgs64.h) with the first sg MACs
    of each wave's tile counting carries on the scalar unit, the rest per
    lane; t = 73..80 (the last giant row partly or fully used)."""
    cases = [("t80", 300_001, 80, 1), ("t73", 100_003, 73, 0), ("t77", 4099, 77, 1), ("t79_tiny", 37, 79, 0)]
    with knob("bsgs64_sg", sg):
        res = _run(64, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("shapes", [1, 0])
def test_u32_bsgs_shapes(shapes):
    """The round-3 (NB, NA) shapes — (4,5..7) for t 17..28, (6,5) 29..30,
    (6,6) 33..36, (6,7) 41..42, (8,9) 65..72 — and the round-2 ones they
    replaced (knob bsgs_shapes = 0), against the oracle at both ends of each
    range, ragged and misaligned."""
    cases = [(f"t{t}", 100_003 + t, t, t % 4) for t in (17, 20, 21, 24, 25, 28, 29, 30, 33, 36, 41, 42, 65, 72)]
    with knob("bsgs_shapes", shapes):
        res = _run(32, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("prio", [1, 0])
def test_u32_bsgs_prio(prio):
    """Every single-pass u32 BSGS shape and the multi-pass kernels (pass 0 with
    x^80 out, offset passes with and without the x^base cache, a one-row last
    pass) with and without s_setprio around the MAC phase (knob bsgs_prio;
    the default raises it), against the oracle, ragged and misaligned."""
    cases = [(f"t{t}", 100_003 + t, t, t % 4)
             for t in (8, 12, 16, 20, 24, 28, 30, 32, 36, 40, 42, 48, 56, 64, 72, 80, 88, 129, 300)]
    with knob("bsgs_prio", prio):
        res = _run(32, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("prio", [1, 0])
def test_u64_bsgs_prio(prio):
    """u64 baby-step/giant-step with s_setprio in the MAC step and paired
    MACs (knob bsgs64_prio, the default) and in the round-3 form, against the
    oracle: eight- and four-baby shapes, pass 0 with x^80 out, offset passes,
    a one-row last pass."""
    cases = [(f"t{t}", 40_009 + t, t, t % 2) for t in (14, 16, 20, 24, 32, 40, 56, 72, 80, 88, 169, 250)]
    with knob("bsgs64_prio", prio):
        res = _run(64, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("xcache", [1, 0])
def test_u32_passes_xbase_cache(xcache):
    """u32 thresholds > 128 run two or more offset passes; with the per-id
    x^base cache (the default) pass 1 writes x^128 per id, the middle passes
    read and write it, the last one reads it — against the oracle with an
    unaligned head, ragged tails, a partial last pass (t = 129, 250, 300; one
    giant row at t = 81, 88, 129, 136) and
    the 20-pass maximum (t = 1024); knob u32_xcache = 0 is the
    square-and-multiply form."""
    cases = [("t129", 300_001, 129, 1), ("t81", 70_001, 81, 2), ("t88", 50_021, 88, 0), ("t136", 30_011, 136, 1),
             ("t176", 100_003, 176, 3), ("t250", 65_537, 250, 2), ("t300", 40_009, 300, 0),
             ("t1024", 20_011, 1024, 1), ("t1024_tiny", 9, 1024, 3)]
    with knob("u32_xcache", xcache):
        res = _run(32, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("xcache", [1, 0])
def test_u64_passes_xbase_cache(xcache):
    """u64 thresholds > 160: offset passes of 80 powers hand x^(next base)
    on through the per-id cache (knob u64_xcache; 0 = square-and-multiply per
    pass): a partial last pass (t = 161, 250; one giant row at t = 81, 88, 161), full passes only (t = 240) and
    the 13-pass maximum (t = 1024), with ragged tails and a head offset."""
    cases = [("t161", 100_003, 161, 1), ("t81", 70_001, 81, 0), ("t88", 60_013, 88, 1), ("t89", 20_011, 89, 1),
             ("t240", 50_001, 240, 0), ("t250", 30_011, 250, 2), ("t1024", 8_009, 1024, 1),
             ("t1024_tiny", 5, 1024, 0)]
    with knob("u64_xcache", xcache):
        res = _run(64, cases)
    assert all(res.values()), res


def test_u64_bsgs_off_matches_chain():
    """The power-chain path the u64 BSGS kernel replaced gives the same sums."""
    with knob("bsgs64_off", 1):
        res = _run(64, [("t80", 200_001, 80, 1), ("t75", 3001, 75, 0)])
    assert all(res.values()), res


@pytest.mark.parametrize("tmin", [9, 81])
def test_u64_bsgs_small_thresholds(tmin):
    """u64 t = 9..20 on the baby-step/giant-step kernel (NA = 2, 3; knob
    bsgs64_tmin = 9) and on the power chain (81), against the oracle."""
    cases = [(f"t{t}", 50_003 + t, t, t % 2) for t in (9, 12, 13, 14, 16, 17, 20, 21)]
    with knob("bsgs64_tmin", tmin):
        res = _run(64, cases)
    assert all(res.values()), res


@pytest.mark.parametrize("shapes", [1, 0])
def test_u64_bsgs_four_babies(shapes):
    """u64 t = 14..20, 25..28, 33..36 with four babies per id and ceil(t/4)
    giant rows (one baby per wave) and with the 8-baby kernel it replaced
    (knob bsgs64_shapes = 0), against the oracle at both ends of each range
    and at the thresholds that stay on 8 babies."""
    cases = [(f"t{t}", 40_009 + t, t, t % 2) for t in (14, 16, 17, 20, 21, 24, 25, 28, 32, 33, 36, 37, 40, 41)]
    with knob("bsgs64_shapes", shapes):
        res = _run(64, cases)
    assert all(res.values()), res


def test_knob_validation():
    import sidekick_amd as sk
    from sidekick_amd._lib import QuackError
    ctx = sk.get_context(0)
    for name, bad in (("flow_load", 0), ("flow_load", 65), ("root_test", 3), ("no_such_knob", 1),
                      ("matrix_cores", 1), ("flow_sort", 10), ("flow_sort", 0), ("comm_fault", -1), ("bsgs_prio", 2), ("bsgs64_prio", 2),
                      ("grid_mult", 0), ("grid_mult", 9)):
        with pytest.raises(QuackError):
            ctx.set_knob(name, bad)


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


@pytest.mark.parametrize("prio", [1, 0])
def test_passes_prio_saturated_grid(prio):
    """Multi-pass encodes (t > 80) with the x^base cache, on streams long
    enough that every pass launches the capped grid (u32: > 256 CUs x 8 x 256
    threads x 4 ids; u64: > 256 CUs x 8 x 3 rounds of 256-id tiles), for both
    wave-priority instantiations: the cache placed after the partials must
    not overlap the partials of whichever kernel the knobs select."""
    with knob("bsgs_prio", prio):
        res = _run_tiled(32, [("u32_t100", 100_003, 42, 100), ("u32_t200", 100_003, 42, 200)])
    with knob("bsgs64_prio", prio):
        res.update(_run_tiled(64, [("u64_t100", 50_021, 70, 100), ("u64_t200", 50_021, 70, 200)]))
    assert all(res.values()), res


@pytest.mark.parametrize("mult", [1, 3, 8])
def test_encode_grid_mult_saturated(mult):
    """Grid rounds 1 / 3 / 8 on streams above the resident-workgroup count at
    every multiplier (u32 t = 32: 1280 x 8 workgroups of 1024 ids; u64 t = 80
    and 100: 1024 x 8 tiles of 256 ids), so each multiplier really changes
    the grid — against the tiled oracle blocks."""
    with knob("grid_mult", mult):
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
    with knob("grid_mult", mult):
        res = _run(32, c32)
        res.update({f"u64_{k}": v for k, v in _run(64, c64).items()})
    assert all(res.values()), res
