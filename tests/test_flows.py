"""Segmented multi-flow encode vs the oracle's
literal SidekickMulti restatement (sidekick_multi.rs:65-90,101-143)."""
import numpy as np
import pytest

from oracle import coracle, quack_oracle as qo

MY_ADDR = (10, 0, 2, 1, 0x1F, 0x90)   # own dst ip:port (6 bytes)
META_DT = np.dtype([("pkttype", "u1"), ("reserved", "u1"), ("protocol_be", "<u2"), ("len", "<u4")])


def make_flows(n, nflows, seed, stride=67, p_filter=0.1, p_reset=0.01, skew=False, flows=None, reset_until=0.5):
    """n records over nflows AddrKeys; resets (packets to MY_ADDR) only in the
    first reset_until fraction, so the flows after the last reset — the only
    ones a Reset leaves (sidekick_multi.rs:205,265) — hold most packets."""
    rng = np.random.default_rng(seed)
    bufs = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
    bufs[:, 23] = 17
    if flows is None:
        flows = rng.integers(0, 256, size=(nflows, 12), dtype=np.uint8)
        flows[:, 6:12] = (192, 168, 0, 9, 0x11, 0x5C)   # dst side differs from MY_ADDR ...
        flows[: nflows // 2, 9] = rng.integers(0, 256, size=nflows // 2)  # ... and varies for half the flows
    nflows = len(flows)
    if skew:
        f = np.minimum(rng.zipf(1.5, size=n) - 1, nflows - 1)
    else:
        f = rng.integers(0, nflows, size=n)
    key = flows[f]
    bufs[:, 26:30] = key[:, 0:4]
    bufs[:, 34:36] = key[:, 4:6]
    bufs[:, 30:34] = key[:, 6:10]
    bufs[:, 36:38] = key[:, 10:12]
    r = rng.random(n)
    rs = (r < p_reset) & (np.arange(n) < int(reset_until * n))
    bufs[rs, 30:34] = MY_ADDR[:4]
    bufs[rs, 36:38] = MY_ADDR[4:]
    meta = np.zeros(n, dtype=META_DT)
    meta["protocol_be"] = 0x0008
    meta["len"] = 67
    k = (r >= p_reset) & (r < p_reset + p_filter)
    kind = rng.integers(0, 4, size=n)
    meta["pkttype"][k & (kind == 0)] = 4
    meta["protocol_be"][k & (kind == 1)] = 0xDD86
    bufs[k & (kind == 2), 23] = 6
    meta["len"][k & (kind == 3)] = 40
    return bufs, meta


def vector_flows(bufs, meta, my_addr=MY_ADDR):
    """Vectorised SidekickMulti sniff loop (checked against the oracle below):
    ({key: ids in packet order after the last reset}, resets, last reset
    position or -1)."""
    inc = (meta["pkttype"] == 0) | (meta["pkttype"] == 3)
    ok = inc & (meta["protocol_be"] == 0x0008) & (bufs[:, 23] == 17)
    keys = np.concatenate([bufs[:, 26:30], bufs[:, 34:36], bufs[:, 30:34], bufs[:, 36:38]], axis=1)
    rst = ok & np.all(keys[:, 6:12] == np.array(my_addr, dtype=np.uint8), axis=1) if my_addr else np.zeros(len(bufs), bool)
    ins = ok & ~rst & (meta["len"] == 67)
    last_reset = int(np.nonzero(rst)[0][-1]) if rst.any() else -1
    idb = bufs[:, 63:67].astype(np.uint32)
    ids = (idb[:, 0] << 24) | (idb[:, 1] << 16) | (idb[:, 2] << 8) | idb[:, 3]
    out = {}
    for i in np.nonzero(ins[last_reset + 1:])[0] + last_reset + 1:
        out.setdefault(bytes(keys[i]), []).append(int(ids[i]))
    return out, int(rst.sum()), last_reset


@pytest.mark.parametrize("reset_until", [0.0, 0.5, 1.0])
def test_vector_flows_matches_oracle(reset_until):
    bufs, meta = make_flows(3000, 7, seed=1, p_reset=0.05, p_filter=0.2, reset_until=reset_until)
    pre = qo.OracleQuack(8)
    pre.insert(7)
    table = {b"\x01" * 12: pre}            # the caller's table before the batch
    table, st = qo.sniff_multi_batch(table, 8, bufs, meta["pkttype"], meta["protocol_be"], meta["len"], MY_ADDR)
    flows, nres, last_reset = vector_flows(bufs, meta)
    assert st["resets"] == nres and st["last_reset_index"] == last_reset
    assert st["inserted"] == sum(len(v) for v in flows.values())
    if nres:                                 # a Reset wiped the caller's flow too
        assert set(table) == set(flows)
    else:
        assert set(table) == set(flows) | {b"\x01" * 12}
    for k, ids in flows.items():
        w = qo.OracleQuack(8)
        w.insert_all(ids)
        assert table[k].power_sums == w.power_sums and table[k].count == len(ids) and table[k].last_value == ids[-1]


def test_sniff_multi_reset_wipes_every_flow():
    """sidekick_multi.rs:205: a Reset packet replaces the whole map, so a flow
    whose packets all came before it is gone, and a flow seen on both sides
    restarts from the packets after it."""
    bufs, meta = make_flows(40, 2, seed=5, p_reset=0.0, p_filter=0.0)
    k0, k1 = sorted({qo.addr_key(b) for b in bufs})
    bufs[20, 30:34] = MY_ADDR[:4]
    bufs[20, 36:38] = MY_ADDR[4:]
    table, st = qo.sniff_multi_batch({}, 4, bufs, meta["pkttype"], meta["protocol_be"], meta["len"], MY_ADDR)
    assert st["resets"] == 1 and st["last_reset_index"] == 20
    after = {}
    for b in bufs[21:]:
        after.setdefault(qo.addr_key(b), []).append(int.from_bytes(bytes(b[63:67]), "big"))
    assert set(table) == set(after) and st["inserted"] == 19 and st["discarded"] == 20
    for k, ids in after.items():
        assert table[k].count == len(ids) and table[k].last_value == ids[-1]


@pytest.mark.gpu
@pytest.mark.parametrize("n,nflows,t,skew", [(1, 1, 32, False), (1000, 3, 32, False), (70_000, 40, 16, False),
                                             (200_000, 5000, 32, False), (300_000, 64, 80, True),
                                             (150_000, 2, 20, False)])
def test_gpu_flows_vs_oracle(n, nflows, t, skew):
    import torch
    import sidekick_amd as sk
    bufs, meta = make_flows(n, nflows, seed=n + t, skew=skew, reset_until=0.3 if n % 2 else 0.0)
    table = sk.FlowQuacks(t)
    pre_key = None
    flows, nres, last_reset = vector_flows(bufs, meta)
    if flows:                                # pre-existing entry merges with the batch (or is wiped by a reset)
        pre_key = sorted(flows)[0]
        table.insert(pre_key, 424242)
    st = table.insert_packets(torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67,
                              meta=torch.from_numpy(meta.view(np.int64).copy()).cuda(), my_addr=MY_ADDR)
    assert st["resets"] == nres and st["inserted"] == sum(len(v) for v in flows.values())
    assert st["last_reset_index"] == last_reset
    _, ost = qo.sniff_multi_batch({}, t, bufs[: min(n, 5000)], meta["pkttype"], meta["protocol_be"], meta["len"],
                                  MY_ADDR) if n <= 5000 else (None, None)
    if ost is not None:
        assert ost == st
    assert set(table.senders()) == set(flows)
    for k, ids in flows.items():
        q = table.senders()[k]
        want_ids = ([424242] if k == pre_key and nres == 0 else []) + ids
        assert q.power_sums() == coracle.encode_u32(np.array(want_ids, dtype=np.uint32), t), k.hex()
        assert q.count() == len(want_ids) and q.last_value() == ids[-1]


@pytest.mark.gpu
def test_gpu_segments_primitive():
    import torch
    from sidekick_amd.quack import encode_segments
    ids = coracle.splitmix_u32(0xF10, 400_000)
    offs = [0, 0, 1, 5, 70_000, 70_000, 200_003, 400_000]   # empty, tiny, > one 64 Ki work item
    qs = encode_segments(torch.from_numpy(ids.view(np.int32)).cuda(), offs, 32)
    assert len(qs) == len(offs) - 1
    for g, q in enumerate(qs):
        seg = ids[offs[g]:offs[g + 1]]
        assert q.power_sums() == coracle.encode_u32(seg, 32)
        assert q.count() == len(seg) and q.last_value() == (int(seg[-1]) if len(seg) else None)


@pytest.mark.gpu
@pytest.mark.parametrize("t", [1, 5, 8, 9, 12, 13, 16, 17, 24, 25, 32, 33, 40, 48, 56, 64, 65, 80, 81])
def test_gpu_many_small_segments(golden, t):
    """Lane-per-segment kernel (segments <= 4096 ids, t <= 32) beside the
    work-item path (longer segments, t > 32): thousands of ragged segments,
    the 4096/4097 boundary, and lazy-fold wrap ids inside short segments."""
    import torch
    from sidekick_amd.quack import encode_segments
    rng = np.random.default_rng(t)
    lens = rng.integers(0, 200, size=3000)
    lens[::97] = 0
    lens[5], lens[6], lens[7], lens[8] = 4096, 4097, 1, 70_000
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ids = coracle.splitmix_u32(0x5E6 + t, int(offs[-1]))
    cfg = ("4x2" if t <= 8 else "4x3" if t <= 12 else "4x4" if t <= 16 else "6x4" if t <= 24 else "8x4" if t <= 32
           else "8x5" if t <= 40 else "8x6" if t <= 48 else "8x7" if t <= 56 else "8x8" if t <= 64 else "8x10")
    wraps = np.array(golden["bsgs_wrap_ids"][cfg], dtype=np.uint32)
    for j, g in enumerate((10, 11, 5, 6, 2999)):     # first/middle/last id of a segment
        if lens[g]:
            ids[offs[g] + (j % 3) * (lens[g] - 1) // 2] = wraps[j % len(wraps)]
    qs = encode_segments(torch.from_numpy(ids.view(np.int32)).cuda(), offs.tolist(), t)
    assert len(qs) == len(lens)
    for g, q in enumerate(qs):
        seg = ids[offs[g]:offs[g + 1]]
        assert q.power_sums() == coracle.encode_u32(seg, t), (g, len(seg))
        assert q.count() == len(seg) and q.last_value() == (int(seg[-1]) if len(seg) else None)


@pytest.mark.gpu
@pytest.mark.parametrize("t", [16, 32])
def test_gpu_small_segments_misaligned_base(t):
    """The lane-per-segment kernel reads each segment in the 16-byte blocks
    that hold it (masked first/last block): a caller id array starting 4, 8
    or 12 bytes past a 16-byte boundary, segments of 0..40 ids."""
    import torch
    from sidekick_amd.quack import encode_segments
    rng = np.random.default_rng(100 + t)
    lens = rng.integers(0, 41, size=2000)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ids = coracle.splitmix_u32(0xA11 + t, int(offs[-1]) + 3)
    d = torch.from_numpy(ids.view(np.int32)).cuda()
    for off in (1, 2, 3):
        sub = ids[off:off + int(offs[-1])]
        qs = encode_segments(d[off:off + int(offs[-1])], offs.tolist(), t)
        for g, q in enumerate(qs):
            seg = sub[offs[g]:offs[g + 1]]
            assert q.power_sums() == coracle.encode_u32(seg, t), (off, g, len(seg))
            assert q.count() == len(seg) and q.last_value() == (int(seg[-1]) if len(seg) else None)


def check_flows_table(table, flows, t):
    assert set(table.senders()) == set(flows)
    for k, ids in flows.items():
        q = table.senders()[k]
        assert q.power_sums() == coracle.encode_u32(np.array(ids, dtype=np.uint32), t), k.hex()
        assert q.count() == len(ids) and q.last_value() == ids[-1]


@pytest.mark.gpu
def test_gpu_flows_edge_keys_and_table_growth():
    """AddrKeys at the ends of the key space (all-zero / all-0xFF halves, the
    table's packed-word edge cases), then a batch of 60 000 distinct flows
    right after a one-flow batch: the device flow table, sized from the
    previous batch, overflows its probe limit and is regrown."""
    import torch
    import sidekick_amd as sk
    rng = np.random.default_rng(99)
    flows = rng.integers(0, 256, size=(40, 12), dtype=np.uint8)
    flows[0] = 0xFF
    flows[1] = 0
    flows[2, :6], flows[2, 6:] = 0xFF, 0
    flows[3, :6], flows[3, 6:] = 0, 0xFF
    flows[4, :6], flows[4, 6:] = 0xFF, (0xFF, 0xFF, 0xFF, 0xFE, 0xFF, 0xFF)
    for n, fl in ((50_000, flows), (1000, flows[:1]), (400_000, None)):
        if fl is None:
            fl = rng.integers(0, 256, size=(60_000, 12), dtype=np.uint8)
        bufs, meta = make_flows(n, 0, seed=n, flows=fl, p_reset=0.0)
        want, _, _ = vector_flows(bufs, meta)
        table = sk.FlowQuacks(16)
        st = table.insert_packets(torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67,
                                  meta=torch.from_numpy(meta.view(np.int64).copy()).cuda(), my_addr=MY_ADDR)
        assert st["inserted"] == sum(len(v) for v in want.values())
        check_flows_table(table, want, 16)
        assert list(table.senders()) == sorted(want)     # the C ABI returns flows in ascending AddrKey order
        if fl is not flows and len(fl) > 1000:
            assert len(want) > 50_000


@pytest.mark.gpu
def test_gpu_flows_regrow_bail():
    """A batch of 60 000 flows on a fresh context (table from 4096 slots):
    the overflowing passes stop early (k_flow_extract's bail: a workgroup
    whose probe overflowed leaves, the others read the flag every 64th tile)
    and the batch reruns on regrown tables; the records must be the oracle's,
    also with resets (the rerun after the last reset), and byte for byte the
    records of the next batch on the same context (its table sized from this
    one's flows: no regrow)."""
    import torch
    from sidekick_amd.quack import Context, encode_flows
    bufs, meta = make_flows(400_000, 60_000, seed=77, p_reset=0.0005, reset_until=0.3)
    want, nres, _ = vector_flows(bufs, meta)
    d_bufs = torch.from_numpy(bufs.reshape(-1).copy()).cuda()
    d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda()
    ctx = Context(0)
    recs = []
    for call in range(2):
        keys, qs, st = encode_flows(d_bufs, 16, meta=d_meta, my_addr=MY_ADDR, ctx=ctx)
        assert st["resets"] == nres and keys == sorted(want)
        if call == 0:
            for k, q in zip(keys, qs):
                ids = want[k]
                assert q.count() == len(ids) and q.last_value() == ids[-1], k.hex()
                assert q.power_sums() == coracle.encode_u32(np.array(ids, dtype=np.uint32), 16), k.hex()
        recs.append([bytes(q._buf.raw) for q in qs])
    ctx.close()
    assert recs[0] == recs[1]


@pytest.mark.gpu
def test_gpu_flows_group_by_slot_and_by_rank():
    """The grouping sort keys the packets by table slot or by flow rank (a
    slot -> rank remap first); by rank is taken when it saves two 8-bit
    passes or leaves one (knob flow_byslot = 0), and flow_byslot = 1 / 2
    force either key.  Every mode must give the oracle's tables in ascending
    key order, and the records byte for byte alike: 10 000 flows (16 vs 14
    bits), 40 flows (12 vs 6 bits: by rank under the rule), 3 000 flows and
    30 000 flows (17 vs 15 bits: by slot under the rule), with
    resets; flow_hist = 0 so that few flows take the sort too."""
    import torch
    from sidekick_amd.quack import Context, encode_flows
    for nflows, seed in ((10_000, 1), (40, 3), (3_000, 4), (30_000, 5)):
        bufs, meta = make_flows(200_000, nflows, seed=seed, p_reset=0.02)
        want, nres, _ = vector_flows(bufs, meta)
        d_bufs = torch.from_numpy(bufs.reshape(-1).copy()).cuda()
        d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda()
        recs = {}
        for mode in (0, 1, 2):
            ctx = Context(0)
            ctx.set_knob("flow_hist", 0)
            ctx.set_knob("flow_byslot", mode)
            for _ in range(2):   # the second batch's table is sized from the first's flows
                keys, qs, st = encode_flows(d_bufs, 24, meta=d_meta, my_addr=MY_ADDR, ctx=ctx)
            assert st["resets"] == nres
            assert keys == sorted(want)
            for k, q in zip(keys, qs):
                ids = want[k]
                assert q.count() == len(ids) and q.last_value() == ids[-1], (mode, k.hex())
                if mode == 0:
                    assert q.power_sums() == coracle.encode_u32(np.array(ids, dtype=np.uint32), 24), k.hex()
            recs[mode] = [bytes(q._buf.raw) for q in qs]
            ctx.close()
        assert recs[1] == recs[0] and recs[2] == recs[0], nflows


@pytest.mark.gpu
@pytest.mark.parametrize("nflows,t,p_reset,skew", [(1, 32, 0.0, False), (16, 32, 0.01, False), (300, 16, 0.0, True),
                                                   (1500, 48, 0.005, False)])
def test_gpu_flows_histogram_grouping(nflows, t, p_reset, skew):
    """Few flows (a table of <= 8192 slots): the batch is grouped by
    per-workgroup slot histograms and a scatter instead of the radix sort; the
    order inside a flow is arbitrary, so the counts, last ids (from the last
    packet index) and sums must match the oracle, and the records must be the
    radix-sort path's (knob flow_hist = 0) byte for byte — one flow, skewed
    flows, resets, and the work-item path (t > 32) included.  flow_hist =
    8192 forces the histogram path at every flow count here (the product
    takes it up to 32 flows)."""
    import torch
    from sidekick_amd.quack import Context, encode_flows
    bufs, meta = make_flows(250_000 + nflows, nflows, seed=nflows + t, p_reset=p_reset, skew=skew)
    want, nres, _ = vector_flows(bufs, meta)
    d_bufs = torch.from_numpy(bufs.reshape(-1).copy()).cuda()
    d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda()
    recs = {}
    for mode in (8192, 0):
        ctx = Context(0)
        ctx.set_knob("flow_hist", mode)
        keys, qs, st = encode_flows(d_bufs, t, meta=d_meta, my_addr=MY_ADDR, ctx=ctx)
        assert st["resets"] == nres and st["inserted"] == sum(len(v) for v in want.values())
        assert keys == sorted(want)
        for k, q in zip(keys, qs):
            ids = want[k]
            assert q.count() == len(ids) and q.last_value() == ids[-1], k.hex()
        for i in range(0, len(keys), max(1, len(keys) // 40)):
            assert qs[i].power_sums() == coracle.encode_u32(np.array(want[keys[i]], dtype=np.uint32), t)
        recs[mode] = [bytes(q._buf.raw) for q in qs]
        ctx.close()
    assert recs[8192] == recs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["first", "middle", "last", "none"])
def test_gpu_flows_reset_wipes_table(where):
    """A Reset anywhere in the batch wipes every flow made before it, the
    caller's existing table included (sidekick_multi.rs:205,265); a reset as
    the last packet leaves an empty table.  Stats match the literal loop."""
    import torch
    import sidekick_amd as sk
    n = 3000
    bufs, meta = make_flows(n, 12, seed=77, p_reset=0.0)
    pos = {"first": 0, "middle": n // 2, "last": n - 1, "none": None}[where]
    if pos is not None:
        bufs[pos, 30:34] = MY_ADDR[:4]
        bufs[pos, 36:38] = MY_ADDR[4:]
        meta["pkttype"][pos], meta["protocol_be"][pos] = 0, 0x0008
        bufs[pos, 23] = 17
    otab = {b"\x02" * 12: qo.OracleQuack(32)}
    otab, ost = qo.sniff_multi_batch(otab, 32, bufs, meta["pkttype"], meta["protocol_be"], meta["len"], MY_ADDR)
    table = sk.FlowQuacks(32)
    table.insert(b"\x02" * 12, 5)
    st = table.insert_packets(torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67,
                              meta=torch.from_numpy(meta.view(np.int64).copy()).cuda(), my_addr=MY_ADDR)
    assert st == ost
    assert set(table.senders()) == set(otab)
    for k, q in otab.items():
        g = table.senders()[k]
        if k == b"\x02" * 12:
            continue
        assert g.power_sums() == q.power_sums and g.count() == q.count and g.last_value() == q.last_value
    if where == "last":
        assert table.senders() == {}


@pytest.mark.gpu
@pytest.mark.parametrize("nflows", [16, 10_000])
def test_gpu_flows_device_resident_output(nflows):
    """keys/sketches in HBM (written in place by the finalize kernel) are the
    same records as the host-output path, against the literal loop; mixed
    host/device output pointers are rejected."""
    import ctypes as C
    import torch
    from sidekick_amd._lib import lib
    from sidekick_amd.quack import encode_flows, get_context
    bufs, meta = make_flows(150_000, nflows, seed=nflows, p_reset=0.01)
    want, nres, _ = vector_flows(bufs, meta)
    d_bufs = torch.from_numpy(bufs.reshape(-1).copy()).cuda()
    d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda()
    hk, hq, hst = encode_flows(d_bufs, 32, meta=d_meta, my_addr=MY_ADDR)
    dk, dq, dst = encode_flows(d_bufs, 32, meta=d_meta, my_addr=MY_ADDR, device_out=True)
    torch.cuda.synchronize()
    assert hst == dst and dst["resets"] == nres
    assert hk == sorted(want) and [bytes(r) for r in dk.cpu().numpy()] == hk
    recs = dq.cpu().numpy().view(np.uint32)
    for i, (k, q) in enumerate(zip(hk, hq)):
        assert bytes(q._buf.raw) == recs[i].tobytes(), k.hex()
        assert q.power_sums() == coracle.encode_u32(np.array(want[k], dtype=np.uint32), 32)
    # mixed output memory kinds -> QK_E_INVAL
    keys = torch.empty((len(hk), 12), dtype=torch.uint8, device="cuda")
    host_sk = C.create_string_buffer(len(hk) * lib().qk_u32_size(32))
    nf = C.c_size_t()
    rc = lib().qk_u32_encode_flows_device(get_context(0).handle, d_bufs.data_ptr(), bufs.shape[0], 67,
                                          d_meta.data_ptr(), (C.c_uint8 * 6)(*MY_ADDR), 32, keys.data_ptr(), host_sk,
                                          len(hk), C.byref(nf), None, None)
    assert rc == -1


@pytest.mark.gpu
@pytest.mark.parametrize("nflows,skew,p_reset,hist", [(80_000, False, 0.002, 32), (120_000, True, 0.0, 32),
                                                       (80_000, False, 0.0, 0)])
def test_gpu_flows_three_pass_grouping_sort(nflows, skew, p_reset, hist):
    """More than 65 536 flows over 1e6 records: the flow table has > 2^16
    slots, so the grouping sort (radix.h) runs three digit passes — key/value
    arrays in (the first pass's counts fused into the extract), the pair
    array in and out in the middle pass, arrays out (sidekick_multi.rs:65-90's
    per-flow map for a batch).  Against the literal sniff loop's tables:
    every flow's sums, count and last_value, in ascending key order; the
    records of both grouping keys (knob flow_byslot 1 / 2: by slot, three
    passes; by flow rank after the slot -> rank remap) must equal the rule's
    byte for byte.  flow_hist at its default (32 flows) and 0 (never): the
    table is above the few-flow size, so both take the sort."""
    import torch
    from sidekick_amd.quack import Context, encode_flows
    bufs, meta = make_flows(1_000_000, nflows, seed=nflows + int(skew), p_reset=p_reset, skew=skew,
                            reset_until=0.2)
    want, nres, _ = vector_flows(bufs, meta)
    assert len(want) > (1 << 16) or skew
    d_bufs = torch.from_numpy(bufs.reshape(-1).copy()).cuda()
    d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda()
    recs = {}
    for byslot in (0, 1, 2):
        ctx = Context(0)
        ctx.set_knob("flow_hist", hist)
        ctx.set_knob("flow_byslot", byslot)
        keys, qs, st = encode_flows(d_bufs, 32, meta=d_meta, my_addr=MY_ADDR, ctx=ctx)
        assert st["resets"] == nres and st["inserted"] == sum(len(v) for v in want.values())
        assert keys == sorted(want)
        recs[byslot] = [bytes(q._buf.raw) for q in qs]
        if byslot == 0:
            for k, q in zip(keys, qs):
                ids = want[k]
                assert q.count() == len(ids) and q.last_value() == ids[-1], k.hex()
                assert q.power_sums() == coracle.encode_u32(np.array(ids, dtype=np.uint32), 32), k.hex()
        ctx.close()
    assert recs[1] == recs[0] and recs[2] == recs[0]
