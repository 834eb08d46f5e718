"""Packet-batch extraction fused with encode vs the
oracle's literal restatement of the sniff loop (sidekick.rs:76-124)."""
import numpy as np
import pytest

from oracle import coracle, quack_oracle as qo

MY_IP = (10, 0, 2, 1)
PROTO_IP = 0x0008
META_DT = np.dtype([("pkttype", "u1"), ("reserved", "u1"), ("protocol_be", "<u2"), ("len", "<u4")])


def make_batch(n, stride=67, seed=0, reset_at=(), p_filter=0.1):
    rng = np.random.default_rng(seed)
    bufs = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
    bufs[:, 23] = 17
    bufs[:, 30:34] = (192, 168, 1, 7)
    meta = np.zeros(n, dtype=META_DT)
    meta["pkttype"] = 0
    meta["protocol_be"] = PROTO_IP
    meta["len"] = 67
    r = rng.random(n)
    k = r < p_filter
    kind = rng.integers(0, 5, size=n)
    meta["pkttype"][k & (kind == 0)] = 4            # outgoing
    meta["pkttype"][k & (kind == 1)] = 3            # other host: still incoming
    meta["protocol_be"][k & (kind == 2)] = 0xDD86   # IPv6
    bufs[k & (kind == 3), 23] = 6                   # TCP
    meta["len"][k & (kind == 4)] = 60               # underfilled
    for i in reset_at:
        bufs[i, 30:34] = MY_IP
    return bufs, meta


def vector_sniff(bufs, meta, my_ip=MY_IP):
    """Vectorised form of oracle.sniff_batch's classification (checked against
    it below): returns (ids inserted after the last reset, last reset index)."""
    inc = (meta["pkttype"] == 0) | (meta["pkttype"] == 3)
    ok = inc & (meta["protocol_be"] == PROTO_IP) & (bufs[:, 23] == 17)
    reset = ok & np.all(bufs[:, 30:34] == np.array(my_ip, dtype=np.uint8), axis=1) if my_ip else np.zeros(len(bufs), bool)
    ins = ok & ~reset & (meta["len"] == 67)
    last = int(np.nonzero(reset)[0][-1]) if reset.any() else -1
    sel = np.nonzero(ins)[0]
    sel = sel[sel > last]
    idb = bufs[sel, 63:67].astype(np.uint32)
    ids = (idb[:, 0] << 24) | (idb[:, 1] << 16) | (idb[:, 2] << 8) | idb[:, 3]
    return ids.astype(np.uint32), last


def test_oracle_sniff_hand_example():
    bufs, meta = make_batch(6, seed=1, p_filter=0)
    meta["pkttype"][1] = 4                      # outgoing: skipped
    bufs[3, 30:34] = MY_IP                      # reset: wipes packet 0 and 2
    meta["len"][5] = 66                         # underfilled: skipped
    q, st = qo.sniff_batch(qo.OracleQuack(4), bufs, meta["pkttype"], meta["protocol_be"], meta["len"], MY_IP)
    want = qo.OracleQuack(4)
    want.insert(int.from_bytes(bytes(bufs[4, 63:67]), "big"))
    assert q.power_sums == want.power_sums and q.count == 1 and q.last_value == want.last_value
    assert st == {"inserted": 1, "discarded": 2, "resets": 1, "filtered": 2, "last_reset_index": 3}


def test_vector_sniff_matches_oracle():
    for seed in range(5):
        bufs, meta = make_batch(400, seed=seed, reset_at=(17, 200) if seed % 2 else (), p_filter=0.3)
        q, st = qo.sniff_batch(qo.OracleQuack(8), bufs, meta["pkttype"], meta["protocol_be"], meta["len"], MY_IP)
        ids, last = vector_sniff(bufs, meta)
        w = qo.OracleQuack(8)
        w.insert_all(ids.tolist())
        assert w.power_sums == q.power_sums and len(ids) == st["inserted"] and last == st["last_reset_index"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,stride,off,resets", [
    (0, 67, 0, ()), (1, 67, 0, ()), (255, 67, 3, ()), (256, 67, 0, (255,)), (257, 67, 1, (256,)),
    (5000, 67, 7, (0, 1023, 1024)), (5000, 128, 0, (4999,)), (100_003, 67, 13, (33_333,)),
    (1_000_000, 67, 0, (123_456, 999_000)), (1_000_000, 67, 5, ()),
    (5000, 128, 3, ()), (100_003, 67, 13, ()), (70_001, 200, 7, ()),   # t = 32 one-pass: strides, unaligned bases
])
def test_gpu_packets_vs_oracle(n, stride, off, resets):
    import torch
    import sidekick_amd as sk
    from sidekick_amd.quack import encode_packets
    bufs, meta = make_batch(n, stride=stride, seed=n + stride, reset_at=resets)
    raw = np.zeros(n * stride + off, dtype=np.uint8)
    raw[off:] = bufs.reshape(-1)
    d_raw = torch.from_numpy(raw).cuda()
    d_bufs = d_raw[off:]                       # unaligned base when off % 16 != 0
    d_meta = torch.from_numpy(meta.view(np.int64).copy()).cuda() if n else None
    q = sk.PowerSumQuackU32(32)
    q.insert(12345)                            # pre-existing state survives unless a reset happens
    st = encode_packets(q, d_bufs, stride=stride, meta=d_meta, my_ipv4=MY_IP)
    ids, last = vector_sniff(bufs, meta)
    want = coracle.encode_u32(ids, 32)
    if last < 0:
        pre = sk.PowerSumQuackU32(32)
        pre.insert(12345)
        want = [(a + b) % qo.P32 for a, b in zip(want, pre.power_sums())]
    assert q.power_sums() == want
    assert q.count() == len(ids) + (1 if last < 0 else 0)
    assert st["inserted"] == len(ids) and st["last_reset_index"] == last and st["resets"] == len(resets)
    if len(ids):
        assert q.last_value() == int(ids[-1])
    elif last >= 0:
        assert q.last_value() is None


@pytest.mark.gpu
def test_gpu_packets_no_meta_no_ip():
    import torch
    import sidekick_amd as sk
    from sidekick_amd.quack import encode_packets
    n = 70_001
    bufs, meta = make_batch(n, seed=3, p_filter=0.0, reset_at=(10,))
    bufs[5, 23] = 6                            # one TCP packet: still filtered by buf[23]
    q = sk.PowerSumQuackU32(16)
    st = encode_packets(q, torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67, meta=None, my_ipv4=None)
    m = np.zeros(n, dtype=META_DT)
    m["protocol_be"] = PROTO_IP
    m["len"] = 67
    ids, last = vector_sniff(bufs, m, my_ip=None)
    assert last == -1 and st["resets"] == 0       # no own address: packets to 10.0.2.1 are ordinary
    assert q.power_sums() == coracle.encode_u32(ids, 16) and st["inserted"] == n - 1


@pytest.mark.gpu
@pytest.mark.parametrize("t", [4, 5, 8, 9, 12, 13, 16, 24, 25, 28, 31, 32, 33])
def test_gpu_packets_fused_thresholds(golden, t):
    """5 <= t <= 32 without a reset in the batch takes the fused kernel
    (records -> baby-step/giant-step sums, no id array: lane-private
    accumulators up to t = 12, the (8, NA) sums split across the waves
    through LDS from 13 on); the lazy-fold wrap ids of the matching
    configuration sit in records so the exact-recompute branch runs inside
    it; t = 4, 33+ and a batch with a reset take the two-pass path.  All
    against the sniff-loop restatement."""
    import torch
    import sidekick_amd as sk
    from sidekick_amd.quack import encode_packets
    cfg = "4x2" if t <= 8 else "4x3" if t <= 12 else "8x2" if t <= 16 else "8x3" if t <= 24 else "8x4" if t <= 32 \
        else "8x5"
    wraps = np.array(golden["bsgs_wrap_ids"][cfg], dtype=np.uint32)
    for resets in ((), (31_000,)):
        n = 50_001
        bufs, meta = make_batch(n, seed=t * 7 + len(resets), reset_at=resets, p_filter=0.05)
        for j, w in enumerate(wraps):               # identifiers that force the exact branch
            k = 1000 + 97 * j
            bufs[k, 63:67] = np.frombuffer(int(w).to_bytes(4, "big"), dtype=np.uint8)
        q = sk.PowerSumQuackU32(t)
        st = encode_packets(q, torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67,
                            meta=torch.from_numpy(meta.view(np.int64).copy()).cuda(), my_ipv4=MY_IP)
        ids, last = vector_sniff(bufs, meta)
        assert q.power_sums() == coracle.encode_u32(ids, t), (t, resets)
        assert q.count() == len(ids) and st["inserted"] == len(ids) and st["last_reset_index"] == last
        assert st["filtered"] == n - len(ids) - st["discarded"] - st["resets"]
        if len(ids):
            assert q.last_value() == int(ids[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 257, 4097, 300_007, 1_500_013])
def test_gpu_packets_chunk_edges(n):
    """Batch sizes around the chunking (one record; a partial tile; one tile
    and one record; many chunks of 4+ tiles): the same sums, counts and reset
    bookkeeping as the literal loop, fused (t = 12, and t = 32 without a
    reset) and two-pass (t = 32 with a reset)."""
    import torch
    import sidekick_amd as sk
    from sidekick_amd.quack import encode_packets
    for t, resets in ((12, ()), (32, (n // 3,)), (32, ())):
        bufs, meta = make_batch(n, seed=n % 1000 + t, reset_at=resets, p_filter=0.05)
        q = sk.PowerSumQuackU32(t)
        st = encode_packets(q, torch.from_numpy(bufs.reshape(-1).copy()).cuda(), stride=67,
                            meta=torch.from_numpy(meta.view(np.int64).copy()).cuda(), my_ipv4=MY_IP)
        ids, last = vector_sniff(bufs, meta)
        assert q.power_sums() == coracle.encode_u32(ids, t), (n, t, resets)
        assert st["inserted"] == len(ids) and st["last_reset_index"] == last
