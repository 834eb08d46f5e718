"""Multi-rank sharding of the encode path on CPU (gloo, world_size 2 and 3).

Each rank owns a contiguous shard of one global id stream, encodes it (here
with the host path; on GPUs with the gfx950 kernel — same partial layout),
and ONE sum-reduce of the partial words merges the shards on rank 0, exactly
as bench.py does over RCCL.  Rank 0's folded result must equal the oracle on
the whole stream."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import coracle, quack_oracle as qo


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bits, t, n_total, seed, q, empty_last):
    import torch
    import sidekick_amd as sk
    from sidekick_amd import dist as skd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the native protocol (comm.hip): contiguous shards, the payload with
        # per-rank last-id slots, ONE sum-reduce, the root's fold
        start, cnt = skd.shard(n_total, rank, world - 1 if empty_last else world)
        if empty_last and rank == world - 1:
            start, cnt = n_total, 0          # an empty trailing shard: last_value from the rank before
        ids = qo.ids_u32(seed, cnt, start) if bits == 32 else qo.ids_u64(seed, cnt, start)
        local = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
        for x in ids.tolist():
            local.insert(int(x))
        pay = skd.pack_payload(skd.state_to_partial(local), t, bits, rank, world)
        part = torch.from_numpy(pay.view(np.int64).copy())
        dist.reduce(part, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0:
            q.put(skd.fold_payload(part.numpy().view(np.uint64), t, bits, world))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bits,t,empty_last", [(2, 32, 32, False), (3, 32, 16, False), (2, 64, 20, False),
                                                     (3, 32, 8, True), (2, 64, 5, True)])
def test_sharded_encode_reduce_matches_oracle(world, bits, t, empty_last):
    n_total, seed = 3001, 0xD15
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bits, t, n_total, seed, q, empty_last))
             for r in range(world)]
    for p in procs:
        p.start()
    S, count, last = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if bits == 32:
        assert S == coracle.encode_u32_seed(seed, n_total, t)
        assert last == int(qo.ids_u32(seed, 1, n_total - 1)[0])
    else:
        assert S == coracle.encode_u64_seed(seed, n_total, t)
        assert last == int(qo.ids_u64(seed, 1, n_total - 1)[0])
    assert count == n_total


def test_shard_cover():
    from sidekick_amd import dist as skd
    for n in (0, 1, 7, 1000, 10**9 + 3):
        for w in (1, 2, 3, 8):
            parts = [skd.shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0
            assert sum(c for _, c in parts) == n
            for (s0, c0), (s1, _) in zip(parts, parts[1:]):
                assert s0 + c0 == s1


# ---------------------------------------------------------------- sharded decode
def _decode_case(bits, seed, n_total, n_drop, stop_at):
    """Global log, a dropped subset, and the expected single-log answer."""
    rng = np.random.default_rng(seed)
    log = (qo.ids_u32 if bits == 32 else qo.ids_u64)(seed, n_total, 0)
    log[rng.choice(n_total, 3, replace=False)] = log[rng.choice(n_total, 3, replace=False)]  # duplicates
    drops = sorted(rng.choice(n_total, n_drop, replace=False).tolist())
    p = qo.MOD[bits]
    diff = qo.OracleQuack(32, bits)
    for i in drops:
        diff.insert(int(log[i]))
    coeffs = diff.to_coeffs()
    stop = None if stop_at is None else int(log[stop_at])
    want = qo.root_test_indices(coeffs, log.tolist(), p, stop_value=stop)
    return log, coeffs, stop, want


def _oracle_shard_test(bits):
    def run(coeffs, shard, stop):
        vals = shard.tolist()
        pos = qo.root_test_indices(coeffs, vals, qo.MOD[bits], stop_value=stop)
        si = vals.index(stop) if stop is not None and stop in vals else len(vals)
        return pos, si
    return run


def _decode_worker(rank, world, port, bits, seed, n_total, n_drop, stop_at, use_gpu, q):
    import torch
    from sidekick_amd import dist as skd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log, coeffs, stop, want = _decode_case(bits, seed, n_total, n_drop, stop_at)
        c, s = skd.broadcast_coeffs(coeffs if rank == 0 else None, stop if rank == 0 else None, 32, bits)
        assert c == [int(v) for v in coeffs] and s == stop
        start, cnt = skd.shard(n_total, rank, world)
        shard = log[start:start + cnt]
        if use_gpu:
            import sidekick_amd as sk
            qcls = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
            dev = torch.from_numpy(shard.view(np.int32 if bits == 32 else np.int64).copy()).cuda()
            test = lambda cc, _sh, st: qcls(32).root_test_shard(cc, dev, stop_value=st)  # noqa: E731
        else:
            test = _oracle_shard_test(bits)
        got = skd.root_test_sharded(test, c, shard, start, s)
        q.put((rank, got == want, len(want)))
    finally:
        dist.destroy_process_group()


def _run_decode(world, bits, n_total, n_drop, stop_at, use_gpu, seed=0xDEC0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_decode_worker,
                         args=(r, world, port, bits, seed, n_total, n_drop, stop_at, use_gpu, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    return res[0][2]


@pytest.mark.parametrize("world,bits,stop_at", [(2, 32, None), (2, 32, 1500), (3, 32, 200), (3, 64, 2500),
                                                (2, 64, None)])
def test_sharded_root_test_matches_single_log(world, bits, stop_at):
    """SURVEY §8e decode sharding: broadcast coefficients, per-shard root
    test with the stop position, MIN-reduce of the stop, all-gather of hits
    == the single-log root test (media_client.rs:306-313)."""
    nh = _run_decode(world, bits, 3000, 12, stop_at, use_gpu=False)
    assert nh > 0


@pytest.mark.gpu
@pytest.mark.parametrize("bits,stop_at", [(32, None), (32, 40_000), (64, 70_000)])
def test_sharded_root_test_gpu_two_ranks(bits, stop_at):
    """The same merge with each rank's shard tested by the gfx950 root test
    (two processes on one GPU, gloo for the small collectives)."""
    _run_decode(2, bits, 100_000, 20, stop_at, use_gpu=True)


# ---------------------------------------------------------------- host channels
# The collectives comm.hip delegates to a host channel (qk_comm_init_host):
# LoopbackHub (threads of one process) and ProcessGroupChannel (a
# torch.distributed group), called the way the C side calls them — through
# the ctypes function pointers of qk_comm_host_ops.
import ctypes as C  # noqa: E402
import threading  # noqa: E402


def _call_ops(ch, op, a, b=None, root=0):
    ops = ch._ops()
    p = lambda x: x.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731
    if op == "reduce":
        return ops.reduce_sum_u64(None, p(a), len(a), root)
    if op == "bcast":
        return ops.broadcast_u64(None, p(a), len(a), root)
    return ops.allgather_u64(None, p(a), p(b), len(a))


def test_loopback_hub_collectives_through_ctypes():
    from sidekick_amd.dist import LoopbackHub
    world, n = 3, 5
    hub = LoopbackHub(world, timeout=30)
    res = [None] * world

    def rank(r):
        ch = hub.channel(r)
        red = np.arange(n, dtype=np.uint64) + np.uint64(10 * r)
        red[0] = np.uint64(2**64 - 1)                       # the sum wraps mod 2^64, as RCCL's
        rc1 = _call_ops(ch, "reduce", red, root=1)
        bc = np.full(n, r, dtype=np.uint64)
        rc2 = _call_ops(ch, "bcast", bc, root=2)
        send = np.full(n, 100 + r, dtype=np.uint64)
        recv = np.zeros(n * world, dtype=np.uint64)
        rc3 = _call_ops(ch, "gather", send, recv)
        res[r] = (rc1, rc2, rc3, red.copy(), bc.copy(), recv.copy())
    ths = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    for r in range(world):
        rc1, rc2, rc3, red, bc, recv = res[r]
        assert (rc1, rc2, rc3) == (0, 0, 0)
        assert (bc == 2).all()
        assert recv.tolist() == [100 + q for q in range(world) for _ in range(n)]
    want = (np.arange(n, dtype=np.uint64) * world + np.uint64(30)).tolist()
    want[0] = (3 * (2**64 - 1)) % 2**64
    assert res[1][3].tolist() == want


def test_loopback_missing_peer_fails_the_call_not_the_process():
    from sidekick_amd.dist import LoopbackHub
    hub = LoopbackHub(2, timeout=1)
    a = np.zeros(4, dtype=np.uint64)
    assert _call_ops(hub.channel(0), "reduce", a) == -1   # BrokenBarrierError -> nonzero to C


def _pg_channel_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sidekick_amd.dist import ProcessGroupChannel
        ch = ProcessGroupChannel()
        red = np.array([rank + 1, 2**40, 7], dtype=np.uint64)
        rc1 = _call_ops(ch, "reduce", red, root=0)
        bc = np.array([rank, rank], dtype=np.uint64)
        rc2 = _call_ops(ch, "bcast", bc, root=1)
        send = np.array([rank * 10, rank * 10 + 1], dtype=np.uint64)
        recv = np.zeros(2 * world, dtype=np.uint64)
        rc3 = _call_ops(ch, "gather", send, recv)
        q.put((rank, rc1, rc2, rc3, red.tolist(), bc.tolist(), recv.tolist()))
    finally:
        dist.destroy_process_group()


def test_process_group_channel_collectives():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pg_channel_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        rc1, rc2, rc3, red, bc, recv = res[r]
        assert (rc1, rc2, rc3) == (0, 0, 0)
        assert bc == [1, 1] and recv == [0, 1, 10, 11]
    assert res[0][3] == [3, 2**41, 14]
