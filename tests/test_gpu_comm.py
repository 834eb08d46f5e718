"""The native multi-GPU path (qk_comm_*, comm.hip: RCCL over xGMI) on the
GPU box: a one-device communicator, built both ways (ncclCommInitAll from one
process; unique id + ncclCommInitRank), must give the single-GPU encode and
decode bit-exactly — the sharded encode's one ncclReduce, the pack of the
per-rank last-id slots and the root's fold all run; so do the sharded
decode's broadcast and two all-gathers.  (A box has one GPU and RCCL takes
one rank per GPU, so N > 1 runs only on the driver's 8-GPU node; the same
protocol at world 2-3 is rehearsed on CPU in tests/test_dist.py.)"""
import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["create", "init_rank"])
def comm(request):
    from sidekick_amd.dist import Comm
    c = Comm.create([0]) if request.param == "create" else Comm.init_rank(Comm.unique_id(), 0, 1, 0)
    assert (c.world, c.nlocal, c.first_rank) == (1, 1, 0)
    yield c
    c.close()


def _ids(bits, n, seed):
    import torch
    a = coracle.splitmix_u32(seed, n) if bits == 32 else coracle.splitmix_u64(seed, n)
    return a, torch.from_numpy(a.view(np.int32 if bits == 32 else np.int64)).cuda()


@pytest.mark.parametrize("bits,t,n", [(32, 32, 3_000_001), (32, 16, 1000), (32, 80, 100_003), (64, 80, 200_001),
                                      (64, 20, 7)])
def test_sharded_encode_one_device_bit_exact(comm, bits, t, n):
    import sidekick_amd as sk
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    host, ids = _ids(bits, n, 0xC0 + t + bits)
    want = Q(t)
    want.insert(12345)                      # existing content: the stream follows it
    want.insert_batch(ids)
    got = Q(t)
    got.insert(12345)
    comm.encode_sharded([ids], got)
    assert got == want
    full = np.concatenate([np.array([12345], dtype=host.dtype), host])
    assert got.power_sums() == (coracle.encode_u32(full, t) if bits == 32 else coracle.encode_u64(full, t))
    assert got.count() == n + 1 and got.last_value() == int(host[-1])


def test_sharded_encode_async_steps_and_empty_shard(comm):
    import torch
    import sidekick_amd as sk
    host, ids = _ids(32, 1_000_000, 0xA5)
    for _ in range(3):                      # back-to-back async steps reuse the payload buffer
        comm.encode_sharded_async([ids], 32)
    q = sk.PowerSumQuackU32(32)
    comm.encode_sharded_wait(q)
    assert q.power_sums() == coracle.encode_u32(host, 32) and q.count() == len(host)
    empty = torch.empty(0, dtype=torch.int32, device="cuda")
    q2 = sk.PowerSumQuackU32(32)
    q2.insert(9)
    comm.encode_sharded([empty], q2)         # an empty shard keeps the last value and adds nothing
    assert q2.count() == 1 and q2.last_value() == 9
    with pytest.raises(sk.QuackError):
        comm.encode_sharded_wait(q2)         # nothing in flight
    comm.barrier()


@pytest.mark.parametrize("bits", [32, 64])
def test_sharded_decode_one_device_matches_single_gpu(comm, bits):
    import sidekick_amd as sk
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    host, log = _ids(bits, 500_000, 0xDEC + bits)
    rng = np.random.default_rng(bits)
    drops = np.sort(rng.choice(len(host), 24, replace=False))
    keep = np.ones(len(host), bool)
    keep[drops] = False
    a, b = Q(32), Q(32)
    a.insert_batch(log)
    import torch
    b.insert_batch(torch.from_numpy(host[keep].view(np.int32 if bits == 32 else np.int64)).cuda())
    a.sub_assign(b)
    want = a.root_test(a.to_coeffs(), log, stop_value=a.last_value())
    got = comm.decode_sharded(a, [log], bits=bits, stop_at_last=True)
    assert got == want
    assert set(drops.tolist()) - {len(host) - 1} <= set(got)
    # no stop: every hit of the log
    assert comm.decode_sharded(a, [log], bits=bits, stop_at_last=False) == a.root_test(a.to_coeffs(), log)


def test_sharded_decode_undecodable_and_empty(comm):
    import sidekick_amd as sk
    from sidekick_amd._lib import UndecodableError
    host, log = _ids(32, 10_000, 0x77)
    q = sk.PowerSumQuackU32(4)
    for v in host[:9]:
        q.insert(int(v))
    with pytest.raises(UndecodableError):
        comm.decode_sharded(q, [log])
    z = sk.PowerSumQuackU32(4)
    assert comm.decode_sharded(z, [log]) == []
