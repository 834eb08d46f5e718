"""The native multi-GPU path over RCCL with more than one device — runs only on
a node with >= 2 GPUs (the driver's 8-GPU node); a one-GPU box skips it.

One process drives every visible device through `qk_comm_create`
(ncclCommInitAll), the single-process form the reference's Rust callers need
(`sidekick/src/sidekick.rs:58-127`, `sidekick/src/bin/sender.rs:80-116`):
each device encodes its contiguous shard of one global stream and the root's
result must equal the single-GPU encode and the oracle bit-exactly; the
sharded decode must return the single-GPU hit list.  The same protocol at
world 2-8 on one GPU (host channel) is in tests/test_gpu_comm.py."""
import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu


def _ndev():
    import torch
    return torch.cuda.device_count()


needs_two = pytest.mark.skipif("_ndev() < 2", reason="needs >= 2 GPUs in one node")


@pytest.fixture(scope="module")
def comm_all():
    from sidekick_amd.dist import Comm
    n = _ndev()
    if n < 2:
        pytest.skip("needs >= 2 GPUs in one node")
    c = Comm.create(list(range(n)))
    assert (c.world, c.nlocal, c.first_rank) == (n, n, 0)
    yield c
    c.close()


def _shard_views(host, bits, ndev, empty=()):
    """Contiguous shards in rank order, shard r resident on device r."""
    import torch
    from sidekick_amd.dist import shard
    dt = np.int32 if bits == 32 else np.int64
    live = [r for r in range(ndev) if r not in empty]
    views = []
    for r in range(ndev):
        if r in empty:
            views.append(torch.empty(0, dtype=torch.int32 if bits == 32 else torch.int64, device=f"cuda:{r}"))
            continue
        s, c = shard(len(host), live.index(r), len(live))
        views.append(torch.from_numpy(host[s:s + c].view(dt)).to(f"cuda:{r}"))
    return views


@needs_two
@pytest.mark.parametrize("bits,t,n,empty", [(32, 32, 4_000_037, ()), (32, 16, 1_000_003, (1,)),
                                            (64, 80, 600_001, ()), (64, 20, 99, (0,))])
def test_multidevice_sharded_encode_bit_exact(comm_all, bits, t, n, empty):
    import sidekick_amd as sk
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    host = coracle.splitmix_u32(0x11 + t, n) if bits == 32 else coracle.splitmix_u64(0x11 + t, n)
    views = _shard_views(host, bits, comm_all.nlocal, empty)
    got = Q(t)
    got.insert(4242)
    comm_all.encode_sharded(views, got)
    full = np.concatenate([np.array([4242], dtype=host.dtype), host])
    assert got.power_sums() == (coracle.encode_u32(full, t) if bits == 32 else coracle.encode_u64(full, t))
    assert got.count() == n + 1 and got.last_value() == int(host[-1])


@needs_two
def test_multidevice_async_steps(comm_all):
    import sidekick_amd as sk
    host = coracle.splitmix_u32(0xA11, 2_000_000)
    views = _shard_views(host, 32, comm_all.nlocal)
    for _ in range(3):
        comm_all.encode_sharded_async(views, 32)
    q = sk.PowerSumQuackU32(32)
    comm_all.encode_sharded_wait(q)
    assert q.power_sums() == coracle.encode_u32(host, 32) and q.count() == len(host)


@needs_two
@pytest.mark.parametrize("bits,stop", [(32, True), (32, False), (64, True)])
def test_multidevice_sharded_decode_matches_single_gpu(comm_all, bits, stop):
    import torch
    import sidekick_amd as sk
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    n = 300_000
    host = coracle.splitmix_u32(0xD0 + bits, n) if bits == 32 else coracle.splitmix_u64(0xD0 + bits, n)
    rng = np.random.default_rng(bits)
    drops = np.sort(rng.choice(n, 28, replace=False))
    keep = np.ones(n, bool)
    keep[drops] = False
    dt = np.int32 if bits == 32 else np.int64
    log0 = torch.from_numpy(host.view(dt)).cuda()
    a, b = Q(32), Q(32)
    a.insert_batch(log0)
    b.insert_batch(torch.from_numpy(host[keep].view(dt)).cuda())
    a.sub_assign(b)
    want = a.root_test(a.to_coeffs(), log0, stop_value=a.last_value() if stop else None)
    views = _shard_views(host, bits, comm_all.nlocal)
    got = comm_all.decode_sharded(a, views, bits=bits, stop_at_last=stop)
    assert got == want
    assert set(drops.tolist()) - {n - 1} <= set(got)
