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


def _worker(rank, world, port, bits, t, n_total, seed, q):
    import torch
    import sidekick_amd as sk
    from sidekick_amd import dist as skd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, cnt = skd.shard(n_total, rank, world)
        ids = qo.ids_u32(seed, cnt, start) if bits == 32 else qo.ids_u64(seed, cnt, start)
        local = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)
        for x in ids.tolist():
            local.insert(int(x))
        part = torch.from_numpy(skd.state_to_partial(local).view(np.int64).copy())
        skd.reduce_partial_(part, t, bits, dst=0)
        if rank == 0:
            S, count = skd.fold_partial_sum(part.numpy().view(np.uint64), t, bits)
            q.put((S, count))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bits,t", [(2, 32, 32), (3, 32, 16), (2, 64, 20)])
def test_sharded_encode_reduce_matches_oracle(world, bits, t):
    n_total, seed = 3001, 0xD15
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bits, t, n_total, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    S, count = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if bits == 32:
        assert S == coracle.encode_u32_seed(seed, n_total, t)
    else:
        assert S == coracle.encode_u64_seed(seed, n_total, t)
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
