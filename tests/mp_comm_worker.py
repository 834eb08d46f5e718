"""One rank of tests/test_gpu_comm_mp.py: the native communicator (comm.hip)
with its collectives over torch.distributed (gloo) between PROCESSES, every
rank on device 0 — the one-process-per-GPU shape of bench.py --gpus N, with
the real process boundary between ranks.

    python -m torch.distributed.run --nproc-per-node 2 tests/mp_comm_worker.py OUT_DIR
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    import sidekick_amd as sk
    from oracle import coracle
    from sidekick_amd._lib import QK_E_HIP, QK_E_PEER, QK_OK, lib
    from sidekick_amd.dist import Comm, ProcessGroupChannel, shard

    out_dir = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    comm = Comm.init_host(ProcessGroupChannel(), rank, world, 0)
    res = {"rank": rank, "world": world}

    # sharded encode, u32 t = 32 and u64 t = 80, against the oracle on the root
    for bits, t, n in ((32, 32, 2_000_003), (64, 80, 300_001)):
        Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
        host = (coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64)(0xB0 + bits, n)
        s, c = shard(n, rank, world)
        dev = torch.from_numpy(host[s:s + c].view(np.int32 if bits == 32 else np.int64)).cuda()
        q = Q(t)
        q.insert(41)
        comm.encode_sharded([dev], q)
        if rank == 0:
            full = np.concatenate([np.array([41], dtype=host.dtype), host])
            want = coracle.encode_u32(full, t) if bits == 32 else coracle.encode_u64(full, t)
            res[f"encode_u{bits}"] = q.power_sums() == want and q.count() == n + 1 and q.last_value() == int(host[-1])
        else:
            res[f"encode_u{bits}"] = q.count() == 1 and q.last_value() == 41   # untouched

    # sharded decode against the single-GPU hit list, both widths
    for bits in (32, 64):
        Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
        dt = np.int32 if bits == 32 else np.int64
        n = 300_000
        a = (coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64)(0xDE5 + bits, n).copy()
        drops = np.sort(np.random.default_rng(bits).choice(n, 28, replace=False))
        a[150_000:150_400] = a[drops[0]]                       # one shard holds > one hit round
        keep = np.ones(n, bool)
        keep[drops] = False
        log = torch.from_numpy(a.view(dt)).cuda()
        A, B = Q(32), Q(32)
        A.insert_batch(log)
        B.insert_batch(torch.from_numpy(a[keep].view(dt)).cuda())
        A.sub_assign(B)
        want = A.root_test(A.to_coeffs(), log, stop_value=A.last_value())
        s, c = shard(n, rank, world)
        got = comm.decode_sharded(A if rank == 0 else None, [log[s:s + c]], bits=bits, stop_at_last=True)
        res[f"decode_u{bits}"] = got == want and len(want) >= 400

    # a staging fault on rank 1 at the status gather (step 2): every rank
    # returns QK_E_HIP; a fault on rank 1 in the encode's reduce: it returns
    # QK_E_HIP, the root QK_E_PEER; then a clean round
    host = coracle.splitmix_u32(0xFA, 100_000)
    s, c = shard(len(host), rank, world)
    dev = torch.from_numpy(host[s:s + c].view(np.int32)).cuda()
    if rank == 1:
        comm.context(0).set_knob("comm_fault", 1)
    q = sk.PowerSumQuackU32(16)
    rc = lib().qk_u32_encode_sharded(comm.handle, (C.c_void_p * 1)(dev.data_ptr()), (C.c_size_t * 1)(c), q._buf, 0,
                                     None)
    res["fault_encode"] = rc == (QK_E_HIP if rank == 1 else QK_E_PEER if rank == 0 else QK_OK) and q.count() == 0
    if rank == 1:
        comm.context(0).set_knob("comm_fault", 2)
    hits = (C.c_uint64 * 64)()
    nh = C.c_size_t()
    A = sk.PowerSumQuackU32(16)
    for v in host[:5]:
        A.insert(int(v))
    rc = lib().qk_u32_decode_sharded(comm.handle, A._buf if rank == 0 else None, 0, (C.c_void_p * 1)(dev.data_ptr()),
                                     (C.c_size_t * 1)(c), 0, hits, 64, C.byref(nh), None)
    res["fault_decode_rc"] = rc
    res["fault_decode"] = rc == QK_E_HIP
    q = sk.PowerSumQuackU32(16)
    comm.encode_sharded([dev], q)
    res["clean_after_faults"] = rank != 0 or q.power_sums() == coracle.encode_u32(host, 16)

    comm.close()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
