"""Context hygiene on the GPU: growing a context's grow-only buffers never
synchronises the device (hipFree would: stream-ordered free/alloc instead),
so a caller's unrelated work queued on another stream keeps running while
the library's call returns."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_scratch_growth_does_not_wait_for_other_streams():
    import torch
    import sidekick_amd as sk
    from oracle import coracle
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    host = coracle.splitmix_u32(0x51EE, 2_000_000)
    ids = torch.from_numpy(host.view(np.int32)).cuda()
    ctx = sk.Context(0)                       # fresh context: 1 MiB scratch at most so far
    try:
        q0 = sk.PowerSumQuackU32(32)
        q0.insert_batch(ids, ctx=ctx)         # first use: small scratch
        torch.cuda.synchronize()
        ctx.set_grid(16384)                   # 16384 blocks x 32 powers x 8 B = 4 MiB: the scratch grows
        busy, work = torch.cuda.Stream(), torch.cuda.Stream()
        done = torch.cuda.Event()
        with torch.cuda.stream(busy):
            torch.cuda._sleep(int(4e9))       # ~2 s of spinning on an unrelated stream
            done.record(busy)
        t0 = time.perf_counter()
        q = sk.PowerSumQuackU32(32)
        with torch.cuda.stream(work):
            q.insert_batch(ids, ctx=ctx)      # synchronous call on its own stream
        dt = time.perf_counter() - t0
        still_busy = not done.query()
        torch.cuda.synchronize()
        assert q.power_sums() == q0.power_sums() == coracle.encode_u32(host, 32)
        assert still_busy, f"the encode waited for the unrelated stream ({dt:.3f} s)"
    finally:
        ctx.close()
