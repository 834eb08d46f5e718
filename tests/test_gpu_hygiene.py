"""Context hygiene on the GPU: growing a context's grow-only buffers never
synchronises the device (hipFree would; grown-out buffers are retired
instead), so a caller's unrelated work queued on another stream keeps
running while the library's call returns.

The probe runs in a fresh process with GPU_MAX_HW_QUEUES=16: HIP maps
streams round-robin onto that many in-order hardware queues (4 by default),
and two streams sharing one queue serialise whatever the library does.  A
control call that needs no growth must not wait either, else the probe
measures the queue mapping, not the library."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import json, time, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
import sidekick_amd as sk
from oracle import coracle
host = coracle.splitmix_u32(0x51EE, 2_000_000)
ids = torch.from_numpy(host.view(np.int32)).cuda()
busy, work = torch.cuda.Stream(), torch.cuda.Stream()
ctx = sk.Context(0)
q0 = sk.PowerSumQuackU32(32)
q0.insert_batch(ids, ctx=ctx)                     # first use: the default scratch
torch.cuda.synchronize()

def trial(grid):
    ctx.set_grid(grid)
    done = torch.cuda.Event()
    with torch.cuda.stream(busy):
        torch.cuda._sleep(int(4e9))               # ~2 s of spinning on an unrelated stream
        done.record(busy)
    t0 = time.perf_counter()
    q = sk.PowerSumQuackU32(32)
    with torch.cuda.stream(work):
        q.insert_batch(ids, ctx=ctx)              # synchronous call on its own stream
    dt = time.perf_counter() - t0
    still_busy = not done.query()
    torch.cuda.synchronize()
    return {"dt": dt, "still_busy": still_busy, "ok": q.power_sums() == q0.power_sums()}

control = trial(512)                              # fits the current scratch
grow = trial(16384)                               # 16384 blocks x 32 powers x 8 B = 4 MiB: the scratch grows
ctx.trim()
q = sk.PowerSumQuackU32(32)
q.insert_batch(ids, ctx=ctx)
print(json.dumps({"control": control, "grow": grow, "after_trim_ok": q.power_sums() == q0.power_sums(),
                  "oracle_ok": q0.power_sums() == coracle.encode_u32(host, 32)}))
"""


def test_scratch_growth_does_not_wait_for_other_streams():
    import torch
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, "-c", PROBE, ROOT], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["oracle_ok"] and res["after_trim_ok"] and res["control"]["ok"] and res["grow"]["ok"], res
    assert res["control"]["still_busy"], f"the queue mapping serialises the streams: {res}"
    assert res["grow"]["still_busy"], f"growing the scratch waited for the unrelated stream: {res}"
