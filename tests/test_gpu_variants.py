"""Every kernel variant the dispatcher can select, checked against the oracle.

The tuning knobs (QK_TUNE_BSGS_SG: how many 4-wide BSGS accumulator groups —
the a = 0 add row first, then the multiply-accumulate rows — count their
wraps on the scalar unit; QK_TUNE_U64_KMAX: u64 accumulators per
lane) are read once per process, so each variant runs in a child process on
the same GPU, one at a time.  Inputs cover ragged tails (lanes with fewer
iterations than their wave), an unaligned head, and ids that force the rare
lazy-fold wrap branch."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path.insert(0, {root!r})
import sidekick_amd as sk
from oracle import coracle
out = {{}}
bits, cases = {bits}, {cases}
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
print(json.dumps(out))
"""


def _run(env_over, bits, cases):
    env = dict(os.environ, **env_over)
    code = CHILD.format(root=ROOT, bits=bits, cases=cases)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


U32_CASES = [("t32_ragged", 1_000_003, 32, 1), ("t32_small", 77, 32, 3), ("t24", 500_001, 24, 2),
             ("t16", 300_007, 16, 0), ("t12", 200_003, 12, 1), ("t30", 2_000_000, 30, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("sg", [0, 1, 2, 3, 5, 8])
def test_bsgs_scalar_carry_groups(sg):
    res = _run({"QK_TUNE_BSGS_SG": str(sg)}, 32, U32_CASES)
    assert all(res.values()), res


@pytest.mark.gpu
def test_bsgs_scalar_carry_small_grid():
    """Override grid of one workgroup: long per-wave trip counts."""
    code = CHILD.format(root=ROOT, bits=32, cases=[("g1", 3_000_001, 32, 1)]).replace(
        "out = {}", "out = {}\nsk.get_context(0).set_grid(1)")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, QK_TUNE_BSGS_SG="8"),
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert all(json.loads(r.stdout.strip().splitlines()[-1]).values())


@pytest.mark.gpu
@pytest.mark.parametrize("kmax", [20, 40])
def test_u64_lane_split(kmax):
    cases = [("t80", 300_001, 80, 1), ("t40", 200_003, 40, 0), ("t33", 100_001, 33, 1), ("t20", 100_000, 20, 0),
             ("t64", 50_001, 64, 0), ("t200", 20_001, 200, 1)]
    res = _run({"QK_TUNE_U64_KMAX": str(kmax)}, 64, cases)
    assert all(res.values()), res


@pytest.mark.gpu
@pytest.mark.parametrize("sg", [-1, 0, 8, 12, 18])
def test_u64_bsgs_scalar_carry_macs(sg):
    """The u64 baby-step/giant-step kernel (bsgs64.h) with the first sg MACs
    of each wave's tile counting carries on the scalar unit, the rest per
    lane; t = 73..80 (the last giant row partly or fully used)."""
    cases = [("t80", 300_001, 80, 1), ("t73", 100_003, 73, 0), ("t77", 4099, 77, 1), ("t79_tiny", 37, 79, 0)]
    res = _run({"QK_TUNE_BSGS64_SG": str(sg)}, 64, cases)
    assert all(res.values()), res


@pytest.mark.gpu
def test_u64_bsgs_off_matches_chain():
    """The power-chain path the u64 BSGS kernel replaced gives the same sums."""
    res = _run({"QK_TUNE_BSGS64_OFF": "1"}, 64, [("t80", 200_001, 80, 1), ("t75", 3001, 75, 0)])
    assert all(res.values()), res
