"""Parity of the opt-in matrix-core encode variants (mfma8.h u32, mfma64.h
u64) against the oracle, and against the default vector-ALU
kernels on the same large inputs (two independent implementations,
bit-exact).  The variants live only in the opt-in build
libquack_hip_mfma.so (`make -C sidekick_amd/csrc mfma`; the product
libquack_hip.so carries no v_mfma), selected per context with knob
matrix_cores.  test_matrix_core_build_parity runs this module in a child
process with QK_LIB_PATH pointing at that build; in a process on the product
library the module's own tests are skipped."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MFMA_LIB = os.path.join(ROOT, "sidekick_amd", "libquack_hip_mfma.so")
ON_MFMA = os.environ.get("QK_LIB_PATH", "").endswith("libquack_hip_mfma.so")
mfma_only = pytest.mark.skipif(not ON_MFMA, reason="runs in the child process on libquack_hip_mfma.so")


def test_matrix_core_build_parity():
    """The whole module against the opt-in build, in a child process."""
    if ON_MFMA:
        pytest.skip("already the child")
    assert os.path.exists(MFMA_LIB), "build it: make -C sidekick_amd/csrc mfma"
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.abspath(__file__)], cwd=ROOT, env=dict(os.environ, QK_LIB_PATH=MFMA_LIB),
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "failed" not in r.stdout


@pytest.fixture
def matrix_cores():
    from sidekick_amd.quack import get_context
    ctx = get_context(0)
    ctx.set_knob("matrix_cores", 1)
    yield
    ctx.set_knob("matrix_cores", 0)


def dev_u32(a):
    from test_gpu_encode import dev_u32 as f
    return f(a)


def dev_u64(a):
    from test_gpu_encode import dev_u64 as f
    return f(a)


def gpu_state(*a):
    from test_gpu_encode import gpu_state as f
    return f(*a)


# (babies x giants) chain of the matrix-core shape each threshold runs
# (encode.hip enc32_mfma; t > 256: pass 0 is 16 x 16)
def mf_wrap_cfg(t):
    for hi, cfg in ((16, "4x4"), (20, "5x4"), (24, "6x4"), (32, "8x4"), (36, "6x6"), (40, "8x5"), (48, "8x6"),
                    (56, "8x7"), (64, "8x8"), (80, "10x8"), (96, "12x8"), (128, "16x8"), (192, "16x12")):
        if t <= hi:
            return cfg
    return "16x16"


U32_TS = [9, 12, 16, 17, 20, 21, 24, 25, 31, 32, 33, 36, 37, 40, 44, 48, 56, 64, 65, 72, 80, 81, 96, 97, 128,
          129, 160, 192, 193, 256, 257, 300, 512, 513]


@mfma_only
@pytest.mark.parametrize("t", U32_TS)
def test_u32_vs_oracle(matrix_cores, golden, t):
    """Random ids with the shape's lazy-fold wrap ids planted (exact redo
    branch), misaligned starts, a ragged tail."""
    ids = coracle.splitmix_u32(0xC0DE + t, 40_009)
    wraps = np.array(golden["bsgs_wrap_ids"][mf_wrap_cfg(t)], dtype=np.uint32)
    ids[77] = wraps[0]
    ids[5000:5000 + 64 * len(wraps):64] = wraps
    ids[-1] = wraps[-1]
    d = dev_u32(ids)
    for off in (0, 1, 3):
        assert gpu_state(d[off:], t).power_sums() == coracle.encode_u32(ids[off:], t), (t, off)


@mfma_only
@pytest.mark.parametrize("t", [1024])
def test_u32_many_passes(matrix_cores, t):
    ids = coracle.splitmix_u32(0xBEEF, 3_001)
    assert gpu_state(dev_u32(ids), t).power_sums() == coracle.encode_u32(ids, t)


@mfma_only
@pytest.mark.parametrize("n", [0, 1, 63, 64, 255, 256, 257, 4097])
def test_u32_small_and_empty(matrix_cores, n):
    ids = coracle.splitmix_u32(0xE0 + n, n)
    q = gpu_state(dev_u32(ids) if n else dev_u32(np.zeros(0, np.uint32)), 32)
    assert q.power_sums() == coracle.encode_u32(ids, 32) and q.count() == n
    assert q.last_value() == (int(ids[-1]) if n else None)


U64_TS = [9, 16, 17, 24, 32, 33, 48, 49, 64, 65, 72, 80, 81, 96, 160, 161, 200]


@mfma_only
@pytest.mark.parametrize("t", U64_TS)
def test_u64_vs_oracle(matrix_cores, t):
    ids = coracle.splitmix_u64(0xD00D + t, 12_007)
    p = (1 << 64) - 59
    ids[[3, 500, 4097, -1]] = np.array([p - 1, p, (1 << 64) - 1, 0], dtype=np.uint64)   # field edges
    d = dev_u64(ids)
    for off in (0, 1):
        assert gpu_state(d[off:], t, 64).power_sums() == coracle.encode_u64(ids[off:], t), (t, off)


@mfma_only
def test_matches_vector_kernels_at_scale():
    """1e8 u32 ids at t=32 and 2e7 u64 ids at t=80: the matrix-core and the
    vector-ALU encodes agree word for word."""
    import torch
    from sidekick_amd.quack import fill_splitmix, get_context
    ctx = get_context(0)
    for bits, n, t in ((32, 100_000_000, 32), (64, 20_000_000, 80)):
        d = torch.empty(n, dtype=torch.int32 if bits == 32 else torch.int64, device="cuda:0")
        fill_splitmix(ctx, d, 0x5CA1E + bits, 0, bits)
        a = gpu_state(d, t, bits)
        ctx.set_knob("matrix_cores", 1)
        try:
            b = gpu_state(d, t, bits)
        finally:
            ctx.set_knob("matrix_cores", 0)
        assert a.power_sums() == b.power_sums() and a.count() == b.count() == n, bits
        del d
        torch.cuda.empty_cache()


@mfma_only
def test_host_pipeline_accumulates(matrix_cores):
    """encode from host memory runs the accumulate form over chunks."""
    import sidekick_amd as sk
    ids = coracle.splitmix_u32(0xACC, 3_000_017)
    q = sk.PowerSumQuackU32(32)
    q.insert_batch(ids)
    assert q.power_sums() == coracle.encode_u32(ids, 32) and q.count() == len(ids)
