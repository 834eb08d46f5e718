"""Property-based parity (hypothesis): random shapes, thresholds, id
distributions and misalignments against the oracle.  The CPU half drives the
host ABI (per-packet insert/remove, sub/merge, bincode, to_coeffs/eval,
host decode); the -m gpu half drives the batch kernels (encode u32/u64, root
test u32/u64) through the C ABI.  Example counts are bounded so each test
finishes in seconds; failures print the minimal example."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import sidekick_amd as sk
from oracle import coracle, quack_oracle as qo

P = {32: qo.MOD[32], 64: qo.MOD[64]}
SETTINGS = dict(deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


def edge_ids(bits):
    p = P[bits]
    return st.sampled_from([0, 1, 2, p - 2, p - 1, p, p + 1, (1 << bits) - 1, (1 << bits) - 2, 1 << (bits - 1)])


def ids_strategy(bits, max_size):
    return st.lists(st.one_of(st.integers(0, (1 << bits) - 1), edge_ids(bits)), max_size=max_size)


def Q(bits, t):
    return (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)


# ---------------------------------------------------------------- CPU / host ABI
@settings(max_examples=60, **SETTINGS)
@given(bits=st.sampled_from([32, 64]), t=st.integers(1, 70), data=st.data())
def test_host_insert_remove_sub_merge(bits, t, data):
    a_ids = data.draw(ids_strategy(bits, 40))
    b_ids = data.draw(ids_strategy(bits, 40))
    qa, qb = Q(bits, t), Q(bits, t)
    for i in a_ids:
        qa.insert(i)
    for i in b_ids:
        qb.insert(i)
    oa = qo.OracleQuack(t, bits)
    oa.insert_all(a_ids)
    assert qa.power_sums() == oa.power_sums and qa.count() == len(a_ids) & 0xFFFFFFFF
    # merge = the concatenated stream; sub undoes it; remove undoes insert
    m = qa.clone()
    m.merge(qb)
    both = Q(bits, t)
    for i in a_ids + b_ids:
        both.insert(i)
    assert m.power_sums() == both.power_sums() and m.count() == both.count()
    if b_ids:
        assert m.last_value() == b_ids[-1]
    m.sub_assign(qb)
    assert m.power_sums() == qa.power_sums() and m.count() == qa.count()
    for i in b_ids:
        both.remove(i)
    assert both.power_sums() == qa.power_sums()


@settings(max_examples=60, **SETTINGS)
@given(bits=st.sampled_from([32, 64]), t=st.integers(1, 40), data=st.data())
def test_host_bincode_round_trip(bits, t, data):
    q = Q(bits, t)
    for i in data.draw(ids_strategy(bits, 30)):
        q.insert(i)
    raw = q.serialize()
    back = type(q).deserialize(raw)
    assert back.power_sums() == q.power_sums() and back.count() == q.count()
    assert back.last_value() == q.last_value()
    assert len(raw) == 8 + (bits // 8) * t + 1 + (bits // 8 if q.last_value() is not None else 0) + 4


@settings(max_examples=50, **SETTINGS)
@given(bits=st.sampled_from([32, 64]), data=st.data())
def test_host_decode_recovers_missing(bits, data):
    """media_client.rs:295-313 on the host: the difference of two sketches
    decodes to exactly the log entries congruent to a missing id."""
    t = data.draw(st.integers(1, 40))
    log = data.draw(st.lists(st.integers(0, (1 << bits) - 1), min_size=1, max_size=200, unique=True))
    d = data.draw(st.integers(0, min(t, len(log))))
    drop = set(data.draw(st.lists(st.integers(0, len(log) - 1), min_size=d, max_size=d, unique=True)))
    sent, recv = Q(bits, t), Q(bits, t)
    for k, x in enumerate(log):
        sent.insert(x)
        if k not in drop:
            recv.insert(x)
    diff = sent.clone()
    diff.sub_assign(recv)
    assert diff.count() == len(drop)
    pos = diff.decode_host(np.array(log, dtype=np.uint32 if bits == 32 else np.uint64))
    miss = {log[k] % P[bits] for k in drop}
    assert pos == [k for k, x in enumerate(log) if x % P[bits] in miss]


# ---------------------------------------------------------------- GPU kernels
@pytest.mark.gpu
@settings(max_examples=40, **SETTINGS)
@given(bits=st.sampled_from([32, 64]), t=st.integers(1, 160), n=st.integers(0, 70_000),
       off=st.integers(0, 7), seed=st.integers(0, 2**32 - 1))
def test_gpu_encode_random_shapes(bits, t, n, off, seed):
    import torch
    gen = coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64
    ids = gen(seed, n + off)
    rng = np.random.default_rng(seed)
    if n:
        k = rng.integers(0, n + off, size=min(8, n + off))   # sprinkle field-edge ids
        e = np.array([P[bits] - 1, P[bits], (1 << bits) - 1, 0], dtype=ids.dtype)
        ids[k] = e[np.arange(len(k)) % 4]
    dt = torch.int32 if bits == 32 else torch.int64
    d = torch.from_numpy(ids.view(np.int32 if bits == 32 else np.int64)).to("cuda")[off:]
    q = Q(bits, t)
    q.insert_batch(d)
    want = coracle.encode_u32(ids[off:], t) if bits == 32 else coracle.encode_u64(ids[off:], t)
    assert q.power_sums() == want
    assert q.count() == n and q.last_value() == (int(ids[-1]) if n else None)
    assert d.dtype == dt


@pytest.mark.gpu
@settings(max_examples=30, **SETTINGS)
@given(bits=st.sampled_from([32, 64]), d=st.integers(1, 64), n=st.integers(1, 40_000),
       seed=st.integers(0, 2**32 - 1), stop=st.booleans())
def test_gpu_root_test_random(bits, d, n, seed, stop):
    import torch
    gen = coracle.splitmix_u32 if bits == 32 else coracle.splitmix_u64
    log = gen(seed, n)
    rng = np.random.default_rng(seed)
    roots = rng.choice(n, size=min(d, n), replace=False)
    q = Q(bits, len(roots))
    for i in roots:
        q.insert(int(log[i]))
    c = q.to_coeffs()
    stop_value = int(log[rng.integers(0, n)]) if stop else None
    dlog = torch.from_numpy(log.view(np.int32 if bits == 32 else np.int64)).to("cuda")
    got = q.root_test(c, dlog, stop_value=stop_value)
    want, _ = (coracle.root_test_u32 if bits == 32 else coracle.root_test_u64)(c, log)
    want = want.tolist()
    if stop_value is not None:
        first = int(np.nonzero(log == np.array(stop_value, dtype=log.dtype))[0][0])
        want = [w for w in want if w < first]
    assert got == want
