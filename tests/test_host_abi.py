"""C-ABI library on the CPU: it loads, exports every symbol include/*.h
declares, and its host (per-packet) path — insert / remove / sub_assign /
to_coeffs / eval / bincode — is bit-exact against the oracle.  No GPU calls.
Reads like the reference callers (media_client.rs:247-323)."""
import ctypes as C
import os
import random
import re

import numpy as np
import pytest

import sidekick_amd as sk
from sidekick_amd._lib import LIB_PATH, SIGNATURES, lib
from oracle import coracle, quack_oracle as qo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            src = open(os.path.join(inc, fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            syms |= set(re.findall(r"\b(qk_[a-z0-9_]+)\s*\(", src))
    return syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB_PATH)
    L = C.CDLL(LIB_PATH)
    declared = header_symbols()
    assert len(declared) > 40
    for s in sorted(declared):
        assert hasattr(L, s), f"{s} declared in include/ but not exported"
    assert declared == set(SIGNATURES), "ctypes binding out of sync with the header"
    assert lib().qk_version().decode().startswith("quack-hip")


def Q(bits, t):
    return (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(t)


def test_kats(golden):
    for k in golden["kats"]:
        q = Q(k["bits"], k["t"])
        for i in k["ids"]:
            q.insert(i)
        assert q.power_sums() == k["expect"]["power_sums"]
        assert q.count() == k["expect"]["count"]
        assert q.last_value() == k["expect"]["last_value"]


def test_edges(golden):
    for e in golden["edges"]:
        q = Q(e["bits"], e["t"])
        for i in e["ids"]:
            q.insert(int(i))
        assert q.power_sums() == [int(v) for v in e["expect"]["power_sums"]]
        assert q.last_value() == int(e["expect"]["last_value"])


def test_stream_u32_1000(golden):
    s = [s for s in golden["streams"] if s["bits"] == 32 and s["n"] == 1000 and s["t"] == 32][0]
    q = sk.PowerSumQuackU32(32)
    for i in qo.ids_u32(s["seed"], s["n"]).tolist():
        q.insert(i)
    assert q.power_sums() == s["expect"]["power_sums"]


def test_stream_u64_1000(golden):
    s = [s for s in golden["streams"] if s["bits"] == 64 and s["n"] == 1000][0]
    q = sk.PowerSumQuackU64(80)
    for i in qo.ids_u64(s["seed"], s["n"]).tolist():
        q.insert(int(i))
    assert q.power_sums() == [int(v) for v in s["expect"]["power_sums"]]


@pytest.mark.parametrize("bits", [32, 64])
def test_insert_remove_every_threshold_vs_oracle(bits):
    """The host insert walks the powers as four interleaved chains for t >= 8
    (u32 on an AVX-512 CPU: eight chains in the lanes of a zmm): every
    threshold 1..41 (each tail length) plus long walks, and ids at the field
    edges (0, 1, p - 1, p, p + 1, 2^w - 1) match the oracle; remove() undoes
    insert."""
    rnd = random.Random(5 * bits)
    P = qo.MOD[bits]
    edge = [0, 1, 2, P - 1, P, P + 1, (1 << bits) - 1, (1 << bits) - 2, 1 << (bits - 1)]
    for t in list(range(1, 42)) + [63, 64, 65, 80, 257, 1024]:
        ids = edge + [rnd.getrandbits(bits) for _ in range(30)]
        q = Q(bits, t)
        oq = qo.OracleQuack(t, bits)
        for i in ids:
            q.insert(i)
        oq.insert_all(ids)
        assert q.power_sums() == oq.power_sums, t
        for i in ids[::2]:
            q.remove(i)
        rest = ids[1::2]
        assert q.power_sums() == Q_from(rest, bits, t).power_sums(), t
        assert q.count() == len(rest)


@pytest.mark.parametrize("bits", [32, 64])
def test_media_client_flow(bits):
    """media_client.rs:247-323 end to end on the host path: the receiver's
    cumulative quACK minus the proxy's, to_coeffs, eval == 0 over the log,
    then remove() of each missing id leaves a sketch equal to the proxy's."""
    rnd = random.Random(bits)
    t = 20
    log = [rnd.getrandbits(bits) for _ in range(500)]
    drops = set(rnd.sample(range(499), 12))
    mine, proxy = Q(bits, t), Q(bits, t)
    for i, x in enumerate(log):
        mine.insert(x)
        if i not in drops:
            proxy.insert(x)
    diff = mine.clone()
    diff.sub_assign(proxy)
    assert diff.count() == len(drops)
    assert diff.last_value() == mine.last_value()   # sub keeps self.last_value
    coeffs = diff.to_coeffs()
    missing = [x for x in log if sk.arithmetic.eval(coeffs, x).value() == 0]
    assert sorted(missing) == sorted(log[i] for i in drops)
    for x in missing:
        mine.remove(x)
    assert mine.power_sums() == proxy.power_sums() and mine.count() == proxy.count()
    oq = qo.OracleQuack(t, bits)
    oq.insert_all(log)
    assert oq.power_sums == Q_from(log, bits, t).power_sums()


def Q_from(ids, bits, t):
    q = Q(bits, t)
    for i in ids:
        q.insert(i)
    return q


@pytest.mark.parametrize("bits", [32, 64])
def test_to_coeffs_and_eval_match_oracle(bits):
    rnd = random.Random(11 * bits)
    for d in (1, 2, 7, 17, 24, 31, 32, 33, 100, 301):   # d > 16: the AVX-512 Newton dot product (u32)
        q = Q(bits, max(32, d))
        for _ in range(d):
            q.insert(rnd.getrandbits(bits))
        c = q.to_coeffs()
        assert list(c) == qo.newton_coeffs(q.power_sums()[:d], qo.MOD[bits])
        for _ in range(20):
            x = rnd.getrandbits(bits)
            assert sk.arithmetic.eval(c, x).value() == qo.poly_eval(list(c), x, qo.MOD[bits])


def test_errors():
    q = sk.PowerSumQuackU32(0)
    with pytest.raises(sk.QuackError):
        q.insert(1)
    a, b = sk.PowerSumQuackU32(4), sk.PowerSumQuackU32(5)
    with pytest.raises(sk.QuackError):
        a.sub_assign(b)
    u = sk.PowerSumQuackU32(8)
    for i in range(1, 10):
        u.insert(i)
    with pytest.raises(sk.UndecodableError):
        u.to_coeffs()
    e = sk.PowerSumQuackU32(8)
    assert e.to_coeffs() == []
    assert sk.arithmetic.eval(e.to_coeffs(), 5).value() == 1   # P = 1 has no roots


def test_count_wraps():
    q = sk.PowerSumQuackU32(2)
    q.remove(9)
    assert q.count() == 0xFFFFFFFF
    q.insert(9)
    assert q.count() == 0 and q.power_sums() == [0, 0]


@pytest.mark.parametrize("bits", [32, 64])
def test_bincode_roundtrip_and_layout(bits):
    q = Q(bits, 3)
    assert q.serialize() == (3).to_bytes(8, "little") + b"\0" * (3 * bits // 8) + b"\0" + b"\0" * 4
    for i in (1, 2, 3):
        q.insert(i)
    b = q.serialize()
    w = bits // 8
    assert b[:8] == (3).to_bytes(8, "little")
    assert [int.from_bytes(b[8 + w * k: 8 + w * (k + 1)], "little") for k in range(3)] == [6, 14, 36]
    assert b[8 + 3 * w] == 1 and int.from_bytes(b[9 + 3 * w: 9 + 4 * w], "little") == 3
    assert int.from_bytes(b[-4:], "little") == 3
    r = type(q).deserialize(b)
    assert r == q
    with pytest.raises(sk.QuackError):
        type(q).deserialize(b[:-1])


def test_merge_partial_roundtrip():
    from sidekick_amd import dist as skd
    rnd = random.Random(3)
    for bits in (32, 64):
        ids = [rnd.getrandbits(bits) for _ in range(200)]
        whole = Q_from(ids, bits, 9)
        a, b = Q_from(ids[:50], bits, 9), Q_from(ids[50:], bits, 9)
        pa, pb = skd.state_to_partial(a), skd.state_to_partial(b)
        k = skd.reduce_words(9, bits)
        s = pa.copy()
        s[:k] += pb[:k]
        S, cnt = skd.fold_partial_sum(s, 9, bits)
        assert S == whole.power_sums() and cnt == 200
        from sidekick_amd.quack import merge_partial
        m = Q(bits, 9)
        merge_partial(m, s, True, ids[-1])
        assert m == whole


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("n", [1, 7, 31, 32, 33, 1001])
def test_decode_host_edges_and_ragged(bits, n):
    """Host candidate scan (AVX-512 lanes on such CPUs, 32 candidates per
    iteration): logs of every ragged length, ids >= p aliasing small ids, id 0
    as a root, and the stop at last_value inside the scan."""
    import numpy as np
    from oracle import quack_oracle as qo
    P = qo.MOD[bits]
    rng = np.random.default_rng(n + bits)
    log = (qo.ids_u32 if bits == 32 else qo.ids_u64)(0xE0 + n, n, 0)
    dt = np.uint32 if bits == 32 else np.uint64
    edge = np.array([0, 1, 3, P, P + 1, P + 3, 2**bits - 1, P - 1], dtype=dt)
    log[rng.choice(n, min(n, len(edge)), replace=False)] = edge[:min(n, len(edge))]
    for drops in ([0, 1, 3], [P - 1, 7, 11], [int(log[-1])]):
        diff = (sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64)(16)
        for v in drops:
            diff.insert(v)
        for stop in (False, True):
            got = diff.decode_host(log, stop_at_last=stop)
            want = qo.root_test_indices(diff.to_coeffs(), log.tolist(), P,
                                        stop_value=diff.last_value() if stop else None)
            assert got == want, (n, drops, stop)


@pytest.mark.parametrize("bits,d,stop", [(32, 5, False), (32, 32, True), (64, 20, True), (64, 1, False)])
def test_decode_host_matches_oracle(bits, d, stop):
    """qk_*_decode_host (the receiver's short-log path) vs the oracle's root
    test: every entry congruent to a dropped id, in log order, cut at the
    first entry equal to last_value when stopping."""
    import numpy as np
    from oracle import quack_oracle as qo
    rng = np.random.default_rng(d + bits)
    n = 3000
    log = (qo.ids_u32 if bits == 32 else qo.ids_u64)(0xD0 + d, n, 0)
    log[rng.choice(n, 4, replace=False)] = log[rng.choice(n, 4, replace=False)]   # duplicates
    drops = sorted(rng.choice(n, d, replace=False).tolist())
    Q = sk.PowerSumQuackU32 if bits == 32 else sk.PowerSumQuackU64
    diff = Q(32)
    for i in drops:
        diff.insert(int(log[i]))
    got = diff.decode_host(log, stop_at_last=stop)
    want = qo.root_test_indices(diff.to_coeffs(), log.tolist(), qo.MOD[bits],
                                stop_value=diff.last_value() if stop else None)
    assert got == want and len(got) >= (1 if stop else d)
    assert Q(8).decode_host(log) == []                     # empty difference: nothing missing
    big = Q(2)
    for v in log[:3]:
        big.insert(int(v))
    with pytest.raises(sk.UndecodableError):
        big.decode_host(log)
