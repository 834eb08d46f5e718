"""The oracle itself: Python big-int vs C restatement vs golden fixtures vs
algebraic known answers.  (CPU only.)  The oracle is parity-unpinned against
the reference crate (absent submodule); these tests pin it by
independent restatements and the algebra."""
import random

import numpy as np
import pytest

from oracle import coracle, quack_oracle as qo


def _state(ids, t, bits):
    q = qo.OracleQuack(t, bits)
    q.insert_all(ids)
    return q


def test_kats_hand_checked(golden):
    for k in golden["kats"]:
        q = _state(k["ids"], k["t"], k["bits"])
        assert q.power_sums == k["expect"]["power_sums"], k["name"]
        assert q.count == k["expect"]["count"]
        assert q.last_value == k["expect"]["last_value"]


def test_c_oracle_matches_golden_streams(golden):
    for s in golden["streams"]:
        if s["bits"] == 32:
            got = coracle.encode_u32_seed(s["seed"], s["n"], s["t"])
            assert got == s["expect"]["power_sums"], (s["n"], s["t"])
            ids = coracle.splitmix_u32(s["seed"], s["n"])
            assert int(ids[-1]) == s["expect"]["last_value"]
        else:
            got = coracle.encode_u64_seed(s["seed"], s["n"], s["t"])
            assert got == [int(v) for v in s["expect"]["power_sums"]], (s["n"], s["t"])


def test_c_oracle_matches_golden_edges(golden):
    for e in golden["edges"]:
        ids = [int(v) for v in e["ids"]]
        if e["bits"] == 32:
            assert coracle.encode_u32(np.array(ids, dtype=np.uint32), e["t"]) == e["expect"]["power_sums"]
        else:
            assert coracle.encode_u64(np.array(ids, dtype=np.uint64), e["t"]) == \
                [int(v) for v in e["expect"]["power_sums"]]


def test_numpy_path_equals_bigint():
    ids = qo.ids_u32(123, 3000)
    assert qo.encode_u32_np(ids, 33) == _state(ids.tolist(), 33, 32).power_sums


def test_splitmix_generators_agree():
    assert (coracle.splitmix_u32(99, 5000, start=77) == qo.ids_u32(99, 5000, start=77)).all()
    assert (coracle.splitmix_u64(99, 5000, start=77) == qo.ids_u64(99, 5000, start=77)).all()
    assert qo.splitmix64_at(99, 80) == int(qo.ids_u64(99, 1, start=80)[0])


@pytest.mark.parametrize("bits", [32, 64])
def test_ids_alias_mod_p(bits):
    p = qo.MOD[bits]
    a = _state([p + 3, 2 ** bits - 1], 6, bits)
    b = _state([3, 2 ** bits - 1 - p], 6, bits)
    assert a.power_sums == b.power_sums
    z = _state([0, p], 5, bits)
    assert z.power_sums == [0] * 5 and z.count == 2


@pytest.mark.parametrize("bits", [32, 64])
def test_additivity(bits):
    rnd = random.Random(bits)
    ids = [rnd.getrandbits(bits) for _ in range(300)]
    whole = _state(ids, 12, bits)
    a = _state(ids[:111], 12, bits)
    b = _state(ids[111:], 12, bits)
    a.add_assign(b)
    assert a.power_sums == whole.power_sums and a.count == whole.count and a.last_value == whole.last_value


@pytest.mark.parametrize("bits", [32, 64])
def test_decode_recovers_drops_with_duplicates(bits):
    rnd = random.Random(5 + bits)
    log = [rnd.getrandbits(bits) for _ in range(2000)]
    drops = sorted(rnd.sample(range(2000), 10))
    log[1500] = log[drops[2]]   # duplicate value later in the log
    sent, recv = _state(log, 16, bits), qo.OracleQuack(16, bits)
    for i, x in enumerate(log):
        if i not in drops:
            recv.insert(x)
    sent.sub_assign(recv)
    assert sent.count == 10
    c = sent.to_coeffs()
    hits = qo.root_test_indices(c, log, qo.MOD[bits])
    assert set(drops) <= set(hits)
    assert 1500 in hits  # every entry congruent to a root is a hit
    if bits == 32:
        assert coracle.to_coeffs_u32(sent.power_sums[:10]) == c
        h, nh = coracle.root_test_u32(c, np.array(log, dtype=np.uint32))
        assert h.tolist() == hits and nh == len(hits)
        assert qo.root_test_u32_np(c, np.array(log, dtype=np.uint32)).tolist() == hits
    else:
        assert coracle.to_coeffs_u64(sent.power_sums[:10]) == c
        h, nh = coracle.root_test_u64(c, np.array(log, dtype=np.uint64))
        assert h.tolist() == hits


def test_golden_decodes_self_consistent(golden):
    for d in golden["decodes"]:
        bits = d["bits"]
        p = qo.MOD[bits]
        assert set(d["drops"]) <= set(d["hits"])
        if d["dup_at"] is not None:
            assert d["dup_at"] in d["hits"]
        coeffs = [int(c) for c in d["coeffs"]]
        assert qo.newton_coeffs([int(v) for v in d["diff_power_sums"]][:d["diff_count"]], p) == coeffs


def test_undecodable(golden):
    u = golden["undecodable"]
    q = _state(u["ids"], u["t"], 32)
    with pytest.raises(ValueError):
        q.to_coeffs()


def test_stop_value_semantics():
    log = [5, 9, 3, 7, 3]
    q = qo.OracleQuack(4)
    q.insert(3)
    c = q.to_coeffs()
    assert qo.root_test_indices(c, log, qo.P32) == [2, 4]
    assert qo.root_test_indices(c, log, qo.P32, stop_value=7) == [2]
    assert qo.root_test_indices(c, log, qo.P32, stop_value=5) == []


def test_all_cores_restatement_matches_scalar():
    """bench.py's all-cores CPU baseline (one partial per thread, merged)
    equals the 1-core loop on the same stream."""
    from oracle import coracle
    for bits, n, t, thr in ((32, 100_003, 32, 7), (32, 5, 16, 8), (64, 20_001, 80, 3)):
        one = (coracle.encode_u32_seed if bits == 32 else coracle.encode_u64_seed)(0xBEEF, n, t, start=11)
        assert coracle.encode_seed_mt(bits, 0xBEEF, n, t, thr, start=11) == one


def test_bench_construct_runs():
    """Reference-shape microbenchmark leg (tools/bench_configs.py micro)."""
    from oracle import coracle
    for bits in (32, 64):
        ns = coracle.bench_construct(bits, 7, 1000, 16, 3)
        assert 0 < ns < 1e6
    assert coracle.bench_construct(32, 7, 1000, 0, 3) == 0
