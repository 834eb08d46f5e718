"""Host root finding (qk_u32_roots / qk_u64_roots, roots.cpp) against the
oracle: the roots of diff.to_coeffs() are exactly the residues x mod p of the
missing ids, so the root test (media_client.rs:306-313, eval(&coeffs, x) ==
0) can be a set-membership scan.  Coefficients come from the oracle's
Newton identities (oracle/quack_oracle.py OracleQuack.to_coeffs); the found
roots are checked by the oracle's polynomial evaluation too.  CPU only."""
import ctypes as C
import random

import numpy as np
import pytest

from oracle import quack_oracle as qo
from sidekick_amd._lib import QK_E_CAPACITY, lib

P = {32: qo.MOD[32], 64: qo.MOD[64]}


def roots(coeffs, bits):
    f = lib().qk_u32_roots if bits == 32 else lib().qk_u64_roots
    T = C.c_uint32 if bits == 32 else C.c_uint64
    d = len(coeffs)
    c = (T * max(d, 1))(*[int(v) for v in coeffs])
    out = (T * max(d, 1))()
    k = C.c_uint32()
    assert f(c, d, out, d, C.byref(k)) == 0
    return [int(v) for v in out[:k.value]]


def coeffs_of(ids, bits):
    q = qo.OracleQuack(max(len(ids), 1), bits)
    for x in ids:
        q.insert(int(x))
    return q.to_coeffs()


def poly_mul(a, b, p):
    """Coefficients high degree first (monic convention of to_coeffs, leading 1 implicit)."""
    A, B = [1] + list(a), [1] + list(b)
    out = [0] * (len(A) + len(B) - 1)
    for i, x in enumerate(A):
        for j, y in enumerate(B):
            out[i + j] = (out[i + j] + x * y) % p
    return out[1:]


def nonresidue(p, rng):
    while True:
        n = rng.randrange(2, p)
        if pow(n, (p - 1) // 2, p) == p - 1:
            return n


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 17, 32, 33, 64, 100])
def test_roots_of_missing_set(bits, k):
    rng = random.Random(k * 1000 + bits)
    ids = [rng.randrange(1 << bits) for _ in range(k)]
    got = roots(coeffs_of(ids, bits), bits)
    assert got == sorted({x % P[bits] for x in ids})


@pytest.mark.parametrize("bits", [32, 64])
def test_roots_edges_duplicates_and_zero(bits):
    p = P[bits]
    top = (1 << bits) - 1
    ids = [0, 1, p - 1, p, p + 1, top, 1, 1, p - 1, 12345]      # p aliases 0, p+1 aliases 1; repeats
    got = roots(coeffs_of(ids, bits), bits)
    assert got == sorted({x % p for x in ids})
    assert roots([], bits) == []
    assert roots(coeffs_of([0, 0, 0], bits), bits) == [0]            # z^3


@pytest.mark.parametrize("bits", [32, 64])
def test_roots_of_non_splitting_polynomial(bits):
    """P = (linear factors) x (irreducible quadratics): only the GF(p) roots."""
    p = P[bits]
    rng = random.Random(bits)
    lin = [rng.randrange(p) for _ in range(9)]
    c = coeffs_of(lin, bits)
    for _ in range(3):
        n = nonresidue(p, rng)
        s = rng.randrange(p)
        # (z - s)^2 - n = z^2 - 2 s z + s^2 - n, irreducible since n is a non-residue
        c = poly_mul(c, [(-2 * s) % p, (s * s - n) % p], p)
    got = roots(c, bits)
    assert got == sorted(set(lin))
    for r in got:
        assert qo.poly_eval(c, r, p) == 0


@pytest.mark.parametrize("bits", [32, 64])
def test_roots_random_polynomials_match_evaluation(bits):
    """Random (mostly non-splitting) coefficient vectors: every reported root
    evaluates to 0, and planted roots are found."""
    p = P[bits]
    rng = random.Random(99 + bits)
    for d in (1, 2, 3, 7, 20):
        for _ in range(4):
            planted = [rng.randrange(p) for _ in range(rng.randrange(0, 3))]
            rest = [rng.randrange(p) for _ in range(d)]
            c = poly_mul(coeffs_of(planted, bits), rest, p) if planted else rest
            got = roots(c, bits)
            assert set(planted) <= set(got)
            assert all(qo.poly_eval(c, r, p) == 0 for r in got)
            assert len(got) <= len(c) and got == sorted(set(got))


def test_roots_capacity_and_args():
    c = coeffs_of([5, 6, 7], 32)
    T = C.c_uint32
    out = (T * 3)()
    k = C.c_uint32()
    assert lib().qk_u32_roots((T * 3)(*c), 3, out, 2, C.byref(k)) == QK_E_CAPACITY and k.value == 3
    assert lib().qk_u32_roots((T * 3)(*c), 3, out, 3, C.byref(k)) == 0 and list(out) == [5, 6, 7]
    assert lib().qk_u32_roots(None, 3, out, 3, C.byref(k)) != 0


def test_roots_large_degree_u32():
    rng = np.random.default_rng(5)
    ids = rng.integers(0, 1 << 32, size=300, dtype=np.uint64).tolist()
    assert roots(coeffs_of(ids, 32), 32) == sorted({x % P[32] for x in ids})


@pytest.mark.parametrize("k", [300, 700])
def test_roots_large_degree_u64(k):
    """Degrees past the IFMA products' limit (roots.cpp IFMA_MAX = 640) take
    the other vector path; both must find every root."""
    rng = np.random.default_rng(k)
    ids = [int(v) for v in rng.integers(0, 1 << 63, size=k, dtype=np.uint64)]
    ids += [P[64] - 1 - i for i in range(8)]   # coefficients near p: the largest column sums
    assert roots(coeffs_of(ids, 64), 64) == sorted({x % P[64] for x in ids})


@pytest.mark.parametrize("bits", [32, 64])
def test_roots_repeated_and_clustered_classes(bits):
    """Multiplicities up to 5 and many roots sharing a splitting class (roots
    r, r * zeta^L' ... fall in related classes): still exactly the distinct
    roots."""
    p = P[bits]
    rng = random.Random(7 + bits)
    base = [rng.randrange(1, p) for _ in range(12)]
    ids = []
    for i, r in enumerate(base):
        ids += [r] * (1 + i % 5)
    ids += [(base[0] + j) % p for j in range(1, 20)]   # a run of consecutive residues
    assert roots(coeffs_of(ids, bits), bits) == sorted({x % p for x in ids})
