"""CPU oracle for the quACK power-sum path — TEST INFRASTRUCTURE ONLY.

This module is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product
(``sidekick_amd`` + ``libquack_hip.so``) never imports, links or executes
anything under ``oracle/``.

PARITY STATUS: **parity unpinned** against the reference implementation.
The algorithm lives in the ``quack`` crate (git submodule ``ygina/quack``,
``/root/reference/.gitmodules:9-11``), which is an empty directory in
``/root/reference`` with no recoverable pinned revision (``Cargo.lock`` is
git-ignored, ``/root/reference/.gitignore:7``); no Rust toolchain exists here.
The reference tree holds no test vectors for this path.  This
restatement follows

  * the algebra forced once the prime is fixed (power sums, Newton's
    identities, Horner evaluation of the monic polynomial), and
  * the crate's published constants/semantics as recorded in DESIGN.md §1
    (p32 = 2^32-5, p64 = 2^64-59, ids reduced mod p, wrapping u32 count,
    last_value = last inserted id, sub keeps self.last_value),

and is pinned by algebraic known-answer tests (tests/test_oracle.py) plus the
caller contracts visible in the reference tree:

  * ``PowerSumQuackU32::new(threshold)``  sidekick/src/sidekick.rs:32
  * ``quack.insert(id)``                  sidekick/src/sidekick.rs:42, sidekick_multi.rs:82
  * ``my_quack.remove(id)``               media_integration/media/src/bin/media_client.rs:319
  * ``diff.sub_assign(quack)``            media_client.rs:296
  * ``diff.to_coeffs()``                  media_client.rs:304
  * ``arithmetic::eval(&coeffs, id).value() == 0``   media_client.rs:310
  * ``count()`` / ``last_value()``        media_client.rs:231-233,259-260

Everything here is plain Python integers (obviously correct, slow) with a
numpy fast path for u32 encode (products < 2^64 fit uint64 exactly).
"""
from __future__ import annotations

import numpy as np

P32 = 4_294_967_291          # 2^32 - 5, largest 32-bit prime ([RECALL])
P64 = 18_446_744_073_709_551_557  # 2^64 - 59, largest 64-bit prime ([RECALL])
MOD = {32: P32, 64: P64}
MASK = {32: (1 << 32) - 1, 64: (1 << 64) - 1}

GAMMA = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


# --------------------------------------------------------------------------
# Synthetic identifier streams: counter-based splitmix64.
# id_i = mix(seed + (i+1)*GAMMA); u32 ids are the high 32 bits.
# Mirrors rand::thread_rng().gen::<u32>() (media_client.rs:105) in
# distribution (uniform over the full type range), not in values.
# --------------------------------------------------------------------------
def splitmix64_at(seed: int, i: int) -> int:
    z = (seed + (i + 1) * GAMMA) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def splitmix64_np(seed: int, start: int, n: int) -> np.ndarray:
    """Vectorised splitmix64 outputs for indices [start, start+n) as uint64."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed & _M64) + i * np.uint64(GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def ids_u32(seed: int, n: int, start: int = 0) -> np.ndarray:
    return (splitmix64_np(seed, start, n) >> np.uint64(32)).astype(np.uint32)


def ids_u64(seed: int, n: int, start: int = 0) -> np.ndarray:
    return splitmix64_np(seed, start, n)


# --------------------------------------------------------------------------
# The sketch (restatement of quack::PowerSumQuack{U32,U64}).
# --------------------------------------------------------------------------
class OracleQuack:
    """Power-sum quACK over GF(p).  S[k-1] = sum x_i^k (mod p), k = 1..t."""

    def __init__(self, threshold: int, bits: int = 32):
        if bits not in MOD:
            raise ValueError("bits must be 32 or 64")
        self.bits = bits
        self.p = MOD[bits]
        self.threshold = int(threshold)
        self.power_sums = [0] * self.threshold
        self.count = 0            # wrapping u32
        self.last_value = None    # Option<id>

    def clone(self) -> "OracleQuack":
        q = OracleQuack(self.threshold, self.bits)
        q.power_sums = list(self.power_sums)
        q.count = self.count
        q.last_value = self.last_value
        return q

    # insert: sidekick.rs:42 ; x = id mod p, then S_k += x^k
    def insert(self, ident: int) -> None:
        if self.threshold == 0:
            raise ValueError("insert into a threshold-0 quACK")
        p = self.p
        x = ident % p
        y = x
        for k in range(self.threshold):
            self.power_sums[k] = (self.power_sums[k] + y) % p
            y = (y * x) % p
        self.count = (self.count + 1) & 0xFFFFFFFF
        self.last_value = ident

    # remove: media_client.rs:319 ; last_value unchanged
    def remove(self, ident: int) -> None:
        if self.threshold == 0:
            raise ValueError("remove from a threshold-0 quACK")
        p = self.p
        x = ident % p
        y = x
        for k in range(self.threshold):
            self.power_sums[k] = (self.power_sums[k] - y) % p
            y = (y * x) % p
        self.count = (self.count - 1) & 0xFFFFFFFF

    def insert_all(self, ids) -> None:
        for i in ids:
            self.insert(int(i))

    # sub_assign: media_client.rs:296 ; keeps self.last_value
    def sub_assign(self, rhs: "OracleQuack") -> None:
        if rhs.threshold != self.threshold or rhs.bits != self.bits:
            raise ValueError("threshold mismatch")
        p = self.p
        self.power_sums = [(a - b) % p for a, b in zip(self.power_sums, rhs.power_sums)]
        self.count = (self.count - rhs.count) & 0xFFFFFFFF

    # merge of disjoint streams (additivity); last_value from rhs
    # when rhs is non-empty (rhs is the stream-order-later shard).
    def add_assign(self, rhs: "OracleQuack") -> None:
        if rhs.threshold != self.threshold or rhs.bits != self.bits:
            raise ValueError("threshold mismatch")
        p = self.p
        self.power_sums = [(a + b) % p for a, b in zip(self.power_sums, rhs.power_sums)]
        self.count = (self.count + rhs.count) & 0xFFFFFFFF
        if rhs.last_value is not None:
            self.last_value = rhs.last_value

    # to_coeffs: media_client.rs:304 ; Newton's identities
    def to_coeffs(self) -> list:
        d = self.count
        if d > self.threshold:
            raise ValueError("undecodable: count exceeds threshold")
        return newton_coeffs(self.power_sums[:d], self.p)

    # decode_with_log: to_coeffs + root test over the log, in log order.
    def decode_with_log(self, log) -> list:
        if self.count == 0:
            return []
        c = self.to_coeffs()
        return [int(x) for x in log if poly_eval(c, int(x), self.p) == 0]


def newton_coeffs(S, p: int) -> list:
    """c_1..c_d of prod (z - x_i) from power sums S_1..S_d (all mod p)."""
    d = len(S)
    c = [0] * d
    for i in range(d):
        acc = S[i]
        for j in range(i):
            acc += S[j] * c[i - j - 1]
        c[i] = (-acc * pow(i + 1, p - 2, p)) % p
    return c


def poly_eval(coeffs, x: int, p: int) -> int:
    """arithmetic::eval (media_client.rs:310): Horner on the monic poly
    z^d + c_1 z^{d-1} + ... + c_d.  d == 0 -> 1 (never a root)."""
    d = len(coeffs)
    if d == 0:
        return 1
    xm = x % p
    r = xm
    for i in range(d - 1):
        r = ((r + coeffs[i]) * xm) % p
    return (r + coeffs[d - 1]) % p


def root_test_indices(coeffs, log, p: int, stop_value=None) -> list:
    """Positions i (log order) with P(log[i]) == 0.  With stop_value, stop at
    the first i with log[i] == stop_value (media_client.rs:306-309)."""
    out = []
    for i, x in enumerate(log):
        x = int(x)
        if stop_value is not None and x == stop_value:
            break
        if poly_eval(coeffs, x, p) == 0:
            out.append(i)
    return out


# --------------------------------------------------------------------------
# numpy fast path (u32 only): exact because y, x < 2^32 -> y*x < 2^64.
# --------------------------------------------------------------------------
def encode_u32_np(ids: np.ndarray, t: int, chunk: int = 1 << 22) -> list:
    ids = np.asarray(ids, dtype=np.uint32)
    p = np.uint64(P32)
    S = [0] * t
    for s in range(0, len(ids), chunk):
        x = ids[s:s + chunk].astype(np.uint64) % p
        y = x.copy()
        for k in range(t):
            S[k] = (S[k] + int(y.sum(dtype=np.uint64) % p)) % P32
            if k + 1 < t:
                y = (y * x) % p
    return S


def encode_u64_py(ids, t: int) -> list:
    S = [0] * t
    for v in ids:
        x = int(v) % P64
        y = x
        for k in range(t):
            S[k] = (S[k] + y) % P64
            y = (y * x) % P64
    return S


def root_test_u32_np(coeffs, log: np.ndarray, chunk: int = 1 << 22) -> np.ndarray:
    """Vectorised P(x) == 0 test over a u32 log; returns hit positions."""
    log = np.asarray(log, dtype=np.uint32)
    p = np.uint64(P32)
    d = len(coeffs)
    hits = []
    if d == 0:
        return np.zeros(0, dtype=np.int64)
    cs = [np.uint64(c) for c in coeffs]
    for s in range(0, len(log), chunk):
        x = log[s:s + chunk].astype(np.uint64) % p
        r = x.copy()
        for i in range(d - 1):
            r = ((r + cs[i]) % p * x) % p
        r = (r + cs[d - 1]) % p
        hits.append(np.nonzero(r == 0)[0].astype(np.int64) + s)
    return np.concatenate(hits) if hits else np.zeros(0, dtype=np.int64)


# --------------------------------------------------------------------------
# Sniff loop over a batch of captured packets (sidekick/src/sidekick.rs:76-124,
# buffer.rs:6-7,80-106), applied literally, packet by packet.
# --------------------------------------------------------------------------
ID_OFFSET = 63
BUFFER_SIZE = ID_OFFSET + 4
PACKET_HOST, PACKET_OTHERHOST, PACKET_OUTGOING = 0, 3, 4
ETH_P_IP_BE = 0x0008  # (libc::ETH_P_IP as u16).to_be() read as a little-endian u16
IPPROTO_UDP = 17


def sniff_batch(q: "OracleQuack", bufs, pkttype=None, protocol_be=None, lens=None, my_ipv4=None):
    """Apply the sniff loop to records bufs[i] (uint8 rows).  Returns
    (q, stats) where q may be a fresh sketch if a reset happened."""
    stats = {"inserted": 0, "discarded": 0, "resets": 0, "filtered": 0, "last_reset_index": -1}
    n = len(bufs)
    for i in range(n):
        buf = bufs[i]
        pt = PACKET_HOST if pkttype is None else int(pkttype[i])
        proto = ETH_P_IP_BE if protocol_be is None else int(protocol_be[i])
        ln = BUFFER_SIZE if lens is None else int(lens[i])
        if pt not in (PACKET_HOST, PACKET_OTHERHOST):      # :78-80
            stats["filtered"] += 1
            continue
        if proto != ETH_P_IP_BE:                           # :81-84
            stats["filtered"] += 1
            continue
        if int(buf[23]) != IPPROTO_UDP:                    # :85-88
            stats["filtered"] += 1
            continue
        if my_ipv4 is not None and [int(b) for b in buf[30:34]] == list(my_ipv4):  # :92-96
            stats["discarded"] += stats["inserted"]
            stats["inserted"] = 0
            stats["resets"] += 1
            stats["last_reset_index"] = i
            q = OracleQuack(q.threshold, q.bits)
            continue
        if ln != BUFFER_SIZE:                              # :99-102
            stats["filtered"] += 1
            continue
        ident = int.from_bytes(bytes(int(b) for b in buf[ID_OFFSET:ID_OFFSET + 4]), "big")  # buffer.rs:99-106
        q.insert(ident)
        stats["inserted"] += 1
    return q, stats


def addr_key(buf) -> bytes:
    """UdpParser::parse_addr_key (buffer.rs:91-95)."""
    b = [int(v) for v in buf]
    return bytes([b[26], b[27], b[28], b[29], b[34], b[35], b[30], b[31], b[32], b[33], b[36], b[37]])


def sniff_multi_batch(table: dict, threshold: int, bufs, pkttype=None, protocol_be=None, lens=None, my_addr=None):
    """The SidekickMulti sniff loop over a batch, literally:
    process_one_packet (sidekick_multi.rs:101-143), Insert -> SidekickMulti::
    insert (:65-90), Reset -> `senders = HashMap::new()` (:205 in
    start_sidekick_multi, :265 in start_sidekick_multi_frequency_pkts: every
    flow is wiped, not only the reset key's entry).  table: AddrKey ->
    OracleQuack, updated in place."""
    stats = {"inserted": 0, "discarded": 0, "resets": 0, "filtered": 0, "last_reset_index": -1}
    for i in range(len(bufs)):
        buf = bufs[i]
        pt = PACKET_HOST if pkttype is None else int(pkttype[i])
        proto = ETH_P_IP_BE if protocol_be is None else int(protocol_be[i])
        ln = BUFFER_SIZE if lens is None else int(lens[i])
        if pt not in (PACKET_HOST, PACKET_OTHERHOST) or proto != ETH_P_IP_BE or int(buf[23]) != IPPROTO_UDP:
            stats["filtered"] += 1
            continue
        key = addr_key(buf)
        if my_addr is not None and list(key[6:12]) == list(my_addr):
            stats["resets"] += 1
            stats["discarded"] += stats["inserted"]
            stats["inserted"] = 0
            stats["last_reset_index"] = i
            table.clear()
            continue
        if ln != BUFFER_SIZE:
            stats["filtered"] += 1
            continue
        ident = int.from_bytes(bytes(int(b) for b in buf[ID_OFFSET:ID_OFFSET + 4]), "big")
        table.setdefault(key, OracleQuack(threshold)).insert(ident)
        stats["inserted"] += 1
    return table, stats
