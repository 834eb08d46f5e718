"""Caller-side decode loop with the reset protocol.

Mirrors the end host of media_integration/media/src/bin/media_client.rs:205-325
(`listen_for_quacks_power_sum`) as a transport-free state machine: the
application reports what it sends (``on_send``) and every quACK it receives
(``on_quack``); the receiver answers with the sequence numbers to retransmit
and whether to ask the proxy for a reset.

The arithmetic is the engine's: the log prefix is inserted with the batch
encode (GPU) when it is long and with the per-packet host insert otherwise,
and the candidate scan (``arithmetic::eval(&coeffs, id).value() == 0`` over
the log, breaking at ``diff.last_value()``, media_client.rs:306-313) runs as
the GPU root test with the stop value when the log is long.  Both paths are
bit-identical; neither is a fallback for the other.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .quack import PowerSumQuackU32

BATCH_MIN = 4096  # log entries from which the batch (GPU) paths are used


@dataclass
class QuackAction:
    retransmit: list = field(default_factory=list)   # seqnos, in log order
    send_reset: bool = False                          # UDP [0] to the proxy (media_client.rs:272)
    reset_reason: tuple = ()                          # (reordered?, retx?, exceeds threshold?)
    decoded: int = 0                                  # missing ids found


class QuackReceiver:
    """listen_for_quacks_power_sum's state: my_quack, the sent log
    seqno_ids, and the reset debounce (media_client.rs:216-221)."""

    def __init__(self, threshold: int, reset_debounce_s: float = 0.1, batch_min: int = BATCH_MIN):
        self.threshold = int(threshold)
        self.my_quack = PowerSumQuackU32(self.threshold)
        self.seqno_ids: list = []          # [(seqno, id)], in send order (PacketSender.seqno_ids)
        self.last_quack_reset = None
        self.reset_debounce_s = reset_debounce_s
        self.batch_min = batch_min

    def on_send(self, seqno: int, ident: int) -> None:
        self.seqno_ids.append((int(seqno), int(ident) & 0xFFFFFFFF))

    def _insert_prefix(self, upto: int) -> None:
        ids = np.fromiter((i for _, i in self.seqno_ids[: upto + 1]), dtype=np.uint32, count=upto + 1)
        if len(ids) >= self.batch_min:
            self.my_quack.insert_batch(ids)
        else:
            for v in ids.tolist():
                self.my_quack.insert(v)

    def _missing(self, diff: PowerSumQuackU32) -> list:
        coeffs = diff.to_coeffs()
        stop = diff.last_value()
        if len(self.seqno_ids) >= self.batch_min:
            log = np.fromiter((i for _, i in self.seqno_ids), dtype=np.uint32, count=len(self.seqno_ids))
            pos = diff.root_test(coeffs, log, stop_value=stop)
            return [self.seqno_ids[p] for p in pos]
        # short log: the same loop (stop at last_value, eval == 0) on the CPU
        # in one native call (qk_u32_decode_host)
        log = np.fromiter((i for _, i in self.seqno_ids), dtype=np.uint32, count=len(self.seqno_ids))
        return [self.seqno_ids[p] for p in diff.decode_host(log, stop_at_last=True)]

    def on_quack(self, quack: PowerSumQuackU32, now: float) -> QuackAction:
        act = QuackAction()
        if quack.last_value() == self.my_quack.last_value():                       # :233-235
            return act
        last_index = None                                                           # :240-246
        lv = quack.last_value()
        for i, (_, ident) in enumerate(self.seqno_ids):
            if ident == lv:
                last_index = i
                break
        if last_index is not None:                                                  # :247-252
            self._insert_prefix(last_index)
        reset0 = last_index is None                                                 # :257-261
        reset1 = self.my_quack.count() < quack.count()
        # `quack.count() + threshold as u32` is u32 arithmetic (wraps in a release build)
        reset2 = self.my_quack.count() > (quack.count() + self.threshold) & 0xFFFFFFFF
        if reset0 or reset1 or reset2:
            should = self.last_quack_reset is None or now > self.last_quack_reset + self.reset_debounce_s
            act.reset_reason = (reset0, reset1, reset2)
            if should:                                                              # :267-276
                act.send_reset = True
                self.my_quack = PowerSumQuackU32(self.threshold)
                self.seqno_ids = []
                self.last_quack_reset = now
            return act
        if self.last_quack_reset is not None:                                       # :280-283
            self.last_quack_reset = None
        diff = self.my_quack.clone()                                                # :295-300
        diff.sub_assign(quack)
        if diff.count() == 0:
            del self.seqno_ids[: last_index + 1]
            return act
        missing = self._missing(diff)                                               # :304-313
        del self.seqno_ids[: last_index + 1]                                        # :316
        for seqno, ident in missing:                                                # :318-322
            self.my_quack.remove(ident)
            act.retransmit.append(seqno)
        act.decoded = len(missing)
        return act
