"""The integer-issue roofline of the bench line (tools/issue_model.py): its
peak is the decomposition's VALU work (fixed per t, not the emitted
instruction count), so a slower kernel — e.g. one issuing 10 % more
instructions at the same clock — reports a lower fraction; and the committed
bench line's valu.frac recomputes from its own fields."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import issue_model  # noqa: E402


def test_anchor_t32_is_the_decomposition():
    a = issue_model.anchor(32, 32)
    assert a["shape"] == {"NB": 8, "NA": 4}
    assert a["ops_per_id"] == {"lazy_modmuls": 9, "macs": 24, "row0_adds": 8}
    want = (9 * issue_model.LAZY_MODMUL + 32 * issue_model.COST_HEAVY) / 64
    assert abs(a["cycles_per_id"] - want) < 1e-12


@pytest.mark.parametrize("t", [5, 8, 9, 16, 20, 28, 30, 32, 36, 40, 42, 48, 64, 72, 80])
def test_u32_shapes_cover_t(t):
    nb, na = issue_model.u32_shape(t)
    assert nb * na >= t and nb % 2 == 0


def test_u64_anchor_t80():
    a = issue_model.anchor(64, 80)
    assert a["shape"] == {"NBT": 8, "NA": 10}
    assert a["ops_per_id"] == {"p64_products": 15, "macs": 72, "row0_sums": 8, "shifts": 8}
    assert issue_model.anchor(64, 100) is None and issue_model.anchor(32, 300) is None


def test_more_instructions_lower_the_fraction():
    base = issue_model.roofline(32, 32, 10**9, 2.7, 2.1)
    slower = issue_model.roofline(32, 32, 10**9, 2.7 * 1.1, 2.1)   # +10 % issue at the same clock
    assert base["peak"] == slower["peak"]
    assert abs(slower["frac"] - base["frac"] / 1.1) < 1e-12


def test_committed_bench_line_recomputes():
    import issue_roofline
    for rel in ("profiles/r04/bench_n1.json",):
        r = issue_roofline.recompute_bench(os.path.join(ROOT, rel))
        assert r["agree"], r
        assert 0.3 < r["frac"] < 1.0
