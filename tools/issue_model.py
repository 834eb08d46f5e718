"""Algorithmic anchor of the integer-issue roofline (bench.py `roofline.valu`).

The HBM roofline of the encode is far away (0.18 of 8 TB/s): the kernels are
bound by integer instruction issue.  This module prices the *decomposition*
the kernel computes — not the instructions the compiler happened to emit — so
that a kernel issuing more instructions than the decomposition needs reports a
lower fraction:

  u32, baby-step / giant-step shape (NB, NA) of the product's table for t
  (encode.hip enc32):
    (NB - 1) + (NA - 2) lazy modmuls per id     3 v_mad_u64_u32 + 1 v_sub
                                                + half a v_min3 (the wrap check)
    (NA - 1) * NB multiply-accumulates          1 v_mad_u64_u32 each
    NB row-0 adds                               1 v_mad_u64_u32 each
  u64, baby-step / giant-step with NBT babies and NA giant rows (encode.hip
  enc64, bsgs64.h):
    (NBT - 1) + (NA - 2) p64 products per id    7 v_mad_u64_u32 + 3 carry selects
    (NA - 1) * NBT MACs                          4 v_mad_u64_u32 each
    NBT row-0 sums                              2 v_mad_u64_u32 each
    NBT B * 2^32 shifts                         2 v_mad_u64_u32 + 1 carry select

Each instruction at its measured issue cost (profiles/r01/ubench_issue.json,
8 waves/SIMD, SIMD cycles per wave64 instruction): a two-source VALU op
17.97 / 8, a three-source or SGPR-writing one (v_mad_u64_u32, v_min3,
v_cndmask) 33.52 / 8.  The scalar carry counts (s_bcnt1 + s_add per MAC)
co-issue on the scalar unit and are not priced; loads, address arithmetic,
loop control and the reduction epilogue are overhead, not decomposition.
One wave instruction serves 64 ids, so cycles per id = the sum / 64.

  peak      anchor SIMD-cycles per id (this module)
  achieved  the launch's SIMD-cycles per id: clock x kernel time x 1024 SIMDs
            / ids, with the shader clock read in the same run (qk_clock_probe
            beside the running kernel)
  frac      peak / achieved
"""
from __future__ import annotations

COST_SIMPLE = 17.97 / 8       # v_add_u32 / v_sub_u32 / v_mov (profiles/r01/ubench_issue.json "vadd8")
COST_HEAVY = 33.52 / 8        # v_mad_u64_u32, v_min3, v_cndmask ("vmad8", "min3 x8", "cndmask x8")
SIMDS = 1024

LAZY_MODMUL = 3 * COST_HEAVY + COST_SIMPLE + 0.5 * COST_HEAVY
P64_PRODUCT = 7 * COST_HEAVY + 3 * COST_HEAVY
MAD = COST_HEAVY


def u32_shape(t: int):
    """(NB, NA) of the u32 baby-step/giant-step kernel the product runs at t
    (encode.hip enc32, round-3 table); None off the single-pass BSGS range."""
    table = [(5, 8, 4, 2), (9, 12, 4, 3), (13, 16, 4, 4), (17, 20, 4, 5), (21, 24, 4, 6), (25, 28, 4, 7),
             (29, 30, 6, 5), (31, 32, 8, 4), (33, 36, 6, 6), (37, 40, 8, 5), (41, 42, 6, 7), (43, 48, 8, 6),
             (49, 56, 8, 7), (57, 64, 8, 8), (65, 72, 8, 9), (73, 80, 8, 10)]
    for lo, hi, nb, na in table:
        if lo <= t <= hi:
            return nb, na
    return None


def u64_shape(t: int):
    """(NBT, NA) of the u64 kernel at t (encode.hip enc64): four babies at
    t = 14..20, 25..28, 33..36, else eight; None off 14..80."""
    if not 14 <= t <= 80:
        return None
    q4 = (t + 3) // 4
    if t <= 36 and q4 in (4, 5, 7, 9):
        return 4, q4
    return 8, (t + 7) // 8


def anchor(bits: int, t: int):
    """Decomposition of the kernel at (bits, t) and its SIMD-cycles per id, or
    None where the product runs another kernel (power chains, passes)."""
    if bits == 32:
        s = u32_shape(t)
        if s is None:
            return None
        nb, na = s
        ops = {"lazy_modmuls": nb - 1 + na - 2, "macs": (na - 1) * nb, "row0_adds": nb}
        cyc = ops["lazy_modmuls"] * LAZY_MODMUL + (ops["macs"] + ops["row0_adds"]) * MAD
        shape = {"NB": nb, "NA": na}
    else:
        s = u64_shape(t)
        if s is None:
            return None
        nbt, na = s
        ops = {"p64_products": nbt - 1 + na - 2, "macs": (na - 1) * nbt, "row0_sums": nbt, "shifts": nbt}
        cyc = (ops["p64_products"] * P64_PRODUCT + ops["macs"] * 4 * MAD + ops["row0_sums"] * 2 * MAD
               + ops["shifts"] * 3 * COST_HEAVY)
        shape = {"NBT": nbt, "NA": na}
    return {"shape": shape, "ops_per_id": ops, "cycles_per_id": cyc / 64.0,
            "costs": {"simple": COST_SIMPLE, "heavy": COST_HEAVY, "lazy_modmul": LAZY_MODMUL,
                      "p64_product": P64_PRODUCT}}


def roofline(bits: int, t: int, n_ids: int, kernel_ms: float, clock_ghz: float):
    """The integer-issue roofline object of a launch of n_ids at kernel_ms."""
    a = anchor(bits, t)
    if a is None or not clock_ghz or not kernel_ms:
        return None
    achieved = clock_ghz * 1e9 * kernel_ms * 1e-3 * SIMDS / n_ids
    return {"bound": "valu-issue", "unit": "SIMD-cycles/id", "peak": a["cycles_per_id"], "achieved": achieved,
            "frac": a["cycles_per_id"] / achieved, "clock_ghz": clock_ghz, "anchor": a,
            "method": "tools/issue_model.py: the decomposition's VALU work at the measured per-class issue costs "
                      "(fixed per t, independent of the emitted instruction count) against this run's kernel "
                      "time at this run's shader clock"}
