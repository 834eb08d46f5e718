#!/usr/bin/env python3
"""Static kernel stats from a gfx950 assembly file (hipcc -S / --save-temps).

    python tools/kstat.py FILE.s [NAME_SUBSTRING ...]

For every kernel whose mangled name contains one of the substrings: VGPR,
SGPR and spill counts from the metadata, and the instruction mix of its first
loop (the block from the first 'Loop Header' label to the branch back to it):
VALU / SALU totals, multiplies, s_nop count.  Not part of the product.
"""
import collections
import re
import sys


def kernels(text):
    return re.findall(r"^\s+\.name:\s+(\S+)\n", text, re.M)


def meta(text, name):
    k = text.find(".name:           " + name)
    a = text.rfind("  - .", 0, k)          # this kernel's metadata entry
    b = text.find("\n  - .", k)
    m = text[a:b if b > 0 else len(text)]
    get = lambda key: int(re.search(key + r":\s+(\d+)", m).group(1))
    return {"vgpr": get(r"\.vgpr_count"), "sgpr": get(r"\.sgpr_count"), "vspill": get(r"\.vgpr_spill_count"),
            "lds": get(r"\.group_segment_fixed_size")}


def loop_mix(text, name):
    i = text.find(name + ":")
    j = text.find(".Lfunc_end", i)
    body = [l for l in text[i:j].split("\n")]
    hdrs = [k for k, l in enumerate(body) if "Loop Header" in l]
    if not hdrs:
        return None
    h = hdrs[0]
    lab = body[h].split(":")[0]
    end = next((k for k in range(h, len(body)) if ("s_cbranch" in body[k] or "s_branch" in body[k])
                and lab in body[k]), len(body) - 1)
    seg = [l.strip() for l in body[h:end + 1]
           if l.strip() and not l.strip().startswith((";", ".")) and not l.strip().endswith(":")]
    c = collections.Counter(l.split()[0] for l in seg)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    salu = sum(v for k, v in c.items() if k.startswith("s_") and k != "s_nop")
    mul = sum(v for k, v in c.items() if k.startswith(("v_mad_u64", "v_mul", "v_mad_u32", "v_lshl_add_u64")))
    return {"valu": valu, "mul": mul, "salu": salu, "nop": c["s_nop"], "insts": len(seg)}


def main():
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    for name in kernels(text):
        if subs and not any(s in name for s in subs):
            continue
        try:
            m = meta(text, name)
        except AttributeError:
            continue
        print(name, m, loop_mix(text, name))


if __name__ == "__main__":
    main()
