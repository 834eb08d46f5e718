"""The Rust drop-in crate (rust/quack) against the C header, checked without
a Rust toolchain (none in this image): every prototype of include/quack_hip.h
is declared in rust/quack/src/ffi.rs with the same parameter count and the
mechanically mapped types, every #[repr(C)] struct has the header's fields in
order, and the crate exposes the names the reference callers use (SURVEY.md
Appendix B) with no elided bodies."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(ROOT, "rust", "quack")

BASE = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
        "int": "c_int", "size_t": "usize", "double": "f64", "char": "c_char", "void": "c_void"}


def strip_c_comments(src):
    return re.sub(r"/\*.*?\*/", " ", src, flags=re.S)


def c_type_to_rust(decl, is_return=False):
    """'const uint32_t *const *d_ids' -> '*const *const u32' (name dropped)."""
    decl = decl.strip()
    arr = False
    m = re.search(r"\[[^\]]*\]\s*$", decl)
    if m:
        arr = True
        decl = decl[:m.start()]
    toks = re.findall(r"[A-Za-z_]\w*|\*", decl)
    if not is_return:
        assert toks[-1] != "*", ("unnamed parameter", decl)
        toks = toks[:-1]                                  # the parameter name
    base_const = False
    i = 0
    while toks[i] == "const":
        base_const, i = True, i + 1
    base = toks[i]
    cur = BASE.get(base, base)
    i += 1
    if i < len(toks) and toks[i] == "const":
        base_const, i = True, i + 1
    cur_const = base_const
    while i < len(toks):
        assert toks[i] == "*", (decl, toks)
        cur = ("*const " if cur_const else "*mut ") + cur
        i += 1
        cur_const = False
        if i < len(toks) and toks[i] == "const":
            cur_const, i = True, i + 1
    if arr:
        cur = ("*const " if cur_const else "*mut ") + cur
    return cur


def header_prototypes():
    src = strip_c_comments(open(os.path.join(ROOT, "include", "quack_hip.h")).read())
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(qk_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ret = " ".join(ret.split()).replace("extern \"C\"", "").strip()
        args = [] if params.strip() in ("", "void") else [c_type_to_rust(p) for p in params.split(",")]
        r = None if ret == "void" else c_type_to_rust(ret, is_return=True)
        out[name] = (args, r)
    return out


def rust_externs():
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (qk_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        name, params, ret = m.group(1), m.group(2), m.group(3)
        args = []
        for p in params.split(","):
            p = " ".join(p.split())
            if p:
                args.append(p.split(":", 1)[1].strip())
        out[name] = (args, " ".join(ret.split()) if ret else None)
    return out


def test_type_mapping_rules():
    assert c_type_to_rust("const uint32_t *const *d_ids") == "*const *const u32"
    assert c_type_to_rust("void *const *streams") == "*const *mut c_void"
    assert c_type_to_rust("const uint8_t my_ipv4[4]") == "*const u8"
    assert c_type_to_rust("uint8_t id[QK_COMM_ID_BYTES]") == "*mut u8"
    assert c_type_to_rust("qk_ctx **out") == "*mut *mut qk_ctx"
    assert c_type_to_rust("const qk_comm *comm") == "*const qk_comm"
    assert c_type_to_rust("size_t n") == "usize"
    assert c_type_to_rust("const char *", is_return=True) == "*const c_char"


def test_every_header_prototype_is_bound_with_matching_types():
    hdr, rs = header_prototypes(), rust_externs()
    assert len(hdr) > 70
    assert set(hdr) == set(rs), (sorted(set(hdr) - set(rs)), sorted(set(rs) - set(hdr)))
    for name, (args, ret) in hdr.items():
        rargs, rret = rs[name]
        assert rargs == args, (name, args, rargs)
        assert rret == ret, (name, ret, rret)


def header_struct_fields(name):
    src = strip_c_comments(open(os.path.join(ROOT, "include", "quack_hip.h")).read())
    body = re.search(r"typedef struct %s \{(.*?)\}" % name, src, flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            fp = re.search(r"\(\s*\*\s*(\w+)\s*\)", decl)          # function-pointer field
            fields.append(fp.group(1) if fp else re.findall(r"(\w+)\s*(?:\[[^\]]*\])?$", decl)[0])
    return fields


def rust_struct_fields(name):
    src = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    body = re.search(r"pub struct %s \{(.*?)\}" % name, src, flags=re.S).group(1)
    return re.findall(r"pub (\w+):", body)


def test_repr_c_structs_match_header():
    for s in ("qk_u32", "qk_u64", "qk_pkt_meta", "qk_pkt_stats", "qk_flow_key", "qk_comm_host_ops"):
        assert rust_struct_fields(s) == header_struct_fields(s), s


def test_constants_match_header():
    hdr = open(os.path.join(ROOT, "include", "quack_hip.h")).read()
    rs = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    for name in ("QK_MAX_THRESHOLD", "QK_ID_OFFSET", "QK_BUFFER_SIZE", "QK_COMM_ID_BYTES"):
        h = int(re.search(r"#define %s (\d+)u?" % name, hdr).group(1))
        r = int(re.search(r"pub const %s: \w+ = ([\d_]+);" % name, rs).group(1).replace("_", ""))
        assert h == r, name
    for name, val in re.findall(r"(QK_E_\w+) = (-\d+)", hdr):
        assert re.search(r"pub const %s: c_int = %s;" % (name, val), rs), name
    assert "4_294_967_291" in rs and "18_446_744_073_709_551_557" in rs


def test_crate_surface_and_no_elided_bodies():
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    ar = open(os.path.join(CRATE, "src", "arithmetic.rs")).read()
    sm = open(os.path.join(CRATE, "src", "strawmen.rs")).read()
    for needle in ("pub trait PowerSumQuack", "fn new(threshold: usize) -> Self", "fn count(&self) -> u32",
                   "fn last_value(&self) -> Option<Self::Element>", "fn insert(&mut self", "fn remove(&mut self",
                   "fn sub_assign(&mut self, rhs: Self)", "fn to_coeffs(&self)", "fn decode_with_log",
                   "power_sum_quack!(PowerSumQuackU32", "power_sum_quack!(PowerSumQuackU64",
                   "impl Serialize for $name", "impl<'de> Deserialize<'de> for $name",
                   "pub use strawmen::{StrawmanAQuack, StrawmanBQuack}"):
        assert needle in lib, needle
    assert "pub trait ModularArithmetic" in ar and "pub fn eval<T: Field>" in ar
    assert "pub struct StrawmanAQuack" in sm and "pub window: VecDeque<u32>" in sm and "pub window_size: usize" in sm
    for src in (lib, ar, sm):
        assert "todo!" not in src and "unimplemented!" not in src and "/* " not in src
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'name = "quack"' in toml and "strawmen = []" in toml
