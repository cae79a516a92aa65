"""INTEGRATION.md's Rust `-sys` bindings against the C headers (include/bftsim.h, bftsig.h, bftwire.h).

The bindings are not compiled here (no Rust toolchain), so this test does what rustc + the C
compiler would agree on:
  * every `#[repr(C)]` struct: field names in header order, each field's offset and the struct's size
    laid out with C rules from the Rust types, equal to gcc's offsetof / sizeof of the header struct;
  * every `extern "C"` fn: the header prototype's argument count, argument types (pointer constness,
    pointee type, integer width and sign) and return type;
  * every `pub const` equal to the header's #define;
  * every entry point the three headers declare is bound.
A field dropped or retyped in INTEGRATION.md (or the header) fails here.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ("bftsim.h", "bftsig.h", "bftwire.h")

# ------------------------------------------------------------------ Rust side
PRIM = {"u8": (1, 1), "i8": (1, 1), "u16": (2, 2), "i16": (2, 2), "u32": (4, 4), "i32": (4, 4),
        "u64": (8, 8), "i64": (8, 8), "usize": (8, 8), "isize": (8, 8), "f32": (4, 4), "f64": (8, 8),
        "c_int": (4, 4), "c_char": (1, 1)}
RUST_CANON = {"c_int": "i32", "c_char": "char", "c_void": "void", "i8": "char"}


def rust_blocks():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return "\n".join(re.findall(r"```rust\n(.*?)```", md, re.S))


def strip_rust_comments(s):
    return re.sub(r"//[^\n]*", "", s)


def rust_consts(src):
    return {m.group(1): m.group(3) for m in re.finditer(r"pub const (\w+)\s*:\s*(\w+)\s*=\s*([^;]+);", src)}


def rust_structs(src):
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{(.*?)\}", src, re.S):
        fields = []
        for fm in re.finditer(r"(pub\s+)?(\w+)\s*:\s*([^,]+?)\s*(,|$)", m.group(2).strip(), re.S):
            fields.append((fm.group(2), fm.group(3).strip()))
        out[m.group(1)] = fields
    return out


def parse_rust_type(t):
    """-> nested tuple: ('prim', name) | ('ptr', const, inner) | ('arr', inner, n) | ('struct', name)"""
    t = t.strip()
    if t.startswith("*const "):
        return ("ptr", True, parse_rust_type(t[7:]))
    if t.startswith("*mut "):
        return ("ptr", False, parse_rust_type(t[5:]))
    if t.startswith("["):
        inner, n = t[1:-1].rsplit(";", 1)
        return ("arr", parse_rust_type(inner), n.strip())
    if t in PRIM or t == "c_void":
        return ("prim", t)
    return ("struct", t)


def rust_layout(t, structs, consts, memo):
    """(size, align) of a parsed Rust type under #[repr(C)] rules"""
    k = t[0]
    if k == "prim":
        return PRIM[t[1]]
    if k == "ptr":
        return (8, 8)
    if k == "arr":
        n = t[2]
        n = int(consts[n].split(":")[-1].strip() if n in consts else n, 0)
        s, a = rust_layout(t[1], structs, consts, memo)
        return (s * n, a)
    name = t[1]
    if name not in memo:
        memo[name] = struct_layout(name, structs, consts, memo)
    size, align, _ = memo[name]
    return (size, align)


def struct_layout(name, structs, consts, memo):
    off, align, offs = 0, 1, {}
    for f, ty in structs[name]:
        s, a = rust_layout(parse_rust_type(ty), structs, consts, memo)
        off = (off + a - 1) // a * a
        offs[f] = off
        off += s
        align = max(align, a)
    return ((off + align - 1) // align * align, align, offs)


def canon_rust(t, consts=None):
    k = t[0]
    if k == "prim":
        return RUST_CANON.get(t[1], t[1])
    if k == "ptr":
        return f"ptr({'const' if t[1] else 'mut'},{canon_rust(t[2], consts)})"
    if k == "struct":
        return t[1]
    if k == "arr" and consts is not None:
        n = t[2]
        return f"arr({canon_rust(t[1], consts)},{int(consts[n].strip() if n in consts else n, 0)})"
    raise ValueError(t)


def rust_fns(src):
    src = "\n".join(re.findall(r'extern "C" \{(.*?)\n\}', strip_rust_comments(src), re.S))
    out = {}
    for m in re.finditer(r"pub fn (\w+)\s*\(([^)]*)\)\s*(->\s*([^;]+))?;", src, re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip()]
        types = [canon_rust(parse_rust_type(a.split(":", 1)[1])) for a in args]
        ret = canon_rust(parse_rust_type(m.group(4))) if m.group(4) else "void"
        out[m.group(1)] = (types, ret)
    return out


# ------------------------------------------------------------------ C side
C_CANON = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64", "int": "i32",
           "size_t": "usize", "float": "f32", "double": "f64", "char": "char", "void": "void",
           "bftsim_t": "bftsim", "bftsig_t": "bftsig", "bftwire_t": "bftwire"}


def header_text():
    txt = ""
    for h in HEADERS:
        s = open(os.path.join(ROOT, "include", h)).read()
        s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
        txt += s + "\n"
    return txt


def c_defines():
    out = {}
    for h in HEADERS:
        for m in re.finditer(r"#define (BFT\w+)\s+(-?\w+)", open(os.path.join(ROOT, "include", h)).read()):
            out[m.group(1)] = int(m.group(2).rstrip("uU"), 0)
    return out


def c_struct_decls(txt):
    """struct -> [(field, canonical type)] in declaration order"""
    defs = c_defines()
    out = {}
    for m in re.finditer(r"typedef struct (\w+)\s*\{(.*?)\}\s*(\w+)\s*;", txt, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = re.sub(r"\s+", " ", decl.strip())
            if not decl:
                continue
            base = re.match(r"(const )?(\w+)\s*(.*)", decl)
            for d in base.group(3).split(","):
                name = re.sub(r"[\*\s]|\[.*?\]", "", d)
                t = C_CANON.get(base.group(2), base.group(2))
                for i in range(d.count("*")):
                    t = f"ptr({'const' if (base.group(1) and i == 0) else 'mut'},{t})"
                for dim in reversed(re.findall(r"\[(\w+)\]", d)):
                    t = f"arr({t},{defs[dim] if dim in defs else int(dim, 0)})"
                fields.append((name, t))
        out[m.group(3)] = fields
    return out


def c_struct_fields(txt):
    return {k: [f for f, _ in v] for k, v in c_struct_decls(txt).items()}


def canon_c_param(p):
    """`const uint8_t *x` / `bftsim_t **out` / `uint8_t out[32]` / `uint32_t n` -> canonical string"""
    p = re.sub(r"\s+", " ", p.strip())
    arr = re.search(r"\[\w*\]\s*$", p)
    if arr:                                        # array parameter = pointer
        p = p[:arr.start()]
        m = re.match(r"(const )?(\w+) (\w+)$", p.strip())
        return f"ptr({'const' if m.group(1) else 'mut'},{C_CANON.get(m.group(2), m.group(2))})"
    m = re.match(r"(const )?(\w+)\s*(\**)\s*(\w+)?$", p)
    const, base, stars = bool(m.group(1)), C_CANON.get(m.group(2), m.group(2)), m.group(3)
    if not stars:
        return base
    t = base
    for i, _ in enumerate(stars):
        t = f"ptr({'const' if (const and i == 0) else 'mut'},{t})"
    return t


def c_fns(txt):
    txt = re.sub(r"#[^\n]*", "", txt)
    out = {}
    for m in re.finditer(r"([\w \*]+?)\b((?:bftsim|bftsig|bftwire)_\w+)\s*\(([^)]*)\)\s*;", txt):
        ret = canon_c_param(m.group(1).strip() + " r") if "*" in m.group(1) else \
            C_CANON.get(m.group(1).replace("const", "").strip(), m.group(1).strip())
        params = [] if m.group(3).strip() in ("", "void") else [canon_c_param(p) for p in m.group(3).split(",")]
        out[m.group(2)] = (params, ret)
    return out


def gcc_layout(struct_fields):
    lines = ["#include <stdio.h>", "#include <stddef.h>"] + [f'#include "{h}"' for h in HEADERS] + ["int main(void) {"]
    for st, fields in struct_fields.items():
        lines.append(f'printf("{st} sizeof %zu\\n", sizeof({st}));')
        for f in fields:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src])
        out = subprocess.check_output([exe]).decode().split("\n")
    return {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}


# ------------------------------------------------------------------ tests
@pytest.fixture(scope="module")
def sides():
    src = rust_blocks()
    txt = header_text()
    return dict(rs=rust_structs(strip_rust_comments(src)), consts=rust_consts(strip_rust_comments(src)),
                rf=rust_fns(src), cs=c_struct_fields(txt), cf=c_fns(txt))


def test_every_header_struct_is_bound_with_the_same_fields(sides):
    rs, cs = sides["rs"], sides["cs"]
    assert set(cs) == {"bftsim_config", "bftsim_result", "bftsim_stats", "bftsim_crypto_report", "bftwire_batch",
                       "bftwire_tx", "bftwire_block", "bftwire_preprepare"}
    for name, fields in cs.items():
        assert name in rs, f"{name} not bound in INTEGRATION.md"
        assert [f for f, _ in rs[name]] == fields, name


def test_struct_field_types_equal_header(sides):
    """pointee types and widths too (a *mut u32 for a uint64_t * has the same layout but corrupts memory)"""
    decls = c_struct_decls(header_text())
    for name, fields in decls.items():
        rtypes = [canon_rust(parse_rust_type(t), sides["consts"]) for _, t in sides["rs"][name]]
        assert rtypes == [t for _, t in fields], name


def test_struct_layouts_equal_gcc(sides):
    rs, consts = sides["rs"], sides["consts"]
    lay = gcc_layout(sides["cs"])
    memo = {}
    for name in sides["cs"]:
        size, _, offs = struct_layout(name, rs, consts, memo)
        assert size == lay[(name, "sizeof")], (name, size, lay[(name, "sizeof")])
        for f, off in offs.items():
            assert off == lay[(name, f)], (name, f, off, lay[(name, f)])


def test_every_entry_point_is_bound_with_the_header_prototype(sides):
    rf, cf = sides["rf"], sides["cf"]
    assert len(cf) >= 50
    missing = sorted(set(cf) - set(rf))
    assert not missing, f"not bound in INTEGRATION.md: {missing}"
    extra = sorted(set(rf) - set(cf))
    assert not extra, f"bound but not declared in include/: {extra}"
    for name, (cargs, cret) in cf.items():
        rargs, rret = rf[name]
        assert len(rargs) == len(cargs), (name, rargs, cargs)
        for i, (a, b) in enumerate(zip(rargs, cargs)):
            assert a == b, f"{name} argument {i}: rust {a} vs C {b}"
        assert rret == cret, f"{name} returns rust {rret} vs C {cret}"


def test_constants_equal_header_defines(sides):
    defs = c_defines()
    consts = sides["consts"]
    assert len(consts) >= 25
    for name, val in consts.items():
        assert name in defs, name
        assert int(val.strip().rstrip("uU"), 0) == defs[name], name


def test_checker_catches_a_dropped_field(sides):
    """the check itself: removing a config field or narrowing a pointee is detected"""
    rs = {k: list(v) for k, v in sides["rs"].items()}
    rs["bftsim_config"] = [f for f in rs["bftsim_config"] if f[0] != "backlog_mode"]
    lay = gcc_layout({"bftsim_config": sides["cs"]["bftsim_config"]})
    size, _, _ = struct_layout("bftsim_config", rs, sides["consts"], {})
    assert size != lay[("bftsim_config", "sizeof")] or [f for f, _ in rs["bftsim_config"]] != \
        sides["cs"]["bftsim_config"]
    assert canon_rust(parse_rust_type("*mut u32")) != canon_c_param("uint64_t *committed_height")
    assert ("committed_height", canon_rust(parse_rust_type("*mut u32"))) not in \
        c_struct_decls(header_text())["bftsim_result"]
