"""The reference-side Rust binding (bindings/rust/src/sys.rs) against the C
ABI it binds (include/massrt.h). There is no Rust toolchain in this image, so
the binding is parsed, not compiled:

  * every struct the header declares has a #[repr(C)] Rust twin with the same
    fields in the same order, and the repr(C) layout computed from the Rust
    field types equals gcc's sizeof/offsetof of the C struct;
  * every function the header declares is in the `extern "C"` block with the
    same parameter count and types (C type -> Rust type mapping below) and
    return type; the binding declares nothing the header does not.
"""
import re
import shutil
import subprocess

import pytest

from conftest import REPO

SYS_RS = REPO / "bindings" / "rust" / "src" / "sys.rs"
HEADER = REPO / "include" / "massrt.h"
SCALARS = {"f32": (4, 4), "u32": (4, 4), "i32": (4, 4), "u64": (8, 8), "i64": (8, 8), "f64": (8, 8), "u8": (1, 1)}
C2R = {"int": "i32", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64", "float": "f32", "double": "f64",
       "uint8_t": "u8", "char": "c_char", "void": "c_void"}


def rust_structs():
    text = SYS_RS.read_text()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive[^\]]*\]\s*)?pub struct (\w+)\s*\{(.*?)\n\}", text, re.S):
        fields = re.findall(r"pub\s+(\w+)\s*:\s*([^,\n]+),", m.group(2))
        out[m.group(1)] = [(n, t.strip()) for n, t in fields]
    return out


def header_structs():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct\s*\{(.*?)\}\s*(mrt_\w+)\s*;", text, re.S):
        names = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            first, *rest = [d.strip() for d in decl.split(",")]  # "float min[3], max[3]": two fields
            names.append(re.search(r"(\w+)\s*(?:\[\d+\])?$", first).group(1))
            names += [re.match(r"\**\s*(\w+)", r).group(1) for r in rest]
        out[m.group(2)] = names
    return out


def layout(structs, name, memo):
    if name in memo:
        return memo[name]
    off, align, offsets = 0, 1, {}
    for fname, ftype in structs[name]:
        size, al = type_size(structs, ftype, memo)
        off = (off + al - 1) // al * al
        offsets[fname] = off
        off += size
        align = max(align, al)
    size = (off + align - 1) // align * align
    memo[name] = (size, align, offsets)
    return memo[name]


def type_size(structs, t, memo):
    t = t.strip()
    if t.startswith("*"):
        return 8, 8
    m = re.fullmatch(r"\[(.+);\s*(\d+)\]", t)
    if m:
        s, a = type_size(structs, m.group(1), memo)
        return s * int(m.group(2)), a
    if t in SCALARS:
        return SCALARS[t]
    s, a, _ = layout(structs, t, memo)
    return s, a


def test_struct_layouts_match_header(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    rs, hs = rust_structs(), header_structs()
    assert set(hs) <= set(rs), f"structs missing in sys.rs: {sorted(set(hs) - set(rs))}"
    for cname, cfields in hs.items():
        assert [f for f, _ in rs[cname]] == cfields, cname
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for cname, cfields in hs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in cfields:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    (tmp_path / "l.c").write_text("\n".join(lines))
    subprocess.run(["gcc", "-o", str(tmp_path / "l"), str(tmp_path / "l.c")], check=True)
    out = subprocess.run([str(tmp_path / "l")], check=True, capture_output=True, text=True).stdout
    memo = {}
    checked = 0
    for line in out.splitlines():
        key, val = line.rsplit(" ", 1)
        if key.endswith(" size"):
            assert layout(rs, key[:-5], memo)[0] == int(val), key
        else:
            cname, f = key.split(".")
            assert layout(rs, cname, memo)[2][f] == int(val), key
        checked += 1
    assert checked > 100


def c_to_rust(ctype: str) -> str:
    """C parameter/return type -> the Rust FFI spelling ("const mrt_ctx*" -> "*const mrt_ctx")."""
    words = ctype.replace("*", " * ").split()
    stars = words.count("*")
    const = stars > 0 and "const" in words[: words.index("*")]
    r = C2R.get(next(w for w in words if w not in ("const", "*")), None)
    r = r or next(w for w in words if w not in ("const", "*"))
    for k in range(stars):  # innermost pointer first
        r = ("*const " if (k == 0 and const) else "*mut ") + r
    return r


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    text = re.sub(r"#define[^\n]*\n", "", text)
    out = {}
    for m in re.finditer(r"([A-Za-z_0-9\* ]+?)\b(mrt_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        ret = c_to_rust(" ".join(m.group(1).split()))
        params = []
        for p in " ".join(m.group(3).split()).split(","):
            p = p.strip()
            if p in ("void", ""):
                continue
            typ = re.sub(r"\b\w+$", "", p).strip()  # drop the parameter name
            params.append(c_to_rust(typ))
        out[m.group(2)] = (ret, params)
    return out


def rust_functions():
    text = SYS_RS.read_text()
    block = text[text.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, re.S):
        params = [re.sub(r"^\w+\s*:\s*", "", p.strip()) for p in " ".join(m.group(2).split()).split(",") if p.strip()]
        ret = (m.group(3) or "").strip()
        out[m.group(1)] = (ret, [" ".join(p.split()) for p in params])
    return out


def test_functions_match_header():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 50
    assert sorted(h) == sorted(r), (sorted(set(h) - set(r)), sorted(set(r) - set(h)))
    for name, (ret, params) in h.items():
        rret, rparams = r[name]
        ret = "" if ret == "c_void" else ret
        assert rret == ret, (name, rret, ret)
        assert rparams == params, (name, rparams, params)


def test_abi_version_matches():
    m = re.search(r"#define MRT_ABI_VERSION (\d+)", HEADER.read_text())
    r = re.search(r"pub const MRT_ABI_VERSION: i32 = (\d+);", SYS_RS.read_text())
    assert m and r and m.group(1) == r.group(1)
