#!/usr/bin/env python3
"""Rust `extern "C"` block for every function the C ABI declares (include/tfhe_ntt_amd.h), as a tfhe-rs
maintainer's `-sys` module would hold it (INTEGRATION.md carries the output; tests/test_abi.py checks that it
covers the header).

  python tools/gen_rust_sys.py            -> the extern block on stdout
"""
import os
import re
import sys

HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include", "tfhe_ntt_amd.h")
SCALARS = {"size_t": "usize", "uint64_t": "u64", "uint32_t": "u32", "uint8_t": "u8", "int": "c_int",
           "unsigned": "c_uint", "double": "f64", "void": "c_void", "char": "c_char"}


def declarations(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(l for l in text.splitlines() if not l.strip().startswith("#") and 'extern "C"' not in l
                     and l.strip() != "}")
    text = re.sub(r"typedef[^;]*;", "", text, flags=re.S)
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(mi_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        yield m.group(1).strip(), m.group(2), [a.strip() for a in m.group(3).split(",") if a.strip()]


def rust_type(c):
    """C declarator type -> Rust: each `*` wraps the type built so far, `*const` when what it points to is const
    (a leading `const`, or a `const` right after the previous `*`)."""
    toks = re.findall(r"\*|\w+", c)
    cur_const, base, i = False, None, 0
    while i < len(toks) and toks[i] != "*":
        if toks[i] == "const":
            cur_const = True
        else:
            base = toks[i]
        i += 1
    name = base or "void"
    r = SCALARS.get(name, name)
    if i == len(toks):
        return "c_int" if name.startswith("mi_") and name.endswith(("format", "variant", "mode", "kind")) else r
    while i < len(toks):
        if toks[i] == "*":
            r = ("*const " if cur_const else "*mut ") + r
            cur_const = i + 1 < len(toks) and toks[i + 1] == "const"
            i += 2 if cur_const else 1
        else:
            i += 1
    return r


def arg(a, i):
    a = " ".join(a.split())
    if a == "void":
        return None
    m = re.match(r"(.*?)(\w+)$", a)
    ctype, name = m.group(1), m.group(2)
    if not ctype.strip():
        ctype, name = a, f"a{i}"
    return f"{name}: {rust_type(ctype)}"


def main(out=sys.stdout):
    text = open(HDR).read()
    lines = ['#[link(name = "tfhe_ntt_amd")]', 'extern "C" {']
    for ret, name, args in declarations(text):
        rargs = [x for x in (arg(a, i) for i, a in enumerate(args)) if x]
        r = rust_type(ret)
        lines.append(f"    pub fn {name}({', '.join(rargs)}){'' if r == 'c_void' else ' -> ' + r};")
    lines.append("}")
    print("\n".join(lines), file=out)


if __name__ == "__main__":
    main()
