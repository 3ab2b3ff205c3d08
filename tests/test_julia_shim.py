"""The Julia drop-in (julia/FlashSDF.jl) against the C-ABI it binds: every
`ccall` names a function include/flashsdf.h declares (and the library exports),
with the same arity and argument kinds, and the shim's immutable structs mirror
the header's C structs field for field. Julia is absent from the image (SURVEY.md
§8c), so the shim is checked statically; its arithmetic mirrors the tested
Python host (flash/gradientdescent.py, flash/rbf.py)."""
import os
import re

import pytest

from conftest import ROOT

SHIM = os.path.join(ROOT, "julia", "FlashSDF.jl")
HEADER = os.path.join(ROOT, "include", "flashsdf.h")


def _balanced(text, i):
    """text[i] == '(' -> index just past the matching ')'."""
    depth = 0
    for j in range(i, len(text)):
        if text[j] == "(":
            depth += 1
        elif text[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def _split_top(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({":
            depth += 1
        elif ch in ")}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def shim_ccalls():
    text = open(SHIM).read()
    calls = []
    for m in re.finditer(r"ccall\(\(:(fsdf_\w+),\s*lib\),", text):
        rest = text[m.end():]
        ret, _, after = rest.partition(",")
        k = after.index("(")
        end = _balanced(after, k)
        args = _split_top(after[k + 1:end - 1])
        calls.append((m.group(1), ret.strip(), args))
    return calls


def header_protos():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"^(int|const char\*)\s+(fsdf_\w+)\s*\(([^)]*)\)\s*;", text, re.M):
        args = [a.strip() for a in m.group(3).replace("\n", " ").split(",") if a.strip()]
        types = [re.sub(r"\s*\w+$", "", a).replace(" *", "*").strip() for a in args]
        protos[m.group(2)] = (m.group(1), types)
    return protos


def header_structs():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct (fsdf_\w+) \{(.*?)\}", text, re.S):
        fields = []
        for ln in m.group(2).split(";"):
            ln = ln.strip()
            if ln:
                fields.append(ln.rsplit(None, 1))
        out[m.group(1)] = [(t.replace(" *", "*").strip(), n.lstrip("*")) for t, n in fields]
    return out


# C type (as declared) -> the Julia ccall types that pass it correctly
C_TO_JULIA = {
    "fsdf_ctx*": {"Ptr{Void}"}, "const fsdf_ctx*": {"Ptr{Void}"}, "void*": {"Ptr{Void}"},
    "fsdf_ctx**": {"Ref{Ptr{Void}}"},
    "const fsdf_opts*": {"Ref{Opts}"}, "const fsdf_surface*": {"Ptr{Surface}"}, "const fsdf_hull*": {"Ptr{Hull}"},
    "int32_t": {"Int32"}, "int64_t": {"Int64"},
    "const double*": {"Ptr{Float64}"}, "double*": {"Ptr{Float64}", "Ref{Float64}"},
    "int32_t*": {"Ptr{Int32}", "Ref{Int32}"}, "const int32_t*": {"Ptr{Int32}"},
    "int64_t*": {"Ptr{Int64}", "Ref{Int64}"}, "uint64_t*": {"Ptr{UInt64}"},
}
RET = {"int": "Cint", "const char*": "Cstring"}
FIELD = {"int32_t": "Int32", "const double*": "Ptr{Float64}", "const int32_t*": "Ptr{Int32}", "fsdf_hull": "Hull"}
STRUCTS = {"fsdf_opts": "Opts", "fsdf_hull": "Hull", "fsdf_surface": "Surface"}


def test_shim_ccalls_match_header():
    protos = header_protos()
    calls = shim_ccalls()
    names = {c[0] for c in calls}
    # the drop-in path: context, model, cloud, RBF rows, pass, skin, hull builder
    for need in ("fsdf_create", "fsdf_destroy", "fsdf_last_error", "fsdf_set_surfaces", "fsdf_accum_len",
                 "fsdf_set_points", "fsdf_set_rbf_params", "fsdf_eval", "fsdf_skin", "fsdf_convex_hull"):
        assert need in names, need
    for name, ret, args in calls:
        assert name in protos, name
        cret, ctypes_ = protos[name]
        assert ret == RET[cret], (name, ret, cret)
        assert len(args) == len(ctypes_), (name, args, ctypes_)
        for a, c in zip(args, ctypes_):
            assert a in C_TO_JULIA[c], (name, a, c)


def test_shim_structs_match_header():
    text = open(SHIM).read()
    hs = header_structs()
    for cname, jname in STRUCTS.items():
        m = re.search(r"immutable %s\b.*?\n(.*?)\nend" % jname, text, re.S)
        assert m, jname
        jfields = [ln.split("#")[0].strip() for ln in m.group(1).splitlines() if "::" in ln]
        jfields = [tuple(f.split("::")) for f in jfields]
        cf = hs[cname]
        assert len(jfields) == len(cf), (jname, jfields, cf)
        for (jn, jt), (ct, cn) in zip(jfields, cf):
            assert jt == FIELD[ct], (jname, jn, jt, ct)


def test_shim_symbols_exported():
    from flash import _lib
    lib = _lib.load()
    for name, _, _ in shim_ccalls():
        assert hasattr(lib, name), name


def test_shim_accumulator_layout_matches_host():
    """The shim sizes the accumulator with fsdf_accum_len and walks the same
    layout as flash/gradientdescent.py: 1 + 6 per surface, then per RBF skin
    λ (n+4) and E (3n)."""
    text = open(SHIM).read()
    assert "fsdf_accum_len" in text and "zeros(f.ctx.accum_len)" in text
    assert "off = 2 + 6S" in text and "off += 4n + 4" in text
    assert "normalize!(state.mechanism_state)" in text  # src/gradientdescent.jl:30
    assert "f.weight * sum(deformation .^ 2)" in text     # src/gradientdescent.jl:33-37
