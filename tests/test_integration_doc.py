"""The reference-side binding documented in INTEGRATION.md must match the
C-ABI header byte for byte (CPU only, no GPU).

The Rust adapter a maintainer would add (`raytracer/src/gpu.rs`) passes
`&mut RtStats`, `*const RtShapeDesc` and `*const RtCameraDesc` straight to the
library, which fills `sizeof(rt_stats)` bytes of every stats struct it is
given (rt_api.cpp fill_stats). A stale `#[repr(C)]` mirror would therefore
overrun the caller's memory (What's missing 1). This test parses
the Rust structs and the `extern "C"` block out of INTEGRATION.md and the C
declarations out of include/rt_render.h, lays both out with ctypes (repr(C)
and C use the same rules), and requires equal field names, offsets and sizes,
equal function signatures, and every header entry point to be bound. It also
checks the sizes the library itself reports (rt_sizeof_*).
"""
import ctypes
import os
import re

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "rt_render.h")
DOC = os.path.join(REPO, "INTEGRATION.md")
LIB = os.path.join(PKG, "lib", "librtamd.so")

STRUCTS = {"RtShapeDesc": "rt_shape_desc", "RtLightDesc": "rt_light_desc", "RtCameraDesc": "rt_camera_desc",
           "RtStats": "rt_stats", "RtGroupDesc": "rt_group_desc"}
SIZES = {"rt_shape_desc": 680, "rt_light_desc": 48, "rt_camera_desc": 160, "rt_stats": 112, "rt_group_desc": 56}

RUST_SCALAR = {"i32": ctypes.c_int32, "u32": ctypes.c_uint32, "u64": ctypes.c_uint64, "f64": ctypes.c_double,
               "usize": ctypes.c_size_t, "u8": ctypes.c_uint8, "c_int": ctypes.c_int32}
C_SCALAR = {"int32_t": ctypes.c_int32, "uint32_t": ctypes.c_uint32, "uint64_t": ctypes.c_uint64,
            "double": ctypes.c_double, "size_t": ctypes.c_size_t, "uint8_t": ctypes.c_uint8, "int": ctypes.c_int32}


def _doc_rust():
    text = open(DOC).read()
    blocks = re.findall(r"```rust\n(.*?)```", text, flags=re.S)
    assert blocks, "INTEGRATION.md has no rust block"
    return "\n".join(blocks)


def rust_structs():
    src = re.sub(r"//[^\n]*", "", _doc_rust())
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\](?:\s*#\[[^\]]*\])*\s*pub struct (\w+)\s*\{(.*?)\}", src, flags=re.S):
        fields = []
        for fname, ftype in re.findall(r"pub (\w+)\s*:\s*([^,]+?)\s*(?:,|$)", body.strip(), flags=re.M):
            m = re.fullmatch(r"\[(\w+);\s*(\d+)\]", ftype.strip())
            ct = RUST_SCALAR[m.group(1)] * int(m.group(2)) if m else RUST_SCALAR[ftype.strip()]
            fields.append((fname, ct))
        out[name] = fields
    return out


def c_structs():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef struct \w+ \{(.*?)\}\s*(\w+);", src, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            ctype, rest = decl.split(None, 1)
            for item in rest.split(","):
                m = re.fullmatch(r"(\w+)(?:\[(\d+)\])?", item.strip())
                ct = C_SCALAR[ctype] * int(m.group(2)) if m.group(2) else C_SCALAR[ctype]
                fields.append((m.group(1), ct))
        out[name] = fields
    return out


def layout(fields):
    class S(ctypes.Structure):
        _fields_ = fields
    return ctypes.sizeof(S), [(n, getattr(S, n).offset, getattr(S, n).size) for n, _ in fields]


def test_doc_structs_match_header_layout():
    rs, cs = rust_structs(), c_structs()
    for rname, cname in STRUCTS.items():
        assert rname in rs, f"INTEGRATION.md lacks #[repr(C)] {rname}"
        assert cname in cs, f"header lacks {cname}"
        r_size, r_fields = layout(rs[rname])
        c_size, c_fields = layout(cs[cname])
        assert r_fields == c_fields, (rname, r_fields, c_fields)
        assert r_size == c_size == SIZES[cname], (rname, r_size, c_size)


def test_library_reports_the_same_sizes():
    lib = ctypes.CDLL(LIB)
    for fn, cname in (("rt_sizeof_shape_desc", "rt_shape_desc"), ("rt_sizeof_camera_desc", "rt_camera_desc"),
                      ("rt_sizeof_stats", "rt_stats")):
        f = getattr(lib, fn)
        f.restype = ctypes.c_size_t
        assert f() == SIZES[cname] == layout(c_structs()[cname])[0]
    assert lib.rt_abi_version() == 6


def _rust_kind(t):
    t = t.strip()
    if t.startswith("*"):
        return "ptr"
    return {"c_int": "i32", "i32": "i32", "u32": "u32", "u64": "u64", "usize": "usize", "f64": "f64", "u8": "u8"}[t]


def _c_kind(decl, named=True):
    """Kind of a C parameter declaration ("const double m[16]", "uint32_t hsize")
    or, with named=False, of a bare return type ("int", "const char*")."""
    decl = decl.strip()
    if decl == "void":
        return None
    if "*" in decl or "[" in decl:
        return "ptr"
    words = [w for w in decl.split() if w != "const"]
    if named:
        words = words[:-1]
    return {"int": "i32", "int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "size_t": "usize",
            "double": "f64", "uint8_t": "u8"}[words[0]]


def rust_fns():
    src = re.sub(r"//[^\n]*", "", _doc_rust())
    ext = re.search(r'extern "C" \{(.*?)\n\}', src, flags=re.S).group(1)
    out = {}
    for name, args, ret in re.findall(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", ext, flags=re.S):
        kinds = [_rust_kind(a.split(":", 1)[1]) for a in args.split(",") if a.strip()]
        out[name] = (kinds, _rust_kind(ret) if ret else None)
    return out


def c_fns():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"([\w\s\*]+?)\s*\b(rt_\w+)\s*\(([^)]*)\)\s*;", src):
        ret = ret.split("\n")[-1].strip()
        kinds = [] if args.strip() == "void" else [_c_kind(a) for a in args.split(",")]
        out[name] = (kinds, _c_kind(ret, named=False))
    return out


def test_doc_extern_block_binds_every_entry_point_with_its_signature():
    from test_abi import declared_functions
    rf, cf = rust_fns(), c_fns()
    assert sorted(cf) == declared_functions()  # the signature parser saw every declaration
    missing = sorted(set(cf) - set(rf))
    assert not missing, f"INTEGRATION.md's extern block lacks {missing}"
    for name, sig in rf.items():
        assert name in cf, f"INTEGRATION.md binds {name}, which the header does not declare"
        assert sig == cf[name], (name, sig, cf[name])


def test_a_stale_doc_fails():
    """The parser is not vacuous: the round-2 80-byte RtStats is caught."""
    stale = [f for f in rust_structs()["RtStats"] if f[0] not in
             ("rays_shadow_traced", "sphere_tests_executed", "box_tests_executed", "exhaustive", "_pad")]
    assert layout(stale)[0] == 80 != layout(c_structs()["rt_stats"])[0]
