"""The Rust binding of the drop-in (src/hrt_ffi.rs, added by integration/epq_raytracer.patch, which
replaces the Vulkano dispatch of /root/reference/src/raytrace_pipeline.rs:51-266 and
src/diffuse.rs:35-136) and the excerpts INTEGRATION.md quotes, against include/hip_raytrace.h, on the CPU.

There is no Rust toolchain in this image, so the binding is never compiled here.  This test is what
keeps it from drifting from the ABI (the published `hrt_stats` was 56 B while the ABI-4
header's is 64 B, so `hrt_get_stats` would have written 8 B past a Rust caller's struct):

* every `#[repr(C)]` struct of the ```rust blocks has the header struct's fields in the same order, with
  the same types, and the `repr(C)` layout computed from them (size, alignment, every offset) equals what
  gcc lays out for the header (a compiled C probe);
* every `extern "C"` fn exists in the header with the same arity, parameter and return types (widths,
  signedness, pointer depth, pointee type and the outer pointer's constness);
* every `pub const` equals the header's enum / #define value;
* every non-debug function of the header is declared by the binding (an ABI bump that adds an entry point
  and misses the document fails here).
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hip_raytrace.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")
PATCH = os.path.join(ROOT, "integration", "epq_raytracer.patch")

# Rust scalar -> (canonical C type, size, align) on x86-64 / the reference's targets
RUST_SCALARS = {
    "u8": ("uint8_t", 1, 1), "i8": ("int8_t", 1, 1), "u16": ("uint16_t", 2, 2), "i16": ("int16_t", 2, 2),
    "u32": ("uint32_t", 4, 4), "i32": ("int32_t", 4, 4), "u64": ("uint64_t", 8, 8), "i64": ("int64_t", 8, 8),
    "f32": ("float", 4, 4), "f64": ("double", 8, 8), "usize": ("size_t", 8, 8), "isize": ("ptrdiff_t", 8, 8),
    "c_char": ("char", 1, 1), "c_void": ("void", 0, 1), "c_int": ("int32_t", 4, 4), "c_uint": ("uint32_t", 4, 4),
}
# the vulkano shader! records the binding passes verbatim (raytrace_shader::*) and the C records they are
# (src/hrt_ffi.rs defines them itself, in `mod records`, under the GLSL names)
RECORD_NAMES = {"RayTracingMaterial": "hrt_material", "Ray": "hrt_ray", "Sphere": "hrt_sphere",
                "Triangle": "hrt_triangle", "Mesh": "hrt_mesh", "PushConstants": "hrt_push_constants"}
RUST_RECORDS = {"rs::" + k: v for k, v in RECORD_NAMES.items()}
# C spellings -> canonical
C_ALIASES = {"int": "int32_t", "unsigned": "uint32_t", "hrt_status": "int32_t", "long long": "int64_t"}


def _strip_c_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _rust_blocks(text):
    return re.findall(r"```rust\n(.*?)```", text, flags=re.S)


def _rust_source(text=None):
    text = open(DOC).read() if text is None else text
    src = "\n".join(_rust_blocks(text))
    return re.sub(r"//[^\n]*", "", src)


def patch_files(patch_text):
    """path -> (removed lines, added lines) of every file a unified diff touches."""
    out, cur = {}, None
    for line in patch_text.splitlines():
        if line.startswith("+++ "):
            cur = line[4:].split("\t")[0].split("/", 1)[1]
            out[cur] = ([], [])
        elif line.startswith("--- ") or line.startswith("diff ") or line.startswith("@@"):
            continue
        elif cur and line.startswith("+"):
            out[cur][1].append(line[1:])
        elif cur and line.startswith("-"):
            out[cur][0].append(line[1:])
    return out


def ffi_text(patch_text=None):
    """src/hrt_ffi.rs as the patch adds it (a new file: its added lines are the whole file)."""
    patch_text = open(PATCH).read() if patch_text is None else patch_text
    removed, added = patch_files(patch_text)["src/hrt_ffi.rs"]
    assert not removed
    return "\n".join(added) + "\n"


def _strip_rust_comments(src):
    return re.sub(r"//[^\n]*", "", src)


# ---- Rust side ---------------------------------------------------------------------------------

def _split_top(s, sep=","):
    """Split at top-level separators (not inside [] / () / <>)."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "[(<":
            depth += 1
        elif ch in "])>":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out if x.strip()]


def rust_structs(src):
    """name -> [(field, rust type)] for every #[repr(C)] struct with named fields (opaque ones skipped)."""
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[[^\]]*\]\s*)*pub struct (\w+)\s*\{(.*?)\}", src, flags=re.S):
        fields = []
        for f in _split_top(m.group(2)):
            name, ty = [x.strip() for x in f.split(":", 1)]
            name = name.replace("pub ", "").strip()
            fields.append((name, ty))
        if all(n.startswith("_") for n, _ in fields):
            continue  # opaque handle (`_p: [u8; 0]`)
        out[m.group(1)] = fields
    return out


def rust_consts(src):
    return {m.group(1): int(m.group(3), 0)
            for m in re.finditer(r"pub const (\w+)\s*:\s*(\w+)\s*=\s*(-?(?:0x[0-9A-Fa-f]+|\d+))\s*;", src)}


def rust_fns(src):
    """name -> (params [(name, type)], return type or None) from every extern "C" block."""
    out = {}
    for blk in re.finditer(r'extern\s+"C"\s*\{(.*?)\n\}', src, flags=re.S):
        for m in re.finditer(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+?))?\s*;", blk.group(1), flags=re.S):
            params = []
            for p in _split_top(m.group(2)):
                pn, pt = [x.strip() for x in p.split(":", 1)]
                params.append((pn, " ".join(pt.split())))
            ret = " ".join(m.group(3).split()) if m.group(3) else None
            assert m.group(1) not in out or out[m.group(1)] == (params, ret), f"{m.group(1)} declared twice, differently"
            out[m.group(1)] = (params, ret)
    return out


def rust_canon(ty):
    """Canonical form of a Rust FFI type: ('ptr', const, pointee) / ('scalar', c type) / ('record', c struct)
    / ('array', elem, n)."""
    ty = ty.strip()
    m = re.match(r"\*(mut|const)\s+(.*)$", ty)
    if m:
        return ("ptr", m.group(1) == "const", rust_canon(m.group(2)))
    m = re.match(r"\[(.*);\s*(\d+)\]$", ty)
    if m:
        return ("array", rust_canon(m.group(1)), int(m.group(2)))
    if ty in RUST_SCALARS:
        return ("scalar", RUST_SCALARS[ty][0])
    if ty in RUST_RECORDS:
        return ("record", RUST_RECORDS[ty])
    if ty in RECORD_NAMES:
        return ("record", RECORD_NAMES[ty])
    if re.match(r"hrt_\w+$", ty):
        return ("record", ty)
    raise AssertionError(f"unknown Rust FFI type {ty!r}")


def rust_layout(fields, structs):
    """repr(C) layout: (size, align, [offset per field])."""
    def size_align(ty):
        c = rust_canon(ty)
        if c[0] == "ptr":
            return 8, 8
        if c[0] == "scalar":
            _, s, a = next(v for v in RUST_SCALARS.values() if v[0] == c[1])
            return s, a
        if c[0] == "array":
            m = re.match(r"\[(.*);\s*(\d+)\]$", ty.strip())
            s, a = size_align(m.group(1))
            return s * int(m.group(2)), a
        name = next((k for k in structs if RECORD_NAMES.get(k, k) == c[1]), None)
        assert name, f"record {c[1]} has no #[repr(C)] declaration in the binding"
        s, a, _ = rust_layout(structs[name], structs)
        return s, a
    off, align, offs = 0, 1, []
    for _, ty in fields:
        s, a = size_align(ty)
        off = (off + a - 1) // a * a
        offs.append(off)
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


# ---- C side --------------------------------------------------------------------------------------

def c_source():
    return _strip_c_comments(open(HEADER).read())


def c_structs(src):
    """name -> [(field, c type, array length or None)] of every `typedef struct name {...} name;`."""
    out = {}
    for m in re.finditer(r"typedef struct (\w+)\s*\{(.*?)\}\s*(\w+)\s*;", src, flags=re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            dm = re.match(r"((?:const )?[\w ]+?\**)\s+(.*)$", decl)
            base, names = dm.group(1), dm.group(2)
            for nm in names.split(","):
                nm = nm.strip()
                am = re.match(r"(\w+)\s*\[(\w+)\]$", nm)
                fields.append((am.group(1), base, am.group(2)) if am else (nm, base, None))
        out[m.group(3)] = fields
    return out


def c_values(src):
    """Enumerator and #define values of the header."""
    vals = {}
    for blk in re.finditer(r"(?:typedef )?enum \w*\s*\{(.*?)\}", src, flags=re.S):
        nxt = 0
        for item in blk.group(1).split(","):
            item = item.strip()
            if not item:
                continue
            m = re.match(r"(\w+)\s*(?:=\s*(.+))?$", item, flags=re.S)
            nxt = int(m.group(2).strip(), 0) if m.group(2) else nxt
            vals[m.group(1)] = nxt
            nxt += 1
    for m in re.finditer(r"#define (HRT_\w+)\s+(0x[0-9A-Fa-f]+|\d+)u?\b", src):
        vals[m.group(1)] = int(m.group(2), 0)
    return vals


def _unconst(t):
    return " ".join(re.sub(r"\bconst\b", " ", t).split())


def c_canon_type(t):
    t = " ".join(t.replace("*", " * ").split())
    stars = t.count("*")
    if stars:
        # outer pointer: the qualifiers between the previous '*' (or the start) and the last '*'
        i = t.rfind("*")
        pointee = t[:i].strip()
        j = pointee.rfind("*")
        own = pointee[j + 1:] if j >= 0 else pointee
        return ("ptr", "const" in own.split(), c_canon_type(_unconst(pointee) if j < 0 else pointee))
    t = _unconst(t)
    t = C_ALIASES.get(t, t)
    if t in {v[0] for v in RUST_SCALARS.values()}:
        return ("scalar", t)
    if t.startswith("hrt_"):
        return ("record", t)
    raise AssertionError(f"unknown C type {t!r}")


def c_fns(src):
    """name -> ([canonical param types], canonical return or None)."""
    out = {}
    for m in re.finditer(r"([\w][\w \*]*?)\b(hrt_\w+)\s*\(([^()]*)\)\s*;", src):
        ret, name, params = " ".join(m.group(1).split()), m.group(2), m.group(3).strip()
        if ret.startswith("typedef") or "(" in ret:
            continue
        plist = []
        if params and params != "void":
            for p in params.split(","):
                p = " ".join(p.split())
                am = re.match(r"(.*?)(\w+)\s*\[\w+\]$", p)
                if am:  # `const uint8_t id[N]` is a pointer parameter
                    plist.append(c_canon_type(am.group(1) + "*"))
                    continue
                pm = re.match(r"(.*?[\s\*])(\w+)$", p)
                plist.append(c_canon_type(pm.group(1)))
        out[name] = (plist, None if ret == "void" else c_canon_type(ret))
    return out


def c_layout(structs, names):
    """(sizeof, {field: offsetof}) per struct, compiled from the header by gcc."""
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void) {"]
    for s in names:
        lines.append(f'  printf("{s} size %zu\\n", sizeof({s}));')
        for f, _, _ in structs[s]:
            lines.append(f'  printf("{s} {f} %zu\\n", offsetof({s}, {f}));')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        open(c, "w").write("\n".join(lines) + "\n")
        subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-o", exe, c], check=True, capture_output=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    res = {}
    for line in out.splitlines():
        s, k, v = line.split()
        res.setdefault(s, [0, {}])
        if k == "size":
            res[s][0] = int(v)
        else:
            res[s][1][k] = int(v)
    return res


# ---- checks --------------------------------------------------------------------------------------

def _flat_array(c):
    """('array', elem, n) nests -> (scalar elem, total element count); anything else unchanged."""
    n = 1
    while c[0] == "array":
        n *= c[2]
        c = c[1]
    return c, n


def check_binding(text, rust=False, complete=True):
    """Every mismatch between the binding in `text` (INTEGRATION.md's ```rust blocks, or Rust source
    when rust=True) and the header, as strings.  complete: every public header function must be
    declared (the binding itself; INTEGRATION.md only quotes excerpts)."""
    errs = []
    rsrc, csrc = (_strip_rust_comments(text) if rust else _rust_source(text)), c_source()
    rs, cs = rust_structs(rsrc), c_structs(csrc)
    cname = {n: RECORD_NAMES.get(n, n) for n in rs}
    layouts = c_layout(cs, sorted({cname[n] for n in rs if cname[n] in cs}))
    for name, fields in rs.items():
        if cname[name] not in cs:
            errs.append(f"struct {name}: not in the header")
            continue
        cf = cs[cname[name]]
        if [f for f, _ in fields] != [f for f, _, _ in cf]:
            errs.append(f"struct {name}: fields {[f for f, _ in fields]} != header {[f for f, _, _ in cf]}")
            continue
        for (fn, rty), (_, cty, n) in zip(fields, cf):
            got = rust_canon(rty)
            if n:  # C `T x[n]` against Rust [T; n] (or nested arrays of the same element count)
                want = (c_canon_type(cty), int(n))
                got = _flat_array(got) if got[0] == "array" else (got, None)
            else:
                want = c_canon_type(cty)
            if got != want:
                errs.append(f"struct {name}.{fn}: Rust {rty} != C {cty}{'[' + n + ']' if n else ''}")
        size, _, offs = rust_layout(fields, rs)
        csize, coffs = layouts[cname[name]]
        if size != csize:
            errs.append(f"struct {name}: Rust repr(C) size {size} != C sizeof {csize}")
        for (fn, _), o in zip(fields, offs):
            if coffs[fn] != o:
                errs.append(f"struct {name}.{fn}: Rust offset {o} != C offsetof {coffs[fn]}")
    cfn = c_fns(csrc)
    rfn = rust_fns(rsrc)
    for name, (params, ret) in rfn.items():
        if name not in cfn:
            errs.append(f"fn {name}: not in the header")
            continue
        cparams, cret = cfn[name]
        if len(params) != len(cparams):
            errs.append(f"fn {name}: {len(params)} parameters, header {len(cparams)}")
            continue
        for (pn, pt), ct in zip(params, cparams):
            if rust_canon(pt) != ct:
                errs.append(f"fn {name}({pn}): Rust {pt} != C {ct}")
        rret = rust_canon(ret) if ret else None
        if rret != cret:
            errs.append(f"fn {name}: returns Rust {ret} != C {cret}")
    public = {n for n in cfn if not n.startswith("hrt_debug_") or n == "hrt_debug_build"}
    for name in sorted(public - set(rfn) if complete else ()):
        errs.append(f"fn {name}: in the header, missing from the binding")
    vals = c_values(csrc)
    for name, v in rust_consts(rsrc).items():
        if name not in vals:
            errs.append(f"const {name}: not in the header")
        elif vals[name] != v:
            errs.append(f"const {name} = {v}, header {vals[name]}")
    return errs


def test_binding_matches_header():
    errs = check_binding(ffi_text(), rust=True)
    assert not errs, "\n".join(errs)


def test_integration_excerpts_match_header():
    errs = check_binding(open(DOC).read(), complete=False)
    assert not errs, "\n".join(errs)


def test_binding_declares_the_abi_records():
    rs = rust_structs(_strip_rust_comments(ffi_text()))
    assert {"hrt_create_info", "hrt_stats", "hrt_layout"} | set(RECORD_NAMES) <= set(rs)
    size, align, _ = rust_layout(rs["hrt_stats"], rs)
    assert (size, align) == (64, 8)
    size, align, offs = rust_layout(rs["PushConstants"], rs)
    assert (size, align, offs[2], offs[-1]) == (124, 4, 80, 120)


def test_checker_catches_the_r04_drift():
    """The r04 text: hrt_stats without ABI 4's last_frames / reserved (56 B against 64 B)."""
    text = ffi_text()
    old = re.sub(r"\n\s*pub last_frames: u32,\n\s*pub reserved: u32,", "", text)
    assert old != text
    errs = check_binding(old, rust=True)
    assert any("struct hrt_stats" in e for e in errs), errs


def _swap_lines(text, a, b):
    lines = text.split("\n")
    i = next(k for k, ln in enumerate(lines) if ln.strip() == a)
    j = next(k for k, ln in enumerate(lines) if ln.strip() == b)
    lines[i], lines[j] = lines[j], lines[i]
    return "\n".join(lines)


@pytest.mark.parametrize("edit, what", [
    (lambda t: t.replace("pub fn hrt_compute_n(ctx: *mut hrt_context, pc: *const rs::PushConstants, n: u32)",
                         "pub fn hrt_compute_n(ctx: *mut hrt_context, pc: *const rs::PushConstants)"), "fn hrt_compute_n"),
    (lambda t: re.sub(r"HRT_ABI_VERSION: u32 = (\d+);", lambda m: f"HRT_ABI_VERSION: u32 = {int(m.group(1)) + 1};", t),
     "HRT_ABI_VERSION"),
    (lambda t: t.replace("bytes: usize) -> i32;", "bytes: u32) -> i32;", 1), "fn hrt_read_image"),
    (lambda t: t.replace("    pub fn hrt_reset_stats(ctx: *mut hrt_context) -> i32;\n", ""), "hrt_reset_stats"),
    # a shifted push-block field (the block of src/raytrace_pipeline.rs:243-257 packed into the wrong slot)
    (lambda t: _swap_lines(t, "pub num_samples: i32,", "pub jitter_size: f32,"), "struct PushConstants"),
    (lambda t: t.replace("pub cam_alignment_mat: [[f32; 4]; 4],", "pub cam_alignment_mat: [[f32; 4]; 3],"),
     "struct PushConstants"),
    (lambda t: _swap_lines(t, "pub first_index: u32,", "pub len: u32,"), "struct Mesh"),
    (lambda t: t.replace("pub centre: [f32; 3],", "pub centre: [f32; 4],"), "struct Sphere"),
])
def test_checker_catches_edits(edit, what):
    text = ffi_text()
    changed = edit(text)
    assert changed != text, what
    errs = check_binding(changed, rust=True)
    assert any(what in e for e in errs), errs


def test_header_static_asserts_compile_in_c_and_cpp():
    """The header itself pins the records' sizes and key offsets (static_assert / _Static_assert), as
    INTEGRATION.md says: a C and a C++ translation unit that include it compile."""
    src = open(HEADER).read()
    for rec in ("hrt_stats", "hrt_create_info", "hrt_layout", "hrt_push_constants", "hrt_mesh"):
        assert re.search(r"HRT_STATIC_ASSERT\(sizeof\(" + rec + r"\)", src), rec
    with tempfile.TemporaryDirectory() as d:
        for lang, cc in (("c", ["gcc", "-std=c11"]), ("cpp", ["g++", "-std=c++17"])):
            f = os.path.join(d, "t." + lang)
            open(f, "w").write(f'#include "{HEADER}"\nint main(void) {{ return 0; }}\n')
            subprocess.run(cc + ["-Wall", "-Werror", "-c", "-o", os.path.join(d, "t.o"), f], check=True)
