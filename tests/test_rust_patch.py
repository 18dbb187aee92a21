"""integration/epq_raytracer.patch -- the drop-in as a change to the reference's own Rust tree (SURVEY.md
8(f)1) -- checked mechanically on the CPU.  No Rust toolchain exists in this image, so nothing here
compiles it; what is checked is what a reviewer of the patch would check by hand:

* it applies exactly (no fuzz, no offsets) to /root/reference (test skipped where that tree is absent);
* no Vulkano compute remains in src/raytrace_pipeline.rs / src/diffuse.rs (no ComputePipeline, no
  descriptor sets, no `.dispatch(`, no `shader!` compile of raytracing.glsl / image_combiner.glsl);
* src/raytracing_app.rs changes by one line in the pipeline construction of :91-103, so every public
  item of RayTracingApp, RayTracerSettings and the free functions of :147-227 is untouched, and the
  public methods of RayTracePipeline / DiffusePipeline keep their signatures;
* the push block is packed field by field exactly as :243-257 packs it (same expression per field,
  modulo the renamed count fields), into records whose layout test_rust_binding holds to the header;
* every `raytrace_shader::X { .. }` literal in the patched tree (materials.rs, objects.rs, the
  pipeline) names exactly the fields of the binding's record X, and every HrtContext method the
  pipelines call exists.
"""
import os
import re
import shutil
import subprocess

import pytest

from test_rust_binding import PATCH, _strip_rust_comments, check_binding, ffi_text, patch_files

REF = "/root/reference"
needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree absent")
COUNT_RENAMES = {"self.ray_data.1": "self.num_rays", "self.sphere_data.1": "self.num_spheres",
                 "self.mesh_data.2": "self.num_meshes"}


def apply_patch(tmp_path, patch_text=None):
    """A copy of the reference's src/ with the patch applied; returns (tree, patch's stdout)."""
    tree = tmp_path / "ref"
    shutil.copytree(os.path.join(REF, "src"), tree / "src")
    patch_text = open(PATCH).read() if patch_text is None else patch_text
    dry = subprocess.run(["patch", "-p1", "--dry-run", "-d", str(tree)], input=patch_text, text=True,
                         capture_output=True)
    assert dry.returncode == 0, dry.stdout + dry.stderr
    res = subprocess.run(["patch", "-p1", "-d", str(tree)], input=patch_text, text=True, capture_output=True)
    assert res.returncode == 0, res.stdout + res.stderr
    return tree, res.stdout


def read(tree, rel):
    return open(os.path.join(tree, rel)).read()


def pub_fns(src):
    """Normalised signatures of every `pub fn` (generics, parameters, return type), leading '_' of a
    parameter name dropped (an argument the new body no longer reads)."""
    out = {}
    for m in re.finditer(r"pub fn (\w+)\s*(<[^{]*?>)?\s*\((.*?)\)\s*(->\s*[^{]+?)?\s*(where[^{]*)?\{", src, flags=re.S):
        params = ",".join(re.sub(r"^_", "", " ".join(p.split())) for p in m.group(3).split(",") if p.strip())
        out[m.group(1)] = (" ".join((m.group(2) or "").split()), params, " ".join((m.group(4) or "").split()),
                           " ".join((m.group(5) or "").split()))
    return out


def struct_literal(src, path):
    """field -> expression of the first `path { ... }` struct literal in src."""
    m = re.search(r"(?<!-> )" + re.escape(path) + r"\s*\{(.*?)\n\s*\}", src, flags=re.S)
    assert m, path
    fields = {}
    for item in re.split(r",\s*\n", m.group(1).strip().rstrip(",")):
        k, v = item.split(":", 1)
        fields[k.strip()] = " ".join(v.split())
    return fields


def records(ffi):
    body = re.search(r"pub mod records \{(.*?)\n\}", ffi, flags=re.S).group(1)
    return {m.group(1): [f.split(":")[0].replace("pub ", "").strip() for f in m.group(2).split(",") if f.strip()]
            for m in re.finditer(r"pub struct (\w+)\s*\{(.*?)\}", _strip_rust_comments(body), flags=re.S)}


def test_patch_touches_only_the_compute_side():
    files = patch_files(open(PATCH).read())
    assert set(files) == {"build.rs", "src/hrt_ffi.rs", "src/main.rs", "src/raytrace_pipeline.rs",
                          "src/diffuse.rs", "src/raytracing_app.rs"}
    removed, added = files["src/raytracing_app.rs"]
    assert removed == [] and [a.strip() for a in added] == ["diffuse_pipeline.share_context(&raytrace_pipeline);"]
    assert files["src/main.rs"] == ([], ["mod hrt_ffi;"])
    assert "cargo:rustc-link-lib=dylib=hip_raytrace" in "\n".join(files["build.rs"][1])


def test_patched_binding_matches_header():
    assert not check_binding(ffi_text(), rust=True)


@needs_ref
def test_patch_applies_exactly(tmp_path):
    _, out = apply_patch(tmp_path)
    assert not re.search(r"offset|fuzz|FAILED|Reversed|rej", out), out


@needs_ref
def test_no_vulkano_compute_left(tmp_path):
    tree, _ = apply_patch(tmp_path)
    for rel in ("src/raytrace_pipeline.rs", "src/diffuse.rs"):
        src = read(tree, rel)
        for banned in ("ComputePipeline", "PersistentDescriptorSet", "WriteDescriptorSet", ".dispatch(",
                       "shader!", "bind_pipeline_compute", "push_constants(pipeline_layout", "PipelineLayout"):
            assert banned not in src, (rel, banned)
    # the GLSL compute shaders are no longer compiled into the binary; the present pass's are
    assert "shader!" in read(tree, "src/texture_draw_pipeline.rs")


@needs_ref
def test_public_surface_unchanged(tmp_path):
    tree, _ = apply_patch(tmp_path)
    orig = {rel: read(REF, rel) for rel in ("src/raytracing_app.rs", "src/raytrace_pipeline.rs", "src/diffuse.rs")}
    new = {rel: read(tree, rel) for rel in orig}
    # RayTracingApp / RayTracerSettings / free functions: every pub fn and pub struct body identical
    assert pub_fns(new["src/raytracing_app.rs"]) == pub_fns(orig["src/raytracing_app.rs"])
    assert len(pub_fns(orig["src/raytracing_app.rs"])) >= 5
    for name in ("RayTracerSettings", "RayTracingApp"):
        pat = r"pub struct " + name + r"[^{]*\{.*?\n\}"
        assert re.search(pat, new["src/raytracing_app.rs"], flags=re.S).group(0) == \
            re.search(pat, orig["src/raytracing_app.rs"], flags=re.S).group(0), name
    # the pipelines: the reference's public methods keep their signatures (new ones may be added)
    for rel in ("src/raytrace_pipeline.rs", "src/diffuse.rs"):
        before, after = pub_fns(orig[rel]), pub_fns(new[rel])
        assert before, rel
        for name, sig in before.items():
            assert after.get(name) == sig, (rel, name, sig, after.get(name))


@needs_ref
def test_push_block_packed_as_the_reference(tmp_path):
    """raytrace_pipeline.rs:243-257, field by field, against the patched push_constants()."""
    tree, _ = apply_patch(tmp_path)
    want = struct_literal(read(REF, "src/raytrace_pipeline.rs"), "raytrace_shader::PushConstants")
    want = {k: COUNT_RENAMES.get(v.split(" as ")[0], v.split(" as ")[0]) + (" as " + v.split(" as ")[1] if " as " in v else "")
            for k, v in want.items()}
    got = struct_literal(read(tree, "src/raytrace_pipeline.rs"), "raytrace_shader::PushConstants")
    assert list(got) == list(want) and got == want
    # and in the order of the binding's record (== the header's, test_rust_binding)
    assert list(got) == records(ffi_text())["PushConstants"]


@needs_ref
def test_patch_with_shifted_push_field_is_caught(tmp_path):
    """A patch whose binding shifts one push-block field fails the header check."""
    text = open(PATCH).read()
    bad = text.replace("+        pub num_samples: i32,\n+        pub jitter_size: f32,\n",
                       "+        pub jitter_size: f32,\n+        pub num_samples: i32,\n")
    assert bad != text
    tree, _ = apply_patch(tmp_path, bad)
    errs = check_binding(read(tree, "src/hrt_ffi.rs"), rust=True)
    assert any("struct PushConstants" in e for e in errs), errs


@needs_ref
def test_record_literals_name_the_binding_fields(tmp_path):
    """Every `raytrace_shader::X { .. }` literal in the patched crate (materials.rs, objects.rs and the
    pipeline's host prep) names exactly record X's fields -- what rustc would check."""
    tree, _ = apply_patch(tmp_path)
    recs = records(read(tree, "src/hrt_ffi.rs"))
    seen = set()
    for rel in sorted(os.listdir(os.path.join(tree, "src"))):
        src = read(tree, os.path.join("src", rel))
        for m in re.finditer(r"(?<!-> )raytrace_shader::(\w+)\s*\{", src):  # literals, not return types
            i, depth = m.end(), 1
            while depth:
                depth += {"{": 1, "}": -1}.get(src[i], 0)
                i += 1
            body = src[m.end():i - 1]
            names, depth, cur = [], 0, ""
            for ch in body:
                depth += {"(": 1, "[": 1, "{": 1, ")": -1, "]": -1, "}": -1}.get(ch, 0)
                if ch == "," and depth == 0:
                    names.append(cur)
                    cur = ""
                else:
                    cur += ch
            names.append(cur)
            fields = [n.split(":")[0].strip() for n in names if n.strip()]
            assert m.group(1) in recs, (rel, m.group(1))
            assert sorted(fields) == sorted(recs[m.group(1)]), (rel, m.group(1), fields)
            seen.add(m.group(1))
    assert {"RayTracingMaterial", "Sphere", "Triangle", "Mesh", "Ray", "PushConstants"} <= seen


@needs_ref
def test_pipeline_calls_exist_in_binding(tmp_path):
    tree, _ = apply_patch(tmp_path)
    ffi = read(tree, "src/hrt_ffi.rs")
    methods = set(re.findall(r"pub fn (\w+)\s*\(", ffi.split("impl HrtContext")[1].split("impl Drop")[0]))
    for rel in ("src/raytrace_pipeline.rs", "src/diffuse.rs"):
        src = read(tree, rel)
        for name in re.findall(r"\bhrt\.(\w+)\(", src):
            assert name in methods | {"clone", "as_ref"}, (rel, name)  # (of the Rc / the Option)
        for m in re.finditer(r"use super::hrt_ffi::\{([^}]*)\}", src):
            for item in m.group(1).split(","):
                item = item.strip()
                assert re.search(r"\b(pub (struct|type|const|fn|mod) )" + item + r"\b", ffi), (rel, item)
    assert "mod hrt_ffi;" in read(tree, "src/main.rs")
    # braces balance in every patched file (a cheap stand-in for the parser this image lacks)
    for rel in ("src/hrt_ffi.rs", "src/raytrace_pipeline.rs", "src/diffuse.rs", "build.rs"):
        src = re.sub(r'"(\\.|[^"\\])*"', '""', _strip_rust_comments(read(tree, rel)))
        assert src.count("{") == src.count("}") and src.count("(") == src.count(")"), rel
