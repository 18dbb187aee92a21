#!/usr/bin/env python3
"""Regenerates tools/exp/phase_experiments.patch against the current product sources.

The timing-only phase experiments (-DHRT_EXP_TWICE=<phase>: one phase run a second time on opaque
copies of its inputs, the result discarded, so the A/B difference is that phase's marginal cost;
-DHRT_IEEE_DIV: the compiler's division sequences) are kept out of the product sources (VERDICT r02
weak #7).  Phases: 1 primary list (world_hit_tile), 2 raygen, 3 shading, 4 camera tile list,
5 bounce traversal (world_hit_bounce_wq);
-DHRT_EXP_NOBAND: no grazing-band scan (wrong frames, timing only).  tools/ab_build.sh applies the patch when EXP_PATCH=1.

  python3 tools/exp/make_patch.py   (after an edit that moved the anchors below)
"""
import difflib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = "epq_raytracer_amd/csrc"

KERNEL_EDITS = [
    ("namespace hrt {\n\n\n", '''namespace hrt {

#ifdef HRT_EXP_TWICE
__device__ __forceinline__ float exp_zero() {
  float z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}
__device__ __forceinline__ void exp_use(float v) { asm volatile("; use %0" ::"v"(v)); }
#endif

'''),
    ("  const TileList tl = build_tile_list(P, active, centre, list_lds);\n  // bounce batch",
     '''  const TileList tl = build_tile_list(P, active, centre, list_lds);
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 4
  {
    const float z = exp_zero();
    const TileList t2 = build_tile_list(P, active, mk(centre.x + z, centre.y, centre.z), nullptr);
    exp_use((float)t2.n + (float)t2.v + (float)t2.aabb);
  }
#endif
  // bounce batch'''),
    ("        const f3 dir = get_ray_dir(K->pc, centre, state);\n",
     '''        const f3 dir = get_ray_dir(K->pc, centre, state);
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 2
        {
          uint32_t s2 = state + (uint32_t)exp_zero();
          const f3 d2 = normalize(get_ray_dir(K->pc, centre, s2));
          exp_use(d2.x + d2.y + d2.z);
        }
#endif
'''),
    ("        world_hit_tile(HRT_SHADE_KARGS ? kscene() : sc, P, tl, prim, p.pos, p.dir, tests, c);\n",
     '''        world_hit_tile(HRT_SHADE_KARGS ? kscene() : sc, P, tl, prim, p.pos, p.dir, tests, c);
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 1
        {
          const float z = exp_zero();
          Closest c2{kFltMax, 0, 0u, 0u};
          uint32_t t2 = 0;
          world_hit_tile(HRT_SHADE_KARGS ? kscene() : sc, P, tl, prim, p.pos, mk(p.dir.x + z, p.dir.y + z, p.dir.z + z),
                         t2, c2);
          exp_use(c2.t + (float)t2 + (float)c2.idx);
        }
#endif
'''),
    ('''      if constexpr (is_wq(Bounce)) {
        world_hit_bounce_wq<D, Bounce == kBounceWqR>(HRT_SHADE_KARGS ? kscene() : sc, P, bsrc, sec, p.pos, p.dir, tests,
                                                     c, dg);
''', '''      if constexpr (is_wq(Bounce)) {
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 5
        const Closest c_in = c;
#endif
        world_hit_bounce_wq<D, Bounce == kBounceWqR>(HRT_SHADE_KARGS ? kscene() : sc, P, bsrc, sec, p.pos, p.dir, tests,
                                                     c, dg);
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 5
        {
          const float z = exp_zero();
          Closest c2 = c_in;
          uint32_t t2 = 0;
          world_hit_bounce_wq<D, Bounce == kBounceWqR>(HRT_SHADE_KARGS ? kscene() : sc, P, bsrc, sec, p.pos,
                                                       mk(p.dir.x + z, p.dir.y + z, p.dir.z + z), t2, c2, dg);
          exp_use(c2.t + (float)t2 + (float)c2.idx);
        }
#endif
'''),
    ("      total += (uint32_t)__popcll(bb) << b;\n    }\n",
     '''      total += (uint32_t)__popcll(bb) << b;
    }
#ifdef HRT_EXP_NOBAND  // timing only (wrong frames): no grazing-band pairs
    total = 0;
#endif
'''),
    ("      ++segs;\n      const bool ended = shade_step(HRT_SHADE", '''      ++segs;
#if defined(HRT_EXP_TWICE) && HRT_EXP_TWICE == 3
      {
        Path p2 = p;
        p2.dir.x = p2.dir.x + exp_zero();
        uint32_t s2 = state + (uint32_t)exp_zero();
        exp_use((shade_step(HRT_SHADE_KARGS ? kscene() : sc, pc, p2, c, s2) ? 1.0f : 0.0f) + p2.dir.x + p2.dir.y +
                p2.dir.z + p2.light.x + p2.colour.y);
      }
#endif
      const bool ended = shade_step(HRT_SHADE'''),
]

MATH_EDITS = [
    ("__device__ __forceinline__ f3 div3(f3 a, float s) {\n", '''__device__ __forceinline__ f3 div3(f3 a, float s) {
#ifdef HRT_IEEE_DIV  // A/B: the compiler's sequences only
  return {a.x / s, a.y / s, a.z / s};
#endif
'''),
    ("__device__ __forceinline__ f3 normalize(f3 a) {\n", '''__device__ __forceinline__ f3 normalize(f3 a) {
#ifdef HRT_IEEE_DIV
  return a / __builtin_sqrtf(dot(a, a));
#endif
'''),
]


def patched(name, edits):
    src = open(os.path.join(ROOT, CSRC, name)).read()
    out = src
    for old, new in edits:
        if out.count(old) != 1:
            sys.exit(f"{name}: anchor found {out.count(old)} times: {old[:70]!r}")
        out = out.replace(old, new)
    path = f"{CSRC}/{name}"
    diff = difflib.unified_diff(src.splitlines(True), out.splitlines(True), f"b/{path}", f"a/{path}")
    return f"diff --git b/{path} a/{path}\n" + "".join(diff)


def main():
    text = patched("hrt_kernels.hip", KERNEL_EDITS) + patched("hrt_math.h", MATH_EDITS)
    dst = os.path.join(ROOT, "tools/exp/phase_experiments.patch")
    open(dst, "w").write(text)
    print(dst)


if __name__ == "__main__":
    main()
