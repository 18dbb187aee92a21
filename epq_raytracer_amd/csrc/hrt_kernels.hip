// hrt_kernels.hip -- gfx950 kernels for the path-trace dispatch (assets/raytracing.glsl) and the
// progressive accumulator (assets/image_combiner.glsl).
//
// One lane per pixel; each wave owns an 8x8 pixel tile (coherent primary rays), 256-thread
// workgroups (1024 for the LDS-resident scene).  Scene records are read with wave-uniform addresses,
// so triangles stream through SGPRs and every lane tests the same triangle against its own ray.
//
// Kernel variants (hrt_option HRT_OPT_KERNEL_VARIANT, include/hip_raytrace.h), all byte-identical
// to the oracle (tests/test_gpu_parity.py):
//   LITERAL      per-sample / per-bounce loops shaped like raytracing.glsl:308-389, full test on
//                every triangle;
//   BRUTE(_LDS)  the sample and bounce loops fused into one per-lane segment loop (a lane whose path
//                ended starts its next sample), a division-free exact pre-test per triangle in two
//                wave-uniform stages; the correctly rounded 1/det path only runs when some lane may
//                accept (DESIGN.md "exact cull"); triangles via SGPRs or resident in LDS;
//   BUNDLE       primary segments (origin = cam_pos) rejected 64 triangles at a time by bounding the
//                reference's linear forms over the wave's ray directions; bounce segments deferred
//                until a wave has enough of them, then the BRUTE test;
//   BUNDLE_CULL  BUNDLE + a lane-parallel origin-box / direction-cone pre-cull for bounce segments.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "hip_raytrace.h"
#include "hrt_bvh.h"
#include "hrt_kernels.h"
#include "hrt_math.h"

namespace hrt {

#ifndef HRT_TIMELINE
#define HRT_TIMELINE 0  // per-item timeline records (tools/timeline.py; A/B builds only)
#endif
#ifndef HRT_TL_PREPASS
#define HRT_TL_PREPASS 1  // the persistent kernels' whole-tile lists built once per launch (tile_lists, r05)
#endif


#ifndef HRT_SHADE_KARGS
#define HRT_SHADE_KARGS 1  // shading reads the scene pointers from the kernel arguments (kargs)
#endif
#ifndef HRT_RAYGEN_KARGS
#define HRT_RAYGEN_KARGS 1  // the camera read per sample from the kernel arguments (kargs)
#endif

// Read-only views of the uploaded std430 records.
struct Scene {
  const float4* __restrict__ rays;
  const hrt_sphere* __restrict__ spheres;
  const hrt_triangle* __restrict__ tris;
  const hrt_mesh* __restrict__ meshes;
  const float4* __restrict__ nhat;  // normalize(tri.normal) per triangle (tri_normals, same arithmetic)
};

// The kernel arguments through an opaque pointer to the kernarg segment: a field read through it is
// a scalar load at the point of use that the compiler cannot hoist out of the fused loop.  Constants
// needed only inside a phase (a bounce batch, a work item) are read this way at the phase's start, so
// they occupy SGPRs for the phase only instead of for the whole kernel (where ~120 of them were
// spilled into VGPR lanes and read back with v_readlane).
typedef const __attribute__((address_space(4))) TraceParams* KArgs;
__device__ __forceinline__ KArgs kargs() {
  KArgs p = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
// The scene's pointers read at the point of use (shading: after a segment, not held across the loop).
__device__ __forceinline__ Scene kscene() {
  const KArgs K = kargs();
  return Scene{K->rays, K->spheres, K->tris, K->meshes, K->tri_nhat};
}

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 ray_at(f3 o, f3 d, float t) { return o + d * t; }  // :158-160

// lane r's value (r < 64, every caller's index is a lane of this wave): ds_bpermute at r * 4 directly
// (__shfl's width arithmetic added the lane's 64-lane segment base: two VALU per address)
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t r) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(r << 2), (int)v);
}
__device__ __forceinline__ float lane_read(float v, uint32_t r) {
  return __uint_as_float(lane_read(__float_as_uint(v), r));
}
// ray r's mesh filter (its high word only exists with more than 32 meshes)
__device__ __forceinline__ unsigned long long mask_read(unsigned long long m, uint32_t r, int meshes) {
  const uint32_t lo = lane_read((uint32_t)m, r);
  return meshes > 32 ? ((unsigned long long)lane_read((uint32_t)(m >> 32), r) << 32) | lo : lo;
}
__device__ __forceinline__ uint32_t lanes_below(unsigned long long b) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// Exclusive prefix sum of x over the wave's 64 lanes in lane order, and the total (every lane active):
// a Hillis-Steele scan inside each row of 16 lanes by DPP row shifts (lanes past a row's start read 0),
// then each row adds the totals of the rows before it by the row broadcasts of lanes 15 and 31 -- six
// adds with DPP operands instead of a ballot, two lane counts and a shift per bit of x.
// The DPP form is GFX9 wave64 only (row_bcast:15/31 do not exist on GFX10+) and needs every lane active
// (an inactive lane's row sum would be missing from the broadcast): other targets take the ballot scan,
// and HRT_KERNEL_ASSERTS=1 builds check the exec mask on entry.
#ifndef HRT_DPP_SCAN
#define HRT_DPP_SCAN 1
#endif
#ifndef HRT_KERNEL_ASSERTS
#define HRT_KERNEL_ASSERTS 0
#endif
__device__ __forceinline__ uint32_t wave_scan_excl(uint32_t x, uint32_t& total, uint32_t bits = 32u) {
#if HRT_KERNEL_ASSERTS
  if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
#if HRT_DPP_SCAN && (defined(__GFX9__) || !defined(__HIP_DEVICE_COMPILE__))
  (void)bits;
  // (inline: hipcc left each __builtin_amdgcn_mov_dpp as a separate move before a plain add.  Each step
  // reads the previous one's result through DPP, which needs two wait states after a VALU write: the
  // s_nops; in place, so the rows a broadcast's row mask leaves unwritten keep their value, i.e. add 0)
  uint32_t v = x;
  asm volatile(
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
      "s_nop 1\n"
      : "+v"(v));
  total = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  return v - x;
#else
  // bit-plane ballots: x < 2^bits
  uint32_t pos = 0;
  total = 0;
  for (uint32_t b = 0; b < bits; ++b) {
    const unsigned long long bb = __ballot((x >> b) & 1u);
    pos += lanes_below(bb) << b;
    total += (uint32_t)__popcll(bb) << b;
  }
  return pos;
#endif
}

// Cross-lane handoffs through LDS (the pair stacks, the closest-hit slots, the band marks).  A lane's
// store read by ANOTHER lane is a data exchange between threads, so it is written as one: relaxed
// wavefront-scope atomics for the exchanged words and a wavefront-scope acquire-release fence between
// every producer and its consumers (wave_handoff).  On gfx950 these compile to the plain ds_read /
// ds_write and no instruction at all -- a wave's LDS accesses complete in program order -- but they
// stop the compiler from reasoning per lane: with plain accesses it may forward a lane's own store to
// its later load of the same word or move a load above another lane's store (r03: that forwarding lost
// the band marks of lists starting at a lane with no list; tests/test_gpu_boundary.py's protocol tests
// run these helpers through hrt_debug_wq_protocol).
template <class T>
__device__ __forceinline__ void lds_put(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <class T>
__device__ __forceinline__ T lds_get(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
#ifndef HRT_WQ_HANDOFF
#define HRT_WQ_HANDOFF 1
#endif
__device__ __forceinline__ void wave_handoff() {
#if HRT_WQ_HANDOFF
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#endif
}

// local (compacted) row -> global row, hrt_create_info partition.
__device__ __forceinline__ uint32_t global_row(uint32_t lr, const TraceParams& /*P*/) {
  const KArgs K = kargs();  // (once per work item)
  const uint32_t parts = K->part_count, rt = K->row_tile;
  if (parts <= 1) return lr;
  const uint32_t tile = lr / rt, r = lr - tile * rt;
  return (tile * parts + K->part_index) * rt + r;
}

// get_ray_dir, raytracing.glsl:162-166 (u1, u2, u3 in that order)
template <class PC>
__device__ __forceinline__ f3 get_ray_dir(const PC& pc, f3 c, uint32_t& state) {
  // (u01 * 2) * pi: the doubling is exact too, so one multiply by pi 2^-31 (u01_mul)
  const float r = u01_mul(hash(state), 3.14159265358979323846f * 0x1p-31f);
  float sr, cr;
  spec_sincos_angle(r, sr, cr);  // r in [0, 2pi]
  // (r03, measured slower: the zero components of t1 / t2 as signed zeros -- 4.5 M fewer VALU per
  // frame, 2.150 -> 2.163 ms -- and the second normalize's sqrt and reciprocal from the bits of
  // |a|^2 near 1 -- 9 M more, 2.161 ms; profiles/r03/r03p_raygen_ab.jsonl)
  const float j = pc.jitter_size;
  const float s2 = sqrt_rng(u01(hash(state)));
  const f3 t1 = ((mk(0.0f, 0.0f, 1.0f) * cr) * j) * s2;
  const float s3 = sqrt_rng(u01(hash(state)));
  const f3 t2 = ((mk(0.0f, 1.0f, 0.0f) * sr) * j) * s3;
  const f3 nc = (c + t1) + t2;
  const auto& M = pc.cam_alignment_mat;
  const f3 w = mk(__builtin_fmaf(M[8], nc.z, __builtin_fmaf(M[4], nc.y, M[0] * nc.x)),
                  __builtin_fmaf(M[9], nc.z, __builtin_fmaf(M[5], nc.y, M[1] * nc.x)),
                  __builtin_fmaf(M[10], nc.z, __builtin_fmaf(M[6], nc.y, M[2] * nc.x)));
  return normalize_fl(w);
}
#ifndef HRT_NORM_UNIFORM
#define HRT_NORM_UNIFORM 1  // (r04b: with HRT_SKY_ZERO island 1.903 -> 1.876 ms per frame)
#endif
#ifndef HRT_SKY_ZERO
#define HRT_SKY_ZERO 1
#endif
// get_ray_dir for the sky loop (all 64 lanes run it).  Zero: the caller has checked, for the whole
// item, that jitter_size is finite and every active lane's centre has finite c.x != 0 and c.y != 0.  Then the
// zero components of t1 = ((0, 0, 1) cr j) s2 and t2 = ((0, 1, 0) sr j) s3 are signed zeros (cr, sr,
// s2, s3 are finite, s2, s3 >= +0), c.x + t1.x + t2.x == c.x and c.y + t1.y == c.y exactly, and only
// t2.z's sign can matter (when c.z + t1.z is a zero): sign(sr) ^ sign(j).  The same bits as
// get_ray_dir with 8 fewer VALU.
template <bool Zero, class PC>
__device__ __forceinline__ f3 get_ray_dir_sky(const PC& pc, f3 c, uint32_t& state) {
  if constexpr (!Zero) {
#if HRT_NORM_UNIFORM
    const float r = u01_mul(hash(state), 3.14159265358979323846f * 0x1p-31f);  // (u01 * 2) * pi
    float sr, cr;
    spec_sincos_angle(r, sr, cr);
    const float j = pc.jitter_size;
    const float s2 = sqrt_rng(u01(hash(state)));
    const f3 t1 = ((mk(0.0f, 0.0f, 1.0f) * cr) * j) * s2;
    const float s3 = sqrt_rng(u01(hash(state)));
    const f3 t2 = ((mk(0.0f, 1.0f, 0.0f) * sr) * j) * s3;
    const f3 nc = (c + t1) + t2;
    const auto& M = pc.cam_alignment_mat;
    return normalize_wu(mk(__builtin_fmaf(M[8], nc.z, __builtin_fmaf(M[4], nc.y, M[0] * nc.x)),
                           __builtin_fmaf(M[9], nc.z, __builtin_fmaf(M[5], nc.y, M[1] * nc.x)),
                           __builtin_fmaf(M[10], nc.z, __builtin_fmaf(M[6], nc.y, M[2] * nc.x))));
#else
    return get_ray_dir(pc, c, state);
#endif
  } else {
    const float r = u01_mul(hash(state), 3.14159265358979323846f * 0x1p-31f);  // (u01 * 2) * pi
    float sr, cr;
    spec_sincos_angle(r, sr, cr);
    const float j = pc.jitter_size;
    const float s2 = sqrt_rng(u01(hash(state)));
    const float t1z = (cr * j) * s2;  // ((1 cr) j) s2
    const float s3 = sqrt_rng(u01(hash(state)));
    const float t2y = (sr * j) * s3;
    const float z2 = bitsf((fbits(sr) ^ fbits(j)) & 0x80000000u);  // t2.z = ((0 sr) j) s3
    const f3 nc = mk(c.x, c.y + t2y, (c.z + t1z) + z2);
    const auto& M = pc.cam_alignment_mat;
    const f3 w = mk(__builtin_fmaf(M[8], nc.z, __builtin_fmaf(M[4], nc.y, M[0] * nc.x)),
                    __builtin_fmaf(M[9], nc.z, __builtin_fmaf(M[5], nc.y, M[1] * nc.x)),
                    __builtin_fmaf(M[10], nc.z, __builtin_fmaf(M[6], nc.y, M[2] * nc.x)));
    return HRT_NORM_UNIFORM ? normalize_wu(w) : normalize(w);
  }
}

// intersecting_aabb, raytracing.glsl:192-210, restated with its min/max quirks (:202, :206); inv =
// (1/d.x, 1/d.y, 1/d.z) correctly rounded (computed once per ray for all meshes).
__device__ __forceinline__ bool aabb_pass_inv(const hrt_mesh& m, f3 o, f3 inv) {
  float d_max = (((inv.x < 0.0f) ? m.min_point[0] : m.max_point[0]) - o.x) * inv.x;
  float d_min = (((inv.x < 0.0f) ? m.max_point[0] : m.min_point[0]) - o.x) * inv.x;
  if (d_max > 0.0f || d_min > 0.0f) return true;
  d_max = gmax(d_max, (((inv.y < 0.0f) ? m.min_point[1] : m.max_point[1]) - o.y) * inv.y);
  d_min = gmin(d_max, (((inv.y < 0.0f) ? m.max_point[1] : m.min_point[1]) - o.y) * inv.y);
  if (d_max > 0.0f || d_min > 0.0f) return true;
  d_max = gmax(d_max, (((inv.z < 0.0f) ? m.min_point[2] : m.max_point[2]) - o.z) * inv.z);
  d_min = gmax(d_min, (((inv.z < 0.0f) ? m.max_point[2] : m.min_point[2]) - o.z) * inv.z);
  return d_max > 0.0f || d_min > 0.0f;
}
__device__ __forceinline__ bool aabb_pass(const hrt_mesh& m, f3 o, f3 d) {
  return aabb_pass_inv(m, o, mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z));
}

// Result of world_hit: closest distance and what produced it (kind 0 none, 1 sphere, 2 triangle).
struct Closest {
  float t;
  int kind;
  uint32_t idx;   // sphere index or triangle index
  uint32_t mesh;  // mesh index (kind 2)
};

// intersecting_sphere, raytracing.glsl:169-190; returns dist or FLT_MAX (miss).
__device__ __forceinline__ float sphere_dist(const hrt_sphere& s, f3 o, f3 d) {
  const f3 l = o - ld3(s.centre);
  const float a = dot(d, d);
  const float half_b = dot(d, l);
  const float c = dot(l, l) - s.radius * s.radius;
  const float disc = half_b * half_b - a * c;
  if (disc >= 0.0f) return (-half_b - __builtin_sqrtf(disc)) / a;
  return kFltMax;
}

// Exact intersecting_tri (raytracing.glsl:213-241) acceptance against a running closest t:
// true iff the reference returns a hit with 0.001 < dist < best (every early return is a miss).
__device__ __forceinline__ bool tri_accept_exact(const hrt_triangle& tri, f3 o, f3 d, float best, float& t_out) {
  const f3 n = ld3(tri.normal);
  const float dn = dot(d, n);
  const f3 ao = o - ld3(tri.a);
  const f3 dao = cross(ao, d);
  const float det = -dn;
  const float inv_det = 1.0f / det;
  const float dist = dot(ao, n) * inv_det;
  const float u = dot(ld3(tri.edge_two), dao) * inv_det;
  const float v = -dot(ld3(tri.edge_one), dao) * inv_det;
  const float w = 1.0f - u - v;
  t_out = dist;
  return !(dn >= 0.0f) && !(det == 0.0f) && !(dist < 0.0f) && !(u < 0.0f) && !(v < 0.0f) && !(w < 0.0f) &&
         dist > 0.001f && dist < best;
}

// world_hit, raytracing.glsl:267-288.  Spheres first, then meshes, strict '<' against one running
// closest (equivalent to the reference's per-mesh closest + world compare: the first triangle in
// buffer order attaining the minimum wins either way).
__device__ __forceinline__ Closest world_hit_literal(const Scene& sc, const hrt_push_constants& pc, f3 o, f3 d,
                                                     uint32_t& tests) {
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    if (!aabb_pass(mesh, o, d)) continue;
    tests += mesh.len;
    const uint32_t end = mesh.first_index + mesh.len;
    for (uint32_t i = mesh.first_index; i < end; ++i) {
      float t;
      if (tri_accept_exact(sc.tris[i], o, d, c.t, t)) c = Closest{t, 2, i, (uint32_t)m};
    }
  }
  return c;
}

struct HitRecord {
  f3 normal, pos;
  const hrt_material* mat;
};

__device__ __forceinline__ HitRecord resolve_hit(const Scene& sc, const Closest& c, f3 o, f3 d) {
  HitRecord h;
  h.pos = ray_at(o, d, c.t);
  if (c.kind == 1) {
    const hrt_sphere& s = sc.spheres[c.idx];
    h.normal = normalize(h.pos - ld3(s.centre));
    h.mat = &s.material;
  } else {
    const float4 nh = sc.nhat[c.idx];  // = normalize(ld3(sc.tris[c.idx].normal)), computed once per scene
    h.normal = mk(nh.x, nh.y, nh.z);
    h.mat = &sc.meshes[c.mesh].material;
  }
  return h;
}

// environment_light, raytracing.glsl:290-294
template <class PC>
__device__ __forceinline__ f3 environment_light(const PC& pc, f3 d) {
  if (!pc.use_environment_light) return mk(0.0f, 0.0f, 0.0f);
  const float a = 0.5f * (d.y + 1.0f);
  const float oma = 1.0f - a;
  return mk(oma * 1.0f + a * 0.5f, oma * 1.0f + a * 0.7f, oma * 1.0f + a * 1.0f);
}

// adjust_dir, raytracing.glsl:297-305 (both unit-sphere draws always happen: 12 hashes)
#ifndef HRT_FUZZ_FAST
#define HRT_FUZZ_FAST 1
#endif
#ifndef HRT_FUZZ_INT
#define HRT_FUZZ_INT 1  // the fast path's radius test on the hash bits (r03ai)
#endif
__device__ __forceinline__ f3 adjust_dir(f3 d, f3 n, const hrt_material& mat, bool specular, uint32_t& state) {
  const f3 diffuse_dir = normalize_fl(n + unit_sphere(state));
  const float k = 2.0f * dot(n, d);
  const f3 specular_dir = d - n * k;
  const float a = mat.settings[1] * (float)(int)specular;
  const float oma = 1.0f - a;
#if HRT_FUZZ_FAST
  // Without fuzz and specular blend (settings[2] == +-0, a == +-0: a Lambertian hit), mixed + fuzz is
  // diffuse_dir * 1 + specular_dir * (+-0) + unit_sphere * (+-0) component by component, i.e.
  // diffuse_dir itself when each of its components is finite and nonzero (adding a signed zero keeps
  // it), specular_dir is finite, and the fuzz draw is finite: each of its three normal_dist radii
  // sqrt(-2 log u) is finite and nonzero exactly when u01 of its second hash is neither 0 nor 1
  // (spec_log(1) = +0, spec_log(0) = -inf; cos of the angle is never 0, hrt_math.h), so its length
  // is not 0.  Such a lane only advances the RNG by the draw's six hashes.
  const float fz = mat.settings[2];
  uint32_t st = state;
  bool fast = a == 0.0f && fz == 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    hash(st);  // the angle's
#if HRT_FUZZ_INT
    // u01(h) = RN(h) 2^-32 is 0 iff h == 0 and 1 iff RN(h) == 2^32, i.e. h >= 2^32 - 128 (the u32 -> f32
    // conversion rounds to nearest even: 2^32 - 128 is a tie between 2^32 - 256 (odd) and 2^32), so
    // the radius test is one integer compare instead of a conversion, a multiply and two compares
    fast &= hash(st) - 1u < 0xFFFFFF7Fu;
#else
    const float u = u01(hash(st));
    fast &= u != 0.0f && u != 1.0f;
#endif
  }
  const bool finite_nz = fabsf(diffuse_dir.x) < __builtin_inff() && fabsf(diffuse_dir.y) < __builtin_inff() &&
                         fabsf(diffuse_dir.z) < __builtin_inff() && diffuse_dir.x != 0.0f && diffuse_dir.y != 0.0f &&
                         diffuse_dir.z != 0.0f;
  const bool spec_ok = fabsf(specular_dir.x) < __builtin_inff() && fabsf(specular_dir.y) < __builtin_inff() &&
                       fabsf(specular_dir.z) < __builtin_inff();
  if (fast && finite_nz && spec_ok) {
    state = st;
    return normalize_fl(diffuse_dir);
  }
#endif
  const f3 fuzz = unit_sphere(state) * mat.settings[2];
  const f3 mixed = mk(diffuse_dir.x * oma + specular_dir.x * a, diffuse_dir.y * oma + specular_dir.y * a,
                      diffuse_dir.z * oma + specular_dir.z * a);
  return normalize_fl(mixed + fuzz);
}

// Per-lane path state of trace_ray (raytracing.glsl:308-352).
struct Path {
  f3 light, colour, pos, dir;
  int bounce;       // loop index i of :316
  bool not_visible; // has_not_hit_visible_object
};

// One iteration of trace_ray's loop body after world_hit (:318-346).  Returns true when the path
// has ended (break); the caller then adds light*colour.
__device__ __forceinline__ bool shade_step(const Scene& sc, const hrt_push_constants& pc, Path& p, const Closest& c,
                                           uint32_t& state) {
  if (c.kind != 0) {  // hit.hit_dist < FLT_MAX
    const HitRecord hit = resolve_hit(sc, c, p.pos, p.dir);
    const hrt_material& m = *hit.mat;
    const bool invis = (m.settings[3] == 1.0f);
    p.pos = adds(hit.pos, (float)(int)invis * 0.001f);
    if (invis && p.not_visible) {
      p.pos = hit.pos + p.dir * 0.001f;
      return false;  // continue
    }
    p.not_visible = false;
    const bool is_spec = u01(hash(state)) < m.settings[0];
    p.dir = adjust_dir(p.dir, hit.normal, m, is_spec, state);
    const f3 emitted = ld3(m.emission) * m.emission[3];
    p.light = p.light + emitted * p.colour;
    p.colour = p.colour * ld3(m.colour);
    const float prob = gmax(p.colour.x, gmax(p.colour.y, p.colour.z));
    if (u01(hash(state)) >= prob) return true;
    p.colour = div3(p.colour, prob);
    return false;
  }
  p.light = p.light + environment_light(pc, p.dir);
  return true;
}

__device__ __forceinline__ void store_pixel(const TraceParams& /*P*/, uint32_t x, uint32_t lr, f3 col,
                                            uint32_t frame = 0) {
  const KArgs K = kargs();  // (once per work item)
  const size_t idx = (size_t)lr * K->pc.width + x + frame * K->frame_stride;
  uint32_t* img8 = K->img8;
  float4* img32 = K->img32;
  if (img8) img8[idx] = unorm8(col.x) | (unorm8(col.y) << 8) | (unorm8(col.z) << 16) | (255u << 24);
  if (img32) img32[idx] = make_float4(col.x, col.y, col.z, 1.0f);
}

// wave-level sums of the per-lane counters (+ the wave's longest lane), in every lane.
__device__ __forceinline__ void wave_counters(uint32_t segs, uint32_t tests, unsigned long long& s,
                                              unsigned long long& t, uint32_t& mx) {
  s = segs;
  t = tests;
  mx = segs;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    t += __shfl_xor(t, off, 64);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
}
__device__ __forceinline__ void add_counters(const TraceParams& /*P*/, unsigned long long s, unsigned long long t,
                                             unsigned long long mx) {
  unsigned long long* counters = kargs()->counters;
  if (counters && (threadIdx.x & 63) == 0) {
    atomicAdd(&counters[0], s);
    atomicAdd(&counters[1], t);
    atomicAdd(&counters[2], mx);
  }
}
// one atomic each per wave
__device__ __forceinline__ void flush_counters(const TraceParams& P, uint32_t segs, uint32_t tests) {
  if (!kargs()->counters) return;
  unsigned long long s, t;
  uint32_t mx;
  wave_counters(segs, tests, s, t, mx);
  add_counters(P, s, t, mx);
}

__device__ __forceinline__ void lane_pixel(const TraceParams& P, uint32_t& x, uint32_t& lr) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
  lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
}

// ---- literal variant: raytracing.glsl main (:355-389) with trace_ray's loop as written ----------
__global__ __launch_bounds__(256) void trace_literal(TraceParams P) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes, P.tri_nhat};
  const hrt_push_constants& pc = P.pc;
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  const uint32_t y = global_row(lr, P);
  uint32_t segs = 0, tests = 0;
  if (x < pc.width && lr < P.local_rows && y < pc.height) {
    const uint32_t id = x + y * pc.width;
    f3 colour = mk(0.0f, 0.0f, 0.0f);
    uint32_t state = pc.rng_offset * 719393u + id;
    const float4 rc = sc.rays[id];
    const f3 centre = mk(rc.x, rc.y, rc.z);
    const f3 root = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
    for (int s = 0; s < pc.num_samples; ++s) {
      const f3 dir = get_ray_dir(pc, centre, state);
      Path p{mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), root, normalize(dir), 0, true};
      for (int i = 0; i <= pc.max_bounces; ++i) {
        const Closest c = world_hit_literal(sc, pc, p.pos, p.dir, tests);
        ++segs;
        if (shade_step(sc, pc, p, c, state)) break;
      }
      colour = colour + p.light * p.colour;
    }
    colour = div3(colour, (float)pc.num_samples);
    store_pixel(P, x, lr, colour);
  }
  flush_counters(P, segs, tests);
}

// ---- exact pre-test shared by the tuned variants ----------------------------------------------------
//
// Exact cull (proof in DESIGN.md): with det = -dot(d,n) > 0 and inv = RN(1/det) > 0, the reference
// can only accept a triangle if none of these division-free rejections holds (when det >= 2^-60):
//   R6  num_t <  RN(det * 0.000999)           (then dist < 0.001)
//   R3  num_u < -RN(det * 2^-60)              (then u = RN(num_u*inv) < 0, no underflow to -0)
//   R4  num_v >  RN(det * 2^-60)              (then v < 0)
//   R5  RN(num_u - num_v) > RN(det * (1+2^-16))   (then w = 1-u-v < 0)
//   R7  num_t >  RN(best_k * det), best_k = RN(best * (1+2^-16))   (then dist > best)
// A lane that passes the pre-test is only a candidate; the exact reference expression decides.
constexpr float kTiny = 8.673617379884035e-19f;   // 2^-60
constexpr float kOnePlus = 1.0000152587890625f;   // 1 + 2^-16
constexpr float kTMin = 0.000999f;

// Division-free quantities of one triangle test, computed exactly as the reference does.
struct TriPre {
  float num_t, num_u, num_v, det;
  bool cand;
};

__device__ __forceinline__ bool pre_reject(const TriPre& q, float best_k) {
  const float tiny = q.det * kTiny;
  const bool r = (q.num_t < q.det * kTMin) | (q.num_u < -tiny) | (q.num_v > tiny) |
                 ((q.num_u - q.num_v) > q.det * kOnePlus) | (q.num_t > best_k * q.det);
  return r & !(q.det < kTiny);
}

// The reference's remaining arithmetic (raytracing.glsl:227-238) for a candidate lane.
__device__ __forceinline__ void tri_exact(const TriPre& q, uint32_t i, uint32_t m, Closest& c, float& best_k) {
  const float inv_det = 1.0f / q.det;
  const float dist = q.num_t * inv_det;
  const float u = q.num_u * inv_det;
  const float v = -q.num_v * inv_det;
  const float w = 1.0f - u - v;
  if (!(dist < 0.0f) && !(u < 0.0f) && !(v < 0.0f) && !(w < 0.0f) && dist > 0.001f && dist < c.t) {
    c = Closest{dist, 2, i, m};
    best_k = dist * kOnePlus;
  }
}

// Two-stage test of one triangle record (a, e1, e2, n as float4 with unused w): stage 1 computes
// ao and num_t and leaves when no lane has num_t > 0 (necessary for dist > 0.001 since inv > 0);
// stage 2 completes the pre-test.
// Lanes with on == false take part in the arithmetic but never in a decision (callers use it for the
// per-lane mesh filter instead of an exec-mask branch around each triangle).
__device__ __forceinline__ void tri_two_stage(const float4& A, const float4& B, const float4& C, const float4& N,
                                              uint32_t i, uint32_t m, f3 o, f3 d, Closest& c, float& best_k,
                                              bool on = true) {
  const f3 n = mk(N.x, N.y, N.z);
  const f3 ao = o - mk(A.x, A.y, A.z);
  TriPre q;
  q.num_t = dot(ao, n);
  const bool front = on & (q.num_t > 0.0f);
  if (!__any(front)) return;
  const float dn = dot(d, n);
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  q.cand = (dn < 0.0f) & front & !pre_reject(q, best_k);
  if (__builtin_expect(__any(q.cand), 0)) {
    if (q.cand) tri_exact(q, i, m, c, best_k);
  }
}

// Triangle sources for the brute-force scan: the std430 buffer (wave-uniform -> SGPRs) or the LDS
// image (3 float4 per triangle = (a.xyz, n.x) (n.yz, e1.xy) (e1.z, e2.xyz)).
struct GlobalTris {
  const float4* __restrict__ t;
  __device__ __forceinline__ void operator()(uint32_t i, float4& A, float4& B, float4& C, float4& N) const {
    A = t[4 * i];
    B = t[4 * i + 1];
    C = t[4 * i + 2];
    N = t[4 * i + 3];
  }
};
struct LdsTris {
  const float4* t;
  __device__ __forceinline__ void operator()(uint32_t i, float4& A, float4& B, float4& C, float4& N) const {
    const float4 p = t[3 * i], q = t[3 * i + 1], r = t[3 * i + 2];
    A = make_float4(p.x, p.y, p.z, 0.0f);
    B = make_float4(q.z, q.w, r.x, 0.0f);
    C = make_float4(r.y, r.z, r.w, 0.0f);
    N = make_float4(p.w, q.x, q.y, 0.0f);
  }
};

// world_hit (raytracing.glsl:267-288) for one lane: spheres, then every triangle of every mesh whose
// (quirky) AABB test passes, two-stage exact test, one running closest hit (ties: first in order).
template <class Src>
__device__ __forceinline__ Closest world_hit_brute(const Scene& sc, const Src& src, const hrt_push_constants& pc, f3 o,
                                                   f3 d, uint32_t& tests) {
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  float best_k = c.t * kOnePlus;  // FLT_MAX*(1+2^-16) = inf: R7 never rejects
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = aabb_pass(mesh, o, d);
    tests += pass ? mesh.len : 0u;
    if (!pass) continue;
    const uint32_t end = mesh.first_index + mesh.len;
    for (uint32_t i = mesh.first_index; i < end; ++i) {
      float4 A, B, C, N;
      src(i, A, B, C, N);
      tri_two_stage(A, B, C, N, i, (uint32_t)m, o, d, c, best_k);
    }
  }
  return c;
}

// ---- BRUTE / BRUTE_LDS: fused sample/bounce loop ---------------------------------------------------
// Each lane runs its pixel's num_samples paths back to back (RNG state chains through them exactly
// as raytracing.glsl:379-385); the wave iterates until every lane's last path has ended.
template <class Src>
__device__ __forceinline__ void trace_fused(const TraceParams& P, const Src& src, uint32_t x, uint32_t lr) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes, P.tri_nhat};
  const hrt_push_constants& pc = P.pc;
  const uint32_t y = global_row(lr, P);
  uint32_t segs = 0, tests = 0;
  const bool active = x < pc.width && lr < P.local_rows && y < pc.height;
  if (active) {
    const uint32_t id = x + y * pc.width;
    f3 colour = mk(0.0f, 0.0f, 0.0f);
    uint32_t state = pc.rng_offset * 719393u + id;
    const float4 rc = sc.rays[id];
    const f3 centre = mk(rc.x, rc.y, rc.z);
    const f3 root = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
    int sample = 0;
    Path p;
    p.bounce = pc.max_bounces + 1;  // "no path in flight"
    while (true) {
      if (p.bounce > pc.max_bounces) {  // start the next sample (or finish)
        if (sample >= pc.num_samples) break;
        ++sample;
        const f3 dir = get_ray_dir(pc, centre, state);
        p = Path{mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), root, normalize(dir), 0, true};
      }
      const Closest c = world_hit_brute(sc, src, pc, p.pos, p.dir, tests);
      ++segs;
      const bool ended = shade_step(sc, pc, p, c, state);
      ++p.bounce;
      if (ended || p.bounce > pc.max_bounces) {
        colour = colour + p.light * p.colour;
        p.bounce = pc.max_bounces + 1;
      }
    }
    colour = div3(colour, (float)pc.num_samples);
    store_pixel(P, x, lr, colour);
  }
  flush_counters(P, segs, tests);
}

__global__ __launch_bounds__(256) void trace_brute(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused(P, GlobalTris{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

// Whole scene resident in LDS, 1024-thread workgroups (16 waves, a 32x32 pixel tile of 8x8 wave
// tiles): the copy is paid once per workgroup, every wave then streams the triangles from LDS with
// broadcast reads instead of scalar loads.
extern __shared__ float4 lds_tris[];
__global__ __launch_bounds__(1024) void trace_brute_lds(TraceParams P) {
  const uint32_t n = P.n_tris;
  for (uint32_t k = threadIdx.x; k < 3 * n; k += blockDim.x) {
    const uint32_t i = k / 3, part = k - 3 * i;
    const hrt_triangle& t = P.tris[i];
    float4 v;
    if (part == 0) v = make_float4(t.a[0], t.a[1], t.a[2], t.normal[0]);
    else if (part == 1) v = make_float4(t.normal[1], t.normal[2], t.edge_one[0], t.edge_one[1]);
    else v = make_float4(t.edge_one[2], t.edge_two[0], t.edge_two[1], t.edge_two[2]);
    lds_tris[k] = v;
  }
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t x = blockIdx.x * 32 + (wave & 3) * 8 + (lane & 7);
  const uint32_t lr = blockIdx.y * 32 + (wave >> 2) * 8 + (lane >> 3);
  trace_fused(P, LdsTris{lds_tris}, x, lr);
}

// ---- BUNDLE / BUNDLE_CULL ------------------------------------------------------------------------
//
// Per-frame prep (camera_lists): for every mesh, the triangles with num_t = dot(cam_pos - a, n) > 0
// -- computed exactly as a primary lane computes it -- compacted in buffer order into records
// (ao, num_t) (e1, index) (e2, -) (n, -), plus 5 float4 bundle-cull records (g, margin) per triangle.
// A triangle left out cannot be accepted by any primary lane (its dist would be <= 0 or NaN).
//
// Bundle cull: for a primary segment every lane's ray starts at cam_pos, so for a fixed triangle the
// reference's det = -d.n, num_u = d.(e2 x ao) and num_v = d.(e1 x ao) are LINEAR in the lane's
// direction d (ao = cam_pos - a is shared).  Bounding d over the wave's directions (axis a, cosine
// range [c_lo, c_hi], sine bound s_hi) bounds each linear form; a triangle is rejected for the whole
// wave when
//   R1  min d.n            > m_n   (every lane: dn >= 0, raytracing.glsl:217)
//   R3  max d.(e2 x ao)    < -m_u  (every lane: u < 0)
//   R4  min d.(e1 x ao)    > m_v   (every lane: v < 0)
//   R5  min d.(g_u-h+n)    > m_w   (every lane: num_u - num_v > det(1+2^-16), so u, v or w < 0)
// with margins m_* = 1e-5 * (product norms) + 2^-40|n| (+2^-14|n| for R5) covering the rounding of the
// reference's own dot/cross sequence (<= ~10 eps * product norm) and of these bounds.  The cull runs
// lane-parallel: lane j bounds triangle base+j, so 64 triangles cost one pass; survivors (in buffer
// order) get the exact per-lane test.
struct Bundle {
  f3 a;
  float c_lo, c_hi, s_hi;
};

// Wave-uniform cull diagnostics (HRT_OPT_COUNTERS = 2), flushed once per wave.
struct Diag {
  uint32_t prim_iters = 0, prim_considered = 0, prim_survivors = 0;
  uint32_t sec_iters = 0, sec_considered = 0, sec_survivors = 0, sec_lanes = 0;
  uint32_t bvh_visits = 0, bvh_prims = 0, bvh_band = 0;  // per lane (BUNDLE_BVH)
  uint64_t cyc_prim = 0, cyc_sec = 0, cyc_shade = 0;  // shader clocks per wave and phase
  uint32_t sec_stage2 = 0, sec_front = 0;
  uint32_t bvh_trips = 0, bvh_leaf_trips = 0;  // BUNDLE_BVH: wave-level traversal trips
  uint32_t band_max = 0, band_len = 0;          // BUNDLE_WQ: longest band list per batch / every lane's, summed
  uint32_t sky_items = 0;                       // work items run by sky_samples
  uint64_t cyc_sky = 0;                         // ... and their shader clocks
  uint32_t prim_lanes = 0, loop_iters = 0, live_lanes = 0;  // fused-loop lane use
  uint32_t wq_fill[4] = {0, 0, 0, 0};  // BUNDLE_WQ: node steps with 1-16 / 17-32 / 33-48 / 49-64 node pairs
  uint32_t wq_members = 0;             // ... the members of the groups this lane popped (valid slots), summed
};

__device__ __forceinline__ float wave_min_all(float v) {  // all 64 lanes active
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {  // all 64 lanes active
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_max_all(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Direction cone of the lanes with sel == true (axis = the first such lane's direction).
__device__ __forceinline__ Bundle make_bundle(bool sel, f3 d) {
  const int lead = __builtin_ctzll(__ballot(sel));
  Bundle b;
  b.a = mk(lane_read(d.x, (uint32_t)lead), lane_read(d.y, (uint32_t)lead), lane_read(d.z, (uint32_t)lead));
  const float lam = sel ? dot(d, b.a) : 3.0f;
  b.c_lo = wave_min_all(lam) - 1e-5f;
  b.c_hi = 1.00001f;
  b.s_hi = (b.c_lo > 0.0f) ? __builtin_sqrtf(fmaxf(0.0f, 1.00002f - b.c_lo * b.c_lo)) * 1.00001f + 1e-6f : 1.00001f;
  return b;
}

__device__ __forceinline__ float lin_lower(float ga, float gn, const Bundle& b) {
  return fminf(b.c_lo * ga, b.c_hi * ga) - b.s_hi * gn;
}
__device__ __forceinline__ float lin_upper(float ga, float gn, const Bundle& b) {
  return fmaxf(b.c_lo * ga, b.c_hi * ga) + b.s_hi * gn;
}

// Spheres for the selected lanes (raytracing.glsl:271-276).
__device__ __forceinline__ void spheres_first(const Scene& sc, const hrt_push_constants& pc, bool sel, f3 o, f3 d,
                                              Closest& c) {
  if (!sel) return;
  c = Closest{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
}

// Read-only scene data seen through the constant address space: a load with a wave-uniform address
// from it is a scalar (s_load) load.
typedef __attribute__((address_space(4))) const float kfloat;
__device__ __forceinline__ const kfloat* to_const(const float4* p) {
  return (const kfloat*)(const __attribute__((address_space(4))) void*)(p);
}
__device__ __forceinline__ float4 ldk(const kfloat* p, uint32_t i) {  // float4 i of p
  return make_float4(p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]);
}

// Exact per-lane test of compacted camera-facing record k (ao and num_t precomputed), entered only
// when some lane has dn < 0.
__device__ __forceinline__ void primary_exact_rec(const float4& A, const float4& B, const float4& C, float dn, f3 d,
                                                  uint32_t m, Closest& c, float& best_k) {
  TriPre q;
  q.num_t = A.w;
  const f3 dao = cross(mk(A.x, A.y, A.z), d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  q.cand = (dn < 0.0f) & !pre_reject(q, best_k);
  if (__builtin_expect(__any(q.cand), 0)) {
    if (q.cand) tri_exact(q, __builtin_bit_cast(uint32_t, B.w), m, c, best_k);
  }
}
__device__ __forceinline__ void primary_exact(const kfloat* ct, uint32_t k, float dn, f3 d, uint32_t m, Closest& c,
                                              float& best_k) {
  primary_exact_rec(ldk(ct, 4 * k), ldk(ct, 4 * k + 1), ldk(ct, 4 * k + 2), dn, d, m, c, best_k);
}
// All 64 bytes of camera record k in one scalar load (s_load_dwordx16)
typedef float kf16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const kf16 kf16c;
__device__ __forceinline__ kf16 ld_rec(const kfloat* ct, uint32_t k) { return *(kf16c*)(ct + 16 * (size_t)k); }

// ---- per-wave primary triangle list ------------------------------------------------------------
// Every primary direction a wave can produce is normalize(M * nc) with nc = centre + (0, t2.y, t1.z),
// |t1.z|, |t2.y| <= jitter_size (get_ray_dir, raytracing.glsl:162-166), i.e. nc in the box X =
// [centre box of the wave's pixels] + [0] x [-j, j] x [-j, j].  The cap around normalize(M * mid(X))
// through the farthest of X's 8 corner directions contains them all (a cap under 90 degrees is
// convex), widened by 1e-5 in cosine for rounding.  The bundle cull against that cap runs ONCE per
// wave; its survivors (camera-list index | mesh << 27, in buffer order) are the only triangles any
// primary segment of the wave can hit, so each primary iteration tests just those.  The list lives
// in one VGPR (entry i in lane i, read back with v_readlane; up to 64 entries) in the LDS-resident
// kernels, and in a per-wave LDS slice of kTileCapLds entries in the others (dense scenes put
// hundreds of triangles in a tile's cap).  A wave whose list overflows culls per iteration.
constexpr uint32_t kTileCapVgpr = 64;
constexpr uint32_t kTileCapLds = 1024;

struct TileList {
  uint32_t v;      // VGPR list: lane i holds entry i
  uint32_t* lds;   // LDS list (nullptr: VGPR list)
  uint32_t n;
  bool ok;
  // aabb_pass of every mesh (<= 8) for a ray from cam_pos by the sign octant of its direction:
  // bit 8m + (sx | sy << 1 | sz << 2) (aabb_truth_table); aabb_ok false -> the literal test
  unsigned long long aabb;
  bool aabb_ok;
  uint32_t tsum;  // lane l: the triangle tests of a primary ray in octant l & 7 (sum of passing meshes' len)
};

// intersecting_aabb's result for origin o depends only on the signs of (bound - o) and of 1/d per
// axis, as long as no product (bound - o) * (1/d) is zero or NaN: each "> 0" test is then a sign
// test, and the quirked min/max chain (raytracing.glsl:199-207) reduces to
//   tx_far > 0 || tx_near > 0 || ty_far > 0 || tz_far > 0 || tz_near > 0.
// So with every bound - o nonzero and not NaN, and |d| <= 1.5 per component (|1/d| >= 2/3, so a
// nonzero product cannot round to 0), aabb_pass(m, o, d) == aabb_pass(m, o, (+-1, +-1, +-1)) with
// d's sign bits (1/+-0 = +-inf keeps the sign).  Lane l evaluates mesh l >> 3 at octant l & 7.
__device__ __forceinline__ void aabb_truth_table(const TraceParams& P, TileList& t) {
  const hrt_push_constants& pc = P.pc;
  const uint32_t lane = threadIdx.x & 63, m = lane >> 3, oct = lane & 7;
  const f3 o = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
  bool pass = false, bad = false;
  uint32_t len = 0;
  if (m < (uint32_t)pc.num_meshes) {
    const hrt_mesh& mesh = kargs()->meshes[m];
    for (int a = 0; a < 3; ++a) {
      const float ov = a == 0 ? o.x : (a == 1 ? o.y : o.z);
      const float lo = mesh.min_point[a] - ov, hi = mesh.max_point[a] - ov;
      bad |= !(lo < 0.0f || lo > 0.0f) || !(hi < 0.0f || hi > 0.0f);  // zero or NaN
    }
    pass = aabb_pass(mesh, o, mk((oct & 1) ? -1.0f : 1.0f, (oct & 2) ? -1.0f : 1.0f, (oct & 4) ? -1.0f : 1.0f));
    len = pass ? mesh.len : 0u;
  }
  t.aabb = __ballot(pass);
  t.aabb_ok = pc.num_meshes <= 8 && !__any(bad);
  // per octant: the tests counter's increment (lanes oct, oct + 8, ... hold its meshes)
  len += (uint32_t)__shfl_xor((int)len, 8, 64);
  len += (uint32_t)__shfl_xor((int)len, 16, 64);
  len += (uint32_t)__shfl_xor((int)len, 32, 64);
  t.tsum = len;
}

__device__ __forceinline__ Bundle tile_bundle(const hrt_push_constants& pc, bool active, f3 centre, bool& ok) {
  const float inf = __builtin_inff();
  const f3 lo = mk(wave_min_all(active ? centre.x : inf), wave_min_all(active ? centre.y : inf),
                   wave_min_all(active ? centre.z : inf));
  const f3 hi = mk(wave_max_all(active ? centre.x : -inf), wave_max_all(active ? centre.y : -inf),
                   wave_max_all(active ? centre.z : -inf));
  const float j = fabsf(pc.jitter_size) * 1.0001f;
  const float* M = pc.cam_alignment_mat;
  auto dir = [&](f3 v) {
    return normalize(mk(M[0] * v.x + M[4] * v.y + M[8] * v.z, M[1] * v.x + M[5] * v.y + M[9] * v.z,
                        M[2] * v.x + M[6] * v.y + M[10] * v.z));
  };
  Bundle b;
  b.a = dir(mk(0.5f * lo.x + 0.5f * hi.x, 0.5f * lo.y + 0.5f * hi.y, 0.5f * lo.z + 0.5f * hi.z));
  const uint32_t lane = threadIdx.x & 63;
  const f3 corner = mk((lane & 1) ? hi.x : lo.x, (lane & 2) ? hi.y + j : lo.y - j, (lane & 4) ? hi.z + j : lo.z - j);
  const float lam = lane < 8 ? dot(dir(corner), b.a) : 3.0f;
  b.c_lo = wave_min_all(lam) - 1e-5f;
  b.c_hi = 1.00001f;
  b.s_hi = __builtin_sqrtf(fmaxf(0.0f, 1.00002f - b.c_lo * b.c_lo)) * 1.00001f + 1e-6f;
  // a sane cap (NaN -> false; fminf skips a NaN corner, so a corner that overflowed is checked here)
  ok = b.c_lo > 0.5f && !__any(!(lam == lam));
  return b;
}

// Bundle rules R3-R5 of camera-list records [base, base + 64) against b (lane j: record base + j).
__device__ __forceinline__ bool bundle_keep(const float4* __restrict__ cr, uint32_t k, const Bundle& b) {
  const float4 C0 = cr[5 * k], C1 = cr[5 * k + 1], C2 = cr[5 * k + 2], C3 = cr[5 * k + 3], C4 = cr[5 * k + 4];
  const float na = dot(mk(C0.x, C0.y, C0.z), b.a), ua = dot(mk(C1.x, C1.y, C1.z), b.a);
  const float va = dot(mk(C2.x, C2.y, C2.z), b.a), wa = dot(mk(C3.x, C3.y, C3.z), b.a);
  const bool rej = (lin_lower(na, C4.x, b) > C0.w) | (lin_upper(ua, C4.y, b) < -C1.w) |
                   (lin_lower(va, C4.z, b) > C2.w) | (lin_lower(wa, C4.w, b) > C3.w);
  return !rej;
}

// Builds the wave's list (all 64 lanes active; the caller synchronises before reading it).
__device__ __forceinline__ TileList build_tile_list(const TraceParams& P, bool active, f3 centre, uint32_t* lds) {
  const hrt_push_constants& pc = P.pc;
  TileList t{0u, lds, 0u, false, 0ull, false, 0u};
  const uint32_t cap = lds ? kTileCapLds : kTileCapVgpr;
  if (pc.num_meshes > 32 || !__any(active)) return t;
  bool ok;
  const Bundle b = tile_bundle(pc, active, centre, ok);
  if (!ok) return t;
  aabb_truth_table(P, t);
  const uint32_t lane = threadIdx.x & 63;
  const KArgs K = kargs();  // (once per work item)
  const uint32_t* cam_start = K->cam_start;
  const uint32_t* cam_count = K->cam_count;
  const float4* cam_cull = K->cam_cull;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const uint32_t k0 = cam_start[m], k1 = k0 + cam_count[m];
    for (uint32_t base = k0; base < k1; base += 64) {
      const uint32_t k = base + lane;
      const bool keep = k < k1 && bundle_keep(cam_cull, k, b);
      unsigned long long mask = __ballot(keep);
      const uint32_t cnt = (uint32_t)__popcll(mask);
      if (t.n + cnt > cap) return t;  // ok stays false: per-iteration cull
      if (lds) {  // lane-parallel append in buffer order
        if (keep) lds_put(&lds[t.n + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))], k | ((uint32_t)m << 27));
        t.n += cnt;
      } else {
        while (mask) {  // few survivors: append each to the next lane
          const uint32_t e = (base + (uint32_t)__builtin_ctzll(mask)) | ((uint32_t)m << 27);
          mask &= mask - 1ull;
          t.v = lane == t.n ? e : t.v;
          ++t.n;
        }
      }
    }
  }
  t.ok = true;
  wave_handoff();  // the list's entries (other lanes' stores) before the reads of world_hit_tile
  return t;
}

// Primary segments from the wave's list (ALL 64 lanes active).  Per lane: spheres, the meshes' AABB
// quirk (raytracing.glsl:279) and its test count, then the listed triangles in buffer order.
// Returns the entries it tested (the others: no primary lane's mesh vote; diagnostics).
__device__ __forceinline__ uint32_t world_hit_tile(const Scene& sc, const TraceParams& P, const TileList& tl, bool prim,
                                                   f3 o, f3 d, uint32_t& tests, Closest& c) {
  const hrt_push_constants& pc = P.pc;
  spheres_first(sc, pc, prim, o, d, c);
  // primary lanes start at cam_pos (the table's origin): bit 8m of pm is mesh m's AABB test, by the
  // direction's octant (one 64-bit shift of the wave's table and one lane read of its test count) or,
  // off the table's domain, by the literal test
  const bool octant = tl.aabb_ok && fabsf(d.x) <= 1.5f && fabsf(d.y) <= 1.5f && fabsf(d.z) <= 1.5f;
  const uint32_t oct = (fbits(d.x) >> 31) | ((fbits(d.y) >> 31) << 1) | ((fbits(d.z) >> 31) << 2);
  unsigned long long pm = tl.aabb >> oct;
  const uint32_t oct_tests = lane_read(tl.tsum, oct);
  if (prim && octant) {
    tests += oct_tests;
  } else if (prim) {
    pm = 0ull;
    for (int m = 0; m < pc.num_meshes; ++m) {
      if (aabb_pass(sc.meshes[m], o, d)) {
        pm |= 1ull << (8 * m);
        tests += sc.meshes[m].len;
      }
    }
  }
  float best_k = c.t * kOnePlus;
  const kfloat* ct = to_const(HRT_SHADE_KARGS ? kargs()->cam_tris : P.cam_tris);
  auto entry = [&](uint32_t i) {
    return tl.lds ? __builtin_amdgcn_readfirstlane(lds_get(&tl.lds[i])) : (uint32_t)__builtin_amdgcn_readlane((int)tl.v, (int)i);
  };
  // (r03: requesting the next entry's record before this one's test was slower, island 2.259 -> 2.338)
#ifndef HRT_LIST_UNIFORM
#define HRT_LIST_UNIFORM 1
#endif
  // (the list length through readfirstlane: hipcc had lost its uniformity through build_tile_list's
  // early returns and ran the entry loop as a divergent loop with a VGPR trip count)
  const uint32_t n = HRT_LIST_UNIFORM ? __builtin_amdgcn_readfirstlane(tl.n) : tl.n;
  uint32_t tested = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t e = entry(i);
    const uint32_t kk = e & 0x07FFFFFFu, m = e >> 27;
    const bool pass = prim && ((pm >> (8 * m)) & 1ull);
    if (!__any(pass)) continue;
    ++tested;
    {
    // the whole record in one load: the exact test's operands arrive with the normal (one K$ round
    // trip per entry instead of two dependent ones)
    const kf16 R = ld_rec(ct, kk);
    const float dn = pass ? dot(d, mk(R[12], R[13], R[14])) : 0.0f;
    if (__any(dn < 0.0f))
      primary_exact_rec(make_float4(R[0], R[1], R[2], R[3]), make_float4(R[4], R[5], R[6], R[7]),
                        make_float4(R[8], R[9], R[10], R[11]), dn, d, m, c, best_k);
    }
  }
  return tested;
}

// Primary segments of the lanes with prim == true.  Called with ALL 64 lanes of the wave active.
template <bool D>
__device__ __forceinline__ void world_hit_bundle(const Scene& sc, const TraceParams& P, bool prim, f3 o, f3 d,
                                                 uint32_t& tests, Closest& c, Diag& dg) {
  const hrt_push_constants& pc = P.pc;
  const Bundle b = make_bundle(prim, d);
  spheres_first(sc, pc, prim, o, d, c);
  float best_k = c.t * kOnePlus;
  const kfloat* ct = to_const(P.cam_tris);
  const float4* __restrict__ cr = P.cam_cull;
  const uint32_t lane = threadIdx.x & 63;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = prim && aabb_pass(mesh, o, d);
    if (prim) tests += pass ? mesh.len : 0u;
    if (!__any(pass)) continue;
    const uint32_t k0 = P.cam_start[m], k1 = k0 + P.cam_count[m];
    for (uint32_t base = k0; base < k1; base += 64) {
      const uint32_t k = base + lane;
      bool keep = false;
      if (k < k1) {
        const float4 C0 = cr[5 * k], C1 = cr[5 * k + 1], C2 = cr[5 * k + 2], C3 = cr[5 * k + 3], C4 = cr[5 * k + 4];
        const float na = dot(mk(C0.x, C0.y, C0.z), b.a), ua = dot(mk(C1.x, C1.y, C1.z), b.a);
        const float va = dot(mk(C2.x, C2.y, C2.z), b.a), wa = dot(mk(C3.x, C3.y, C3.z), b.a);
        const bool rej = (lin_lower(na, C4.x, b) > C0.w) | (lin_upper(ua, C4.y, b) < -C1.w) |
                         (lin_lower(va, C4.z, b) > C2.w) | (lin_lower(wa, C4.w, b) > C3.w);
        keep = !rej;
      }
      unsigned long long mask = __ballot(keep);
      if (D && P.diag) {
        dg.prim_considered += min(64u, k1 - base);
        dg.prim_survivors += (uint32_t)__popcll(mask);
      }
      while (mask) {
        const uint32_t kk = __builtin_amdgcn_readfirstlane(base + (uint32_t)__builtin_ctzll(mask));
        mask &= mask - 1ull;
        if (pass) {
          const float4 N = ldk(ct, 4 * kk + 3);
          const float dn = dot(d, mk(N.x, N.y, N.z));
          if (__any(dn < 0.0f)) primary_exact(ct, kk, dn, d, (uint32_t)m, c, best_k);
        }
      }
    }
  }
}

// Triangle sources of the bounce cull: lane(k) -> (a, n) of triangle k for the lane-parallel cull,
// uniform(k) -> (a, e1, e2, n) of a wave-uniform survivor.
struct CullGlobal {  // std430 buffer; survivors through the constant address space (s_load)
  const float4* __restrict__ T;
  const kfloat* Tk;
  __device__ __forceinline__ void lane(uint32_t k, float4& A, float4& N) const {
    A = T[4 * k];
    N = T[4 * k + 3];
  }
  __device__ __forceinline__ void uniform(uint32_t k, float4& A, float4& B, float4& C, float4& N) const {
    A = ldk(Tk, 4 * k);
    B = ldk(Tk, 4 * k + 1);
    C = ldk(Tk, 4 * k + 2);
    N = ldk(Tk, 4 * k + 3);
  }
};
struct CullLds {  // LDS image, 3 float4 per triangle: (a, n.x) (n.yz, e1.xy) (e1.z, e2)
  const float4* t;
  __device__ __forceinline__ void lane(uint32_t k, float4& A, float4& N) const {
    const float4 p = t[3 * k], q = t[3 * k + 1];
    A = make_float4(p.x, p.y, p.z, 0.0f);
    N = make_float4(p.w, q.x, q.y, 0.0f);
  }
  __device__ __forceinline__ void uniform(uint32_t k, float4& A, float4& B, float4& C, float4& N) const {
    LdsTris{t}(k, A, B, C, N);
  }
};

// ---- cooperative tiles ------------------------------------------------------------------------------
// A heavy tile's frame time is its sequential chain of bounce batches, each a dependent survivor loop
// (profiles/r01k_*).  In a cooperative tile every wave of the workgroup runs the same 64 pixels with
// identical state; the bounce cull's 64-triangle chunks (numbered across meshes in scan order) are
// dealt out over the W waves, chunk j to wave j mod W, and the per-lane closest hits are merged with
// one 64-bit LDS min per lane over
// key = bits(t) << 32 | id, id = 0 for "no triangle" (the sphere / miss result every wave shares)
// and 1 + (mesh << 26 | index) for a triangle.  For t >= 0 the float bits order like t, and the
// reference's scan (spheres, then meshes in order, triangles in index order, strict <) keeps the
// first of equal distances, which is the lowest id: the merge gives exactly the serial result.
// Slots are triple-buffered so that one barrier per batch suffices: wave 0 clears slot r+1 before
// the barrier of batch r, when every wave has finished reading it (batch r-2).
struct Coop {
  uint32_t w, W;                 // this wave, waves in the group (1: not cooperative)
  unsigned long long* ex;        // 3 x 64 slots (LDS)
  uint32_t round;
  uint32_t work;                 // this wave's share of the tile's work units (the planner's cost)
  // persistent loops: the wave sums its items' counters here and flushes them once at the end
  // (three same-address global atomics per item serialised in L2: ~40 ns per item, the floor of
  // low-spp frames -- 4K 4 spp took 5.1 ms per frame)
  bool defer = false;
  unsigned long long acc_s = 0, acc_t = 0, acc_m = 0;
  bool hot = false;              // the item's wave runs at issue priority 3 (tile_loop)
  uint32_t cache_tile = 0xFFFFFFFFu;  // a whole tile's item: its tile (the launch's tile_lists record), else ~0
#if HRT_TIMELINE
  unsigned long long t_setup = 0;  // s_memrealtime when the item's tile list was built (timeline builds)
  unsigned long long t_sky = 0;    // ... 1 if the item ran as a sky item
#endif
};

__device__ __forceinline__ void coop_merge(Coop& co, Closest& c) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long* slot = co.ex + 64 * (co.round % 3);
  if (co.w == 0) co.ex[64 * ((co.round + 1) % 3) + lane] = ~0ull;
  const uint32_t id = c.kind == 2 ? ((c.mesh << 26) | c.idx) + 1u : 0u;
  const unsigned long long key = ((unsigned long long)__float_as_uint(c.t) << 32) | id;
  atomicMin(&slot[lane], key);
  __syncthreads();
  const unsigned long long best = slot[lane];
  ++co.round;
  const uint32_t bid = (uint32_t)best;
  if (bid != 0) c = Closest{__uint_as_float((uint32_t)(best >> 32)), 2, (bid - 1u) & 0x03FFFFFFu, (bid - 1u) >> 26};
}

// Bounce segments with a lane-parallel pre-cull (BUNDLE_CULL).  For the bounce lanes (origins o_l,
// directions d_l) and triangle (a, n):
//   S1  num_t = (o - a).n is linear in o: if max over the lanes' origin box B of (o - a).n
//       < -1e-5 |o - a|max |n|_1, every lane computes num_t <= 0 -> dist <= 0 (or NaN): rejected;
//   R1  dn = d.n is linear in d: if min over the lanes' direction cone of d.n > 1e-5 |n|_1, every
//       lane has dn >= 0: rejected.
// Lane j bounds triangle base+j; survivors (buffer order) get the exact per-lane two-stage test.
// Called with ALL 64 lanes active.
template <bool D, class Src>
__device__ __forceinline__ void world_hit_bounce_cull(const Scene& sc, const TraceParams& P, const Src& src, bool sec,
                                                      f3 o, f3 d, uint32_t& tests, Closest& c, Diag& dg, Coop& co) {
  const hrt_push_constants& pc = P.pc;
  const float inf = __builtin_inff();
  const f3 lo = mk(wave_min_all(sec ? o.x : inf), wave_min_all(sec ? o.y : inf), wave_min_all(sec ? o.z : inf));
  const f3 hi = mk(wave_max_all(sec ? o.x : -inf), wave_max_all(sec ? o.y : -inf), wave_max_all(sec ? o.z : -inf));
  const Bundle b = make_bundle(sec, d);
  const bool box_ok = (hi.x - lo.x) <= 3.0e38f && (hi.y - lo.y) <= 3.0e38f && (hi.z - lo.z) <= 3.0e38f;
  const f3 ctr = mk(0.5f * lo.x + 0.5f * hi.x, 0.5f * lo.y + 0.5f * hi.y, 0.5f * lo.z + 0.5f * hi.z);
  // half widths, enlarged so that |o - ctr| <= hw per axis for every bounce lane despite rounding
  const f3 hw = mk((hi.x - ctr.x) * 1.0001f, (hi.y - ctr.y) * 1.0001f, (hi.z - ctr.z) * 1.0001f);
  spheres_first(sc, pc, sec, o, d, c);
  float best_k = c.t * kOnePlus;
  const uint32_t lane = threadIdx.x & 63;
  // cooperative tiles: 64-triangle chunk j of the scan (numbered across meshes) goes to wave j mod W
  const uint32_t cw = __builtin_amdgcn_readfirstlane(co.w);
  uint32_t chunk0 = 0;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = sec && aabb_pass(mesh, o, d);
    if (sec) tests += pass ? mesh.len : 0u;
    const uint32_t k0 = mesh.first_index, k1 = k0 + mesh.len;
    const uint32_t skip = (cw + co.W - chunk0 % co.W) % co.W;  // this wave's first chunk of the mesh
    chunk0 += (mesh.len + 63) / 64;
    if (!__any(pass)) continue;
    for (uint32_t base_v = k0 + 64 * skip; base_v < k1; base_v += 64 * co.W) {
      const uint32_t base = __builtin_amdgcn_readfirstlane(base_v);  // uniform: scalar survivor indices
      const uint32_t k = base + lane;
      bool keep = false;
      if (k < k1) {
        float4 A, N;
        src.lane(k, A, N);
        const f3 n = mk(N.x, N.y, N.z);
        const f3 ca = ctr - mk(A.x, A.y, A.z);
        const float an = fabsf(n.x), bn = fabsf(n.y), cn = fabsf(n.z);
        const float nn = an + bn + cn;                                                      // >= |n|
        const float spread = an * hw.x + bn * hw.y + cn * hw.z;                             // max (o - ctr).n
        const float reach = fabsf(ca.x) + fabsf(ca.y) + fabsf(ca.z) + hw.x + hw.y + hw.z;  // >= |o - a|
        const bool s1 = box_ok && (dot(ca, n) + spread + 1e-5f * reach * nn < 0.0f);
        const bool r1 = lin_lower(dot(n, b.a), nn, b) > 1e-5f * nn;
        keep = !(s1 | r1);
      }
      unsigned long long mask = __ballot(keep);
      co.work += 1u + (uint32_t)__popcll(mask);  // one unit per chunk culled and per survivor tested
      if (D && P.diag) {
        dg.sec_considered += min(64u, k1 - base);
        dg.sec_survivors += (uint32_t)__popcll(mask);
      }
      while (mask) {
        // wave-uniform by construction (global source: constant address space -> s_load)
        const uint32_t k1 = __builtin_amdgcn_readfirstlane(base + (uint32_t)__builtin_ctzll(mask));
        mask &= mask - 1ull;
        float4 A, B, C, N;
        src.uniform(k1, A, B, C, N);
        if (D && P.diag && pass) {  // how far the two-stage test gets for this survivor
          const f3 ao = o - mk(A.x, A.y, A.z);
          const bool s2 = dot(ao, mk(N.x, N.y, N.z)) > 0.0f;
          dg.sec_stage2 += __any(s2) ? 1u : 0u;
          dg.sec_front += __any(s2 && dot(d, mk(N.x, N.y, N.z)) < 0.0f) ? 1u : 0u;
        }
        tri_two_stage(A, B, C, N, k1, (uint32_t)m, o, d, c, best_k, pass);
      }
    }
  }
  if (co.W > 1) coop_merge(co, c);
}

// ---- BUNDLE_BVH: per-lane hierarchy traversal for bounce segments ----------------------------------
// Each bounce lane walks the BVH (hrt_bvh.h) in preorder with escape indices (one register of
// state).  For a triangle (a, e1, e2, n) and the lane's ray (o, d), |d| = 1 (DESIGN.md "BVH cull"):
//   back     d.n^ >= 2e-5: the reference's dn = d.n rounds to > 0 and raytracing.glsl:219 rejects;
//   band     -tau_g - 1e-5 < d.n^ < 2e-5 (tau_g = P.bvh_band_tau, the scene's): grazing; the reference's arithmetic is rounding noise
//            there and may accept anywhere in the triangle's plane, so these triangles are listed per
//            cube-map direction cell (hrt_bvh.cpp build_band_lists) and every lane tests its cell's
//            list exactly;
//   front    d.n^ <= -tau with tau >= kBandTau: an accepted triangle's reference (u, v, w) >= 0 puts
//            the exact intersection of the ray's line with the triangle's plane inside the triangle
//            inflated by eta (barycentrics >= -eta), at a line parameter within rel*t + abs of the
//            accepted dist, where
//              eta = 6e + (1.01 rho + 3.2e + 18.4e G R) / (tau - rho - 4e-7)
//              abs = 2.1 (4.2e + rho) R / (tau - rho - 4e-7),  rel = 2.1 (3.2e + rho) / (...) + 4e
//            (e = 2^-24, R >= |o - a| over the node, G and rho from the node record).
// So a node is skipped when its normal cone is entirely back-facing, or when the ray segment
// t in [-abs, best (1 + rel) + abs] misses the node box grown by 2 eta tri_ext (plus coordinate
// rounding) at tau = kBandTau and R = the lane origin's distance to the farthest scene-box corner
// (node margin a + b R and abs = abs_coef R precomputed by hrt_bvh.cpp): no triangle below can then
// be accepted with dist <= best except band triangles, which the band list covers.  Equal distances are
// resolved by the scan key (first in the reference's mesh/index order wins).

// The exact per-lane test of one BVH entry (triangle idx of mesh m, scan key), raytracing.glsl:213-241
// with the running closest (ties: lower key).
__device__ __forceinline__ void bvh_tri_test(const float4& A, const float4& B, const float4& C, const float4& N,
                                             uint32_t key, uint32_t idx, uint32_t m, f3 o, f3 d, Closest& c,
                                             uint32_t& bkey, float& best_k) {
  const f3 n = mk(N.x, N.y, N.z);
  const f3 ao = o - mk(A.x, A.y, A.z);
  TriPre q;
  q.num_t = dot(ao, n);
  if (!(q.num_t > 0.0f)) return;
  const float dn = dot(d, n);
  if (!(dn < 0.0f)) return;
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  if (pre_reject(q, best_k)) return;
  const float inv_det = 1.0f / q.det;
  const float dist = q.num_t * inv_det;
  const float u = q.num_u * inv_det;
  const float v = -q.num_v * inv_det;
  const float w = 1.0f - u - v;
  if (!(dist < 0.0f) && !(u < 0.0f) && !(v < 0.0f) && !(w < 0.0f) && dist > 0.001f &&
      (dist < c.t || (dist == c.t && key < bkey))) {
    c = Closest{dist, 2, idx, m};
    bkey = key;
    best_k = dist * kOnePlus;
  }
}

// BVH entry k from 64 B records (a, key) (e1, mesh) (e2, index) (n, -) (leaf prims, irregular list).
__device__ __forceinline__ void bvh_prim_test(const float4* __restrict__ pr, uint32_t k, unsigned long long mask, f3 o,
                                              f3 d, Closest& c, uint32_t& bkey, float& best_k) {
  const float4 A = pr[4 * k], B = pr[4 * k + 1];
  // all four record loads before the mesh filter (one memory round trip per test, not two: the
  // compiler would otherwise sink C and N below the branch)
  const float4 C = pr[4 * k + 2], N = pr[4 * k + 3];
  asm volatile("; record %0 %1" ::"v"(C.x), "v"(N.x));
  const uint32_t m = __builtin_bit_cast(uint32_t, B.w);
  if (!((mask >> m) & 1ull)) return;  // mesh failed its (quirky) AABB test for this lane
  bvh_tri_test(A, B, C, N, __builtin_bit_cast(uint32_t, A.w), __builtin_bit_cast(uint32_t, C.w), m, o, d, c, bkey,
               best_k);
}

// Hierarchy sources: node k (4 float4) and leaf / band entry k.
struct BvhGlobal {
  const float4* __restrict__ nodes;
  const float4* __restrict__ prims;
  __device__ __forceinline__ void node(uint32_t k, float4& N0, float4& N1, float4& N2, float4& N3) const {
    N0 = nodes[4 * k];
    N1 = nodes[4 * k + 1];
    N2 = nodes[4 * k + 2];
    N3 = nodes[4 * k + 3];
  }
  __device__ __forceinline__ void prim(uint32_t k, unsigned long long mask, f3 o, f3 d, Closest& c, uint32_t& bkey,
                                       float& best_k) const {
    bvh_prim_test(prims, k, mask, o, d, c, bkey, best_k);
  }
};
struct BvhLds {  // nodes and the triangle image in LDS; entry k = triangle | mesh << 26, key = kbase[m] + triangle
  const float4* nodes;
  const float4* tris;
  const uint32_t* entries;
  const uint32_t* kbase;
  __device__ __forceinline__ void node(uint32_t k, float4& N0, float4& N1, float4& N2, float4& N3) const {
    N0 = nodes[4 * k];
    N1 = nodes[4 * k + 1];
    N2 = nodes[4 * k + 2];
    N3 = nodes[4 * k + 3];
  }
  __device__ __forceinline__ void prim(uint32_t k, unsigned long long mask, f3 o, f3 d, Closest& c, uint32_t& bkey,
                                       float& best_k) const {
    const uint32_t e = entries[k], idx = e & 0x03FFFFFFu, m = e >> 26;
    if (!((mask >> m) & 1ull)) return;
    float4 A, B, C, N;
    LdsTris{tris}(idx, A, B, C, N);
    bvh_tri_test(A, B, C, N, kbase[m] + idx, idx, m, o, d, c, bkey, best_k);
  }
};

// true when the node may hold a triangle the reference accepts for (o, d) with dist <= best.
// R >= |o - a| for every vertex of the scene (the lane's origin to the root box's farthest corner),
// abs = abs_coef R: the per-lane part of the node test, computed once per bounce segment.
__device__ __forceinline__ bool bvh_node_visit(const float4& N0, const float4& N1, const float4& N2, const float4& N3,
                                               f3 o, f3 d, f3 inv, float R, float abs_t, float t_hi) {
  const float x = N2.x * d.x + N2.y * d.y + N2.z * d.z;  // cos(angle(d, axis)) within 2e-6
  const float xa = fmaxf(fabsf(x) - 2e-6f, 0.0f);
  const float s_up = __builtin_sqrtf(fmaxf(1.0f - xa * xa, 0.0f)) + 1e-6f;
  if (x * N2.w - s_up * N3.x - 1e-6f > 1e-5f) return false;  // back: every dn > 0
  const float mg = N0.w + N1.w * R;
  const float tx0 = ((N0.x - mg) - o.x) * inv.x, tx1 = ((N1.x + mg) - o.x) * inv.x;
  const float ty0 = ((N0.y - mg) - o.y) * inv.y, ty1 = ((N1.y + mg) - o.y) * inv.y;
  const float tz0 = ((N0.z - mg) - o.z) * inv.z, tz1 = ((N1.z + mg) - o.z) * inv.z;
  const float tn = fmaxf(fmaxf(-abs_t, fminf(tx0, tx1)), fmaxf(fminf(ty0, ty1), fminf(tz0, tz1)));
  const float tf = fminf(fminf(t_hi, fmaxf(tx0, tx1)), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
  return !((tn - fabsf(tn) * 1e-6f) > (tf + fabsf(tf) * 1e-6f));  // NaN -> visit
}
// Cube-map cell of a direction (hrt_bvh.cpp face_dir is the inverse): face = 2 * major axis +
// (component < 0), (u, v) = the two minor components over the major one's magnitude.
__device__ __forceinline__ uint32_t dir_cell(f3 d, uint32_t res) {
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  // operands selected per lane, then one pair of divides (the same quotients as dividing inside
  // each face's branch, without a wave running up to three divergent pairs)
  const bool fx = ax >= ay && ax >= az, fy = !fx && ay >= az;
  const uint32_t face = fx ? (d.x < 0.0f ? 1u : 0u) : fy ? (d.y < 0.0f ? 3u : 2u) : (d.z < 0.0f ? 5u : 4u);
  const float den = fx ? ax : fy ? ay : az;
  const float u = (fx ? d.y : fy ? d.z : d.x) / den;
  const float v = (fx ? d.z : fy ? d.x : d.y) / den;
  const float s = 0.5f * (float)res;
  const int iu = min((int)res - 1, max(0, (int)((u + 1.0f) * s)));  // NaN converts to 0
  const int iv = min((int)res - 1, max(0, (int)((v + 1.0f) * s)));
  return (face * res + (uint32_t)iu) * res + (uint32_t)iv;
}

// Grazing-band pre-check: d.n^ of an entry's prim (its unit normal from TraceParams::bvh_band_nhat)
// inside the window (hrt_bvh.h "Grazing-band entries").
struct BandCheck {
  f3 d;
  float lo, hi;
  __device__ __forceinline__ explicit BandCheck(f3 d0, float lo0, float hi0) : d(d0), lo(lo0), hi(hi0) {}
  __device__ __forceinline__ bool in(const float4& nh) const {
    const float dn = __builtin_fmaf(d.z, nh.z, __builtin_fmaf(d.y, nh.y, d.x * nh.x));
    return dn > lo && dn < hi;
  }
};
// Entry k of the band lists: its prim index (16-bit words unless the scene has more than 65536 prims;
// the 16-bit array is padded to whole dwords).  One dword load either way, no branch on the width (a
// branch between a round's loads makes the normal's wait drain the next round's entry load too).
__device__ __forceinline__ uint32_t band_entry(const void* band, uint32_t wide, uint32_t k) {
  const uint32_t w = static_cast<const uint32_t*>(band)[wide ? k : k >> 1];
  return wide ? w : (w >> ((k & 1u) << 4)) & 0xFFFFu;
}

// Bounce segments through the hierarchy.  Called with ALL 64 lanes active (spheres and the
// irregular list are wave-uniform loops; the traversal and the band list are per lane).
template <bool D, class Bvh>
__device__ __forceinline__ void world_hit_bounce_bvh(const Scene& sc, const TraceParams& P, const Bvh& bvh, bool sec,
                                                     f3 o, f3 d, uint32_t& tests, Closest& c, Diag& dg) {
  const hrt_push_constants& pc = P.pc;
  spheres_first(sc, pc, sec, o, d, c);
  unsigned long long mask = 0ull;
  if (sec) {
    for (int m = 0; m < pc.num_meshes; ++m) {
      const hrt_mesh& mesh = sc.meshes[m];
      if (aabb_pass(mesh, o, d)) {
        mask |= 1ull << m;
        tests += mesh.len;
      }
    }
  }
  uint32_t bkey = 0;  // spheres (and "no hit") win every tie
  float best_k = c.t * kOnePlus;
  for (uint32_t k = 0; k < P.bvh_n_irregular; ++k)
    if (sec) bvh_prim_test(P.bvh_irregular, k, mask, o, d, c, bkey, best_k);
  const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float R = 0.0f;
  if (P.bvh_n_nodes) {  // farthest root-box corner from the origin, rounded up
    float4 R0, R1, R2, R3;
    bvh.node(0, R0, R1, R2, R3);
    const float fx = fmaxf(fabsf(o.x - R0.x), fabsf(R1.x - o.x)), fy = fmaxf(fabsf(o.y - R0.y), fabsf(R1.y - o.y));
    const float fz = fmaxf(fabsf(o.z - R0.z), fabsf(R1.z - o.z));
    R = __builtin_amdgcn_sqrtf(fx * fx + fy * fy + fz * fz) * 1.0001f;  // 1 ulp, inside the x1.0001
  }
  const float abs_t = P.bvh_abs_coef * R;
  const uint32_t end = P.bvh_n_nodes;
  uint32_t node = (sec && mask) ? 0u : end;
  uint32_t visits = 0, prim_tests = 0, band_tests = 0;
  if (sec && mask) {
    const uint32_t cell = dir_cell(d, P.bvh_dir_res);
    const uint32_t b0 = P.bvh_band_off[cell], b1 = P.bvh_band_off[cell + 1];
    if (D && P.diag) dg.band_len += b1 - b0;  // (the same sum as BUNDLE_WQ's, which reads the cell records)
    // Pre-check: an entry whose d.n^ is outside (-tau_g - 2e-5, 3e-5) is not in this lane's band
    // (-tau_g - 1e-5, 2e-5).
    const BandCheck bc(d, -P.bvh_band_tau - 2e-5f, 3e-5f);
    uint32_t k = b0;
    for (; k + 4 <= b1; k += 4) {
      uint32_t qs[4];
      float4 nh[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) qs[j] = band_entry(P.bvh_band, P.bvh_band_wide, k + j);
#pragma unroll
      for (int j = 0; j < 4; ++j) nh[j] = P.bvh_band_nhat[qs[j]];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (bc.in(nh[j])) {
          bvh.prim(qs[j], mask, o, d, c, bkey, best_k);
          ++band_tests;
        }
      }
    }
    for (; k < b1; ++k) {
      const uint32_t q = band_entry(P.bvh_band, P.bvh_band_wide, k);
      if (bc.in(P.bvh_band_nhat[q])) {
        bvh.prim(q, mask, o, d, c, bkey, best_k);
        ++band_tests;
      }
    }
  }
  uint32_t trips = 0, leaf_trips = 0;  // wave-level loop iterations (diagnostics)
  while (node < end) {
    if (D && P.diag) ++trips;
    float4 N0, N1, N2, N3;
    bvh.node(node, N0, N1, N2, N3);
    const uint32_t info = __builtin_bit_cast(uint32_t, N3.z);
    const uint32_t esc = __builtin_bit_cast(uint32_t, N3.w);
    const float t_hi = c.t * (1.0f + P.bvh_rel_t) + abs_t;
    const bool visit = bvh_node_visit(N0, N1, N2, N3, o, d, inv, R, abs_t, t_hi);
    const uint32_t count = info >> 27;
    ++visits;
    if (D && P.diag && __any(visit && count)) ++leaf_trips;
    if (visit && count) {
      const uint32_t first = info & 0x07FFFFFFu;
      for (uint32_t k = first; k < first + count; ++k) bvh.prim(k, mask, o, d, c, bkey, best_k);
      prim_tests += count;
    }
    node = (visit && !count) ? node + 1 : esc;
  }
  if (D && P.diag) {
    dg.bvh_visits += visits;
    dg.bvh_prims += prim_tests;
    dg.bvh_band += band_tests;
    // trips run by the whole wave: the maximum over its lanes (the loop is divergent)
    dg.bvh_trips += wave_max_u(trips);
    dg.bvh_leaf_trips += wave_max_u(leaf_trips);
  }
}

// ---- BUNDLE_WQ: pair-queue hierarchy traversal for bounce segments --------------------------------
// The per-lane traversal above (BUNDLE_BVH) keeps one node cursor per lane: a wave runs as many
// trips as its longest lane (123 per batch vs 55 visits per lane on island) and a leaf's triangles
// serially, and a heavy 8x8 tile spends ~600K clocks per bounce batch either way (profiles/
// r01k_tile_profiles.jsonl, BUNDLE_CULL_LDS: ~850 survivor triangles x every lane).  Here the work of
// a bounce batch is a set of (ray, node group) and (ray, triangle) PAIRS held in two per-wave LIFO
// stacks in LDS; every step hands 64 pairs of one kind to the 64 lanes, so lanes stay full whatever the
// rays' directions.  A node pair tests every member of a group (the 2..4 children of a kept node of
// the wide image, hrt_bvh.h make_wq_nodes) for its ray, pushes the inner ones (sorted: the farther
// below, and all of a step's nearest children above all its farther ones, so the next step descends
// toward the rays' nearest hits) and the leaves' triangles.  The ray of a pair is read
// from its owner lane (ds_bpermute); its closest hit so far is a 64-bit LDS slot (t bits << 32 |
// (mesh << 26 | triangle) + 1), lowered with ds_min_u64: the minimum over every triangle the
// reference accepts of (dist, scan position), i.e. raytracing.glsl's strict '<' in scan order (spheres
// hold key 0 and win ties, as they are scanned first).  A child is dropped only by BUNDLE_BVH's exact
// node test (wq_node_visit) against the slot's current t, which only ever exceeds the final one.
// When the node stack could overflow, the popped groups' subtrees are walked stacklessly instead.
#ifndef HRT_WQ_CONE
#define HRT_WQ_CONE 1    // the nodes' back-face (normal cone) test
#endif
#ifndef HRT_WQ_BRANCHLESS
#define HRT_WQ_BRANCHLESS 1  // member test without the back-face early-out branch (r03s: island -0.6%, cave -0.3% with ALL4)
#endif
#ifndef HRT_WQ_ALL4
#define HRT_WQ_ALL4 1  // all four member slots tested, masked past the group's count (r03s, with BRANCHLESS)
#endif
#ifndef HRT_WQ_SELECT
#define HRT_WQ_SELECT 1  // a member's outcome as selects instead of a branch (r03t)
#endif
#ifndef HRT_WQ_CONE_SQ
#define HRT_WQ_CONE_SQ 1  // the members' back-face test squared, no square root (r03t)
#endif
#ifndef HRT_WQ_FMA_SLACK
#define HRT_WQ_FMA_SLACK 1  // member test: slack compare and the cone's first product as fmas (r03t)
#endif
#ifndef HRT_WQ_LEAF_FLAT
#define HRT_WQ_LEAF_FLAT 1  // kept leaves' triangle pairs pushed by one loop over the lane's count (r03u: island -1.3%, cave -1.7%)
#endif
#ifndef HRT_WQ_TRI_SELECT
#define HRT_WQ_TRI_SELECT 1  // the triangle pre-test's rejections as one predicate (r03y: cave -0.4%)
#endif
#ifndef HRT_WQ_PUSH_DUMP
#define HRT_WQ_PUSH_DUMP 0  // (A/B) inner-member pushes without a branch (non-pushing lanes store to a dump word)
#endif
#ifndef HRT_WQ_BAND_PLANE
#define HRT_WQ_BAND_PLANE 1  // band entries whose plane the ray starts behind are dropped (r03aa: band tests per cave lane 3.9 -> 0.8; island -0.9%, cave -1.6%)
#endif
#ifndef HRT_WQ_MIXED
#define HRT_WQ_MIXED 1   // short node and triangle stacks share one step
#endif
#ifndef HRT_WQ_EARLY_REC
#define HRT_WQ_EARLY_REC 1  // a node step's first member pair read before the slot read (r04)
#endif
#ifndef HRT_WQ_BAND_EARLY
#define HRT_WQ_BAND_EARLY 0  // (r05b: neutral, island 1.786 / 1.787, cave 5.405 / 5.400 ms) a bounce lane's direction-cell offsets requested at the batch's start (r05)
#endif
#ifndef HRT_WQ_BAND_AHEAD
#define HRT_WQ_BAND_AHEAD 1  // band-list rounds whose entry loads are in flight at once (1: one round ahead)
#endif
#ifndef HRT_WQ_TRI_MIN
#define HRT_WQ_TRI_MIN 64u  // a triangle step runs once this many triangle pairs wait (or no node pair is left)
#endif

// Widest node group the kernel tests per stack entry (hrt_bvh.h kWqMaxWidth).  Measured (r02,
// profiles/r02j_wq_groups_ab.jsonl): 8 slots ran the 4-wide image 9% slower (registers), and the
// triangle stack of an 8-wide image does not fit the LDS; fully ordering the 4 slots (5
// compare-exchanges, HRT_WQ_FULLSORT) instead of only putting the nearest last (3) was 0.9% slower.
constexpr uint32_t kWqSlots = 4;

struct WqLds {
  const float4* nodes;        // BVH nodes (LDS copy)
  unsigned long long* slot;   // 64 per wave: closest hit so far per ray (owner lane)
  uint32_t* ns;               // node-group stack: group word (fc | (count - 1) << 16) << 6 | ray
  uint32_t* ts;               // triangle-pair stack: leaf prim << 6 | ray
  uint32_t ncap;              // node stack capacity (>= 256)
};

__device__ __forceinline__ f3 shfl3(f3 v, uint32_t r) {
  return mk(lane_read(v.x, r), lane_read(v.y, r), lane_read(v.z, r));
}

// BUNDLE_WQ node image (hrt_bvh.h make_wq_nodes): 3 float4 per node, cone in binary16.
__device__ __forceinline__ float half_lo(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xFFFFu)); }
__device__ __forceinline__ float half_hi(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); }
// The cone's sine from its image word: the image holds S >= sin^2 x 1.00001 (hrt_bvh.h [10]), so
// sqrt(S), widened by the hardware root's error, is an upper bound of sin
__device__ __forceinline__ float wq_sin_up(uint32_t w10) { return __builtin_amdgcn_sqrtf(half_lo(w10)) * 1.0000005f; }
__device__ __forceinline__ uint32_t wq_info(const float4* nodes, uint32_t k) {  // leaf info / right child
  return __builtin_bit_cast(uint32_t, nodes[3 * k + 2].w);
}
__device__ __forceinline__ uint32_t wq_escape(const float4* nodes, uint32_t k) {
  return __builtin_bit_cast(uint32_t, nodes[3 * k + 2].z) >> 16;
}
// compare-exchange of two pushed-child slots: the smaller key (the farther child) first
__device__ __forceinline__ void wq_order(float& ka, uint32_t& ea, float& kb, uint32_t& eb) {
  const bool sw = kb < ka;
  const float k = sw ? kb : ka;
  kb = sw ? ka : kb;
  ka = k;
  const uint32_t e = sw ? eb : ea;
  eb = sw ? ea : eb;
  ea = e;
}

// bvh_node_visit on the 48 B image: the cone axis carries up to kWqAxisErr of binary16 error in d.axis
// (allowed for in both the back-face bound and the sine bound; cos is rounded down and sin up), and
// the hardware square root (1 ulp; +2e-7 keeps the sine an upper bound) -- a node is only ever kept
// more often than by bvh_node_visit.  t_near: the box entry distance (ordering only).
__device__ __forceinline__ bool wq_node_visit_r(const float4& N0, const float4& N1, const float4& N2, f3 o, f3 d,
                                                f3 inv, float R, float abs_t, float t_hi, float& t_near) {
  const uint32_t w8 = __builtin_bit_cast(uint32_t, N2.x), w9 = __builtin_bit_cast(uint32_t, N2.y),
                 w10 = __builtin_bit_cast(uint32_t, N2.z);
  const float x = half_lo(w8) * d.x + half_hi(w8) * d.y + half_lo(w9) * d.z;
  const float xa = fmaxf(fabsf(x) - (2e-6f + kWqAxisErr), 0.0f);
  const float s_up = __builtin_amdgcn_sqrtf(fmaxf(1.0f - xa * xa, 0.0f)) + 1.2e-6f;
  if (HRT_WQ_CONE && (x - kWqAxisErr) * half_hi(w9) - s_up * wq_sin_up(w10) - 1e-6f > 1e-5f) return false;  // back
  const float mg = N0.w + N1.w * R;
  const float tx0 = ((N0.x - mg) - o.x) * inv.x, tx1 = ((N1.x + mg) - o.x) * inv.x;
  const float ty0 = ((N0.y - mg) - o.y) * inv.y, ty1 = ((N1.y + mg) - o.y) * inv.y;
  const float tz0 = ((N0.z - mg) - o.z) * inv.z, tz1 = ((N1.z + mg) - o.z) * inv.z;
  const float tn = fmaxf(fmaxf(-abs_t, fminf(tx0, tx1)), fmaxf(fminf(ty0, ty1), fminf(tz0, tz1)));
  const float tf = fminf(fminf(t_hi, fmaxf(tx0, tx1)), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
  t_near = tn;
  return !((tn - fabsf(tn) * 1e-6f) > (tf + fabsf(tf) * 1e-6f));  // NaN -> visit
}
__device__ __forceinline__ bool wq_node_visit(const float4* nd, f3 o, f3 d, f3 inv, float R, float abs_t, float t_hi,
                                              float& t_near) {
  return wq_node_visit_r(nd[0], nd[1], nd[2], o, d, inv, R, abs_t, t_hi, t_near);
}
// A node step's ray, prepared once for the group's members (wq_member_visit).
struct WqRay {
  f3 o, d, inv;
  f3 oi;       // RN(o * inv) per axis
  float sig;   // 2^-23 max |o * inv|: covers the rounding of oi in each slab distance
  float R, abs_t;
};
__device__ __forceinline__ WqRay wq_ray(f3 o, f3 d, f3 inv, float R, float abs_t) {
  WqRay q;
  q.o = o;
  q.d = d;
  q.inv = inv;
  q.R = R;
  q.abs_t = abs_t;
  q.oi = mk(o.x * inv.x, o.y * inv.y, o.z * inv.z);
  q.sig = fmaxf(fmaxf(fabsf(q.oi.x), fabsf(q.oi.y)), fabsf(q.oi.z)) * 0x1p-23f;
  return q;
}
// wq_node_visit_r for a prepared ray, each slab distance as fma(bound, inv, -o inv): the exact
// (bound - o) inv plus at most 2^-24 of the result and 2^-24 |o inv| (the rounding of oi), covered by
// the 1e-6 relative slack and 2 sig on the interval test (one fma instead of a subtract and a
// multiply per bound: island 3.242 -> 3.228 ms, profiles/r02k_node_test_ab.txt).  inv = +-inf gives
// NaN -> visit.  (Measured and dropped: d.axis from binary16 d with v_dot2_f32_f16, 3.345 ms.)
template <bool NodeR>
__device__ __forceinline__ bool wq_member_visit(const float4& N0, const float4& N1, const float4& N2, const WqRay& q,
                                                float t_hi, float& t_near) {
  const uint32_t w8 = __builtin_bit_cast(uint32_t, N2.x), w9 = __builtin_bit_cast(uint32_t, N2.y),
                 w10 = __builtin_bit_cast(uint32_t, N2.z);
  // (fused: each rounding here is far inside the 2e-6 / 1e-6 slacks, and the host's margins carry 1e-6
  // relative headroom over one rounding of a + b R)
#if HRT_WQ_FMA_SLACK
  // the first product as an fma with +0 (v_fma_mix_f32 reads the binary16 operand directly)
  const float x = __builtin_fmaf(half_lo(w9), q.d.z, __builtin_fmaf(half_hi(w8), q.d.y, __builtin_fmaf(half_lo(w8), q.d.x, 0.0f)));
#else
  const float x = __builtin_fmaf(half_lo(w9), q.d.z, __builtin_fmaf(half_hi(w8), q.d.y, half_lo(w8) * q.d.x));
#endif
  const float xa = fmaxf(fabsf(x) - (2e-6f + kWqAxisErr), 0.0f);
  // (the cone test pays on cave too with per-node radii: without it 7.25 -> 7.43 ms, r03c)
#if HRT_WQ_CONE_SQ
  // The test below squared, without the square root and only ever stricter.  It is back <=> L > s_up sin
  // with L = (x - E) cos - 1.1e-5 and s_up = sqrt(q) + 1.2e-6 (q = max(1 - xa^2, 0); the hardware root is
  // within 1.2e-7 of sqrt(q) on [0, 1]).  Here: L' = (x - E) cos - 1.2e-5 (its two roundings < 2.4e-7
  // below the 1e-6 extra), and s_up^2 <= (sqrt(q) + 1.4e-6)^2 <= q + 3e-6 (sqrt(q) <= 1); the image's
  // S >= sin^2 x 1.00001 (rounded up, hrt_bvh.h [10]) leaves the two roundings of (q2 + 3e-6) S and the one
  // of L'^2 (< 1.8e-7 relative) far inside the x1.00001.  L' > 0 and L'^2 > that imply L > s_up sin.
  // (r04: S precomputed -- one mixed-precision multiply instead of a conversion and three multiplies)
  // NaN -> not back.
  const float q2 = fmaxf(__builtin_fmaf(-xa, xa, 1.0f), 0.0f);
  const float L = __builtin_fmaf(x - kWqAxisErr, half_hi(w9), -1.2e-5f);
  const bool back = HRT_WQ_CONE && L > 0.0f && L * L > __builtin_fmaf(q2 + 3e-6f, half_lo(w10), 0.0f);
#else
  const float s_up = __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-xa, xa, 1.0f), 0.0f)) + 1.2e-6f;
  const bool back = HRT_WQ_CONE && (x - kWqAxisErr) * half_hi(w9) - s_up * wq_sin_up(w10) - 1e-6f > 1e-5f;
#endif
#if !HRT_WQ_BRANCHLESS
  if (back) return false;
#endif
  float Rm = q.R;
  if constexpr (NodeR) {  // trace_bundle_wq_nr (HRT_OPT_WQ_NODE_RADIUS)
    // R for this member: the ray origin's distance to the farthest corner of its box (every vertex
    // below lies in the box), x1.0001 over the roundings and the hardware square root
    const float fx = fmaxf(q.o.x - N0.x, N1.x - q.o.x), fy = fmaxf(q.o.y - N0.y, N1.y - q.o.y),
                fz = fmaxf(q.o.z - N0.z, N1.z - q.o.z);
    Rm = fminf(__builtin_amdgcn_sqrtf(__builtin_fmaf(fz, fz, __builtin_fmaf(fy, fy, fx * fx))) * 1.0001f, q.R);
  }
  // (Cone-scaled margins -- c0 + (a + b R) tau_g / tau_e when the member's normal cone bounds -d.n^ >= tau_e
  // > tau_g -- measured slower: cave 6.37 -> 6.60, island 2.25 -> 2.30 ms, profiles/r03/r03g_cone_margin_ab.)
  const float mg = __builtin_fmaf(N1.w, Rm, N0.w);
  const float tx0 = __builtin_fmaf(N0.x - mg, q.inv.x, -q.oi.x), tx1 = __builtin_fmaf(N1.x + mg, q.inv.x, -q.oi.x);
  const float ty0 = __builtin_fmaf(N0.y - mg, q.inv.y, -q.oi.y), ty1 = __builtin_fmaf(N1.y + mg, q.inv.y, -q.oi.y);
  const float tz0 = __builtin_fmaf(N0.z - mg, q.inv.z, -q.oi.z), tz1 = __builtin_fmaf(N1.z + mg, q.inv.z, -q.oi.z);
  const float tn = fmaxf(fmaxf(-q.abs_t, fminf(tx0, tx1)), fmaxf(fminf(ty0, ty1), fminf(tz0, tz1)));
  const float tf = fminf(fminf(t_hi, fmaxf(tx0, tx1)), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
  t_near = tn;
#if HRT_WQ_BRANCHLESS && HRT_WQ_FMA_SLACK
  // the 1e-6 relative slacks as fmas (one rounding fewer each; the products' roundings were far inside
  // the slacks either way)
  return !back & !(__builtin_fmaf(-fabsf(tn), 1e-6f, tn) > __builtin_fmaf(fabsf(tf), 1e-6f, tf) + 2.0f * q.sig);
#elif HRT_WQ_BRANCHLESS
  return !back & !((tn - fabsf(tn) * 1e-6f) > (tf + fabsf(tf) * 1e-6f) + 2.0f * q.sig);  // NaN -> visit
#else
  return !((tn - fabsf(tn) * 1e-6f) > (tf + fabsf(tf) * 1e-6f) + 2.0f * q.sig);  // NaN -> visit
#endif
}

// Exact reference test (raytracing.glsl:213-241) of BVH leaf prim record (a, -) (e1, -) (e2, -) (n, -):
// true with dist when the reference accepts the triangle (dist > 0.001, u, v, w >= 0); the division-free
// pre-test (pre_reject) skips candidates beyond best_k first.
__device__ __forceinline__ bool wq_tri_accept(const float4& A, const float4& B, const float4& C, const float4& N, f3 o,
                                              f3 d, float best_k, float& dist) {
  const f3 n = mk(N.x, N.y, N.z);
  const f3 ao = o - mk(A.x, A.y, A.z);
  TriPre q;
  q.num_t = dot(ao, n);
#if HRT_WQ_TRI_SELECT
  // the three rejections as one predicate (no early-out branches: in a step of 64 different pairs they
  // almost never skip the whole wave)
  const float dn = dot(d, n);
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  if (!(q.num_t > 0.0f) | !(dn < 0.0f) | pre_reject(q, best_k)) return false;
#else
  if (!(q.num_t > 0.0f)) return false;
  const float dn = dot(d, n);
  if (!(dn < 0.0f)) return false;
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  if (pre_reject(q, best_k)) return false;
#endif
  const float inv_det = 1.0f / q.det;
  dist = q.num_t * inv_det;
  const float u = q.num_u * inv_det;
  const float v = -q.num_v * inv_det;
  const float w = 1.0f - u - v;
  return !(dist < 0.0f) && !(u < 0.0f) && !(v < 0.0f) && !(w < 0.0f) && dist > 0.001f;
}

// closest-hit slot of ray (lane) r: seeded by its owner, lowered by any lane, read for pruning by any
// lane (a stale value only prunes less: the slot never increases) and finally by its owner
__device__ __forceinline__ void wq_slot_seed(unsigned long long* slot, uint32_t lane, unsigned long long v) {
  lds_put(&slot[lane], v);
}
__device__ __forceinline__ void wq_slot_lower(unsigned long long* slot, uint32_t r, unsigned long long v) {
  __hip_atomic_fetch_min(&slot[r], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ float wq_slot_t(const WqLds& wq, uint32_t r) {
  return __uint_as_float(lds_get(reinterpret_cast<const uint32_t*>(wq.slot) + (2 * r + 1)));
}
// pair stacks: the lanes with `push` append v in lane order at the wave-uniform top n
__device__ __forceinline__ void wq_push(uint32_t* st, uint32_t& n, bool push, uint32_t v) {
  const unsigned long long b = __ballot(push);
  if (push) lds_put(&st[n + lanes_below(b)], v);
  n += (uint32_t)__popcll(b);
}

// Leaf prim k for ray r (origin o, direction d, mesh filter mask): test and lower the ray's slot.
struct WqTriRec {
  float4 A, B, C, N;
};
__device__ __forceinline__ WqTriRec wq_tri_rec(const float4* __restrict__ pr, uint32_t k) {
  return WqTriRec{pr[4 * k], pr[4 * k + 1], pr[4 * k + 2], pr[4 * k + 3]};
}
__device__ __forceinline__ void wq_tri_test(const WqTriRec& t, const WqLds& wq, uint32_t r, unsigned long long mask,
                                            f3 o, f3 d) {
  const float4 &A = t.A, &B = t.B, &C = t.C, &N = t.N;
  const uint32_t m = __builtin_bit_cast(uint32_t, B.w);
  float dist;
  // the mesh filter (its quirky AABB test for this ray) joins the acceptance instead of leaving
  // first, so the four record loads issue together (one L2 round trip per triangle step, not two)
  if (wq_tri_accept(A, B, C, N, o, d, wq_slot_t(wq, r) * kOnePlus, dist) && ((mask >> m) & 1ull)) {
    const uint32_t id = ((m << 26) | __builtin_bit_cast(uint32_t, C.w)) + 1u;
    wq_slot_lower(wq.slot, r, ((unsigned long long)__float_as_uint(dist) << 32) | id);
  }
}
__device__ __forceinline__ void wq_leaf_prim(const float4* __restrict__ pr, const WqLds& wq, uint32_t k, uint32_t r,
                                             unsigned long long mask, f3 o, f3 d) {
  wq_tri_test(wq_tri_rec(pr, k), wq, r, mask, o, d);
}


// The grazing-band lists of a wave's lanes laid end to end (world_hit_bounce_wq): lane l's list of n
// entries starts at global slot pos (exclusive prefix of the lengths), total slots.  slot(base, own)
// gives this lane's slot base + lane of a 64-slot round: its owner lane (the last with pos <= slot and a
// non-empty list) and the owner's entry index (b0 + slot - pos; 0 past the end).  The lanes whose lists
// start in the round mark their start slot (lane + 1, one byte each, in 64 bytes of LDS); a slot's owner
// is the mark at its highest marked slot at or below it, or the previous round's last owner when none is
// (carry).  All 64 lanes active.  hrt_debug_band_flatten runs it on given lists (tests/test_gpu_boundary.py).
struct BandFlat {
  uint8_t* marks;
  uint32_t lane, n, pos, total, delta;  // delta = b0 - pos: entry of slot g = the owner's delta + g (mod 2^32)
  uint32_t carry;
  __device__ __forceinline__ uint32_t slot(uint32_t base, uint32_t& own) {
    // (a slot's mark is another lane's store: with plain accesses hipcc forwarded this lane's own
    // clearing store to the load on the path where the lane marks nothing -- losing the start marks of
    // lists that begin at the slot of a lane with no list of its own; lds_put / lds_get / wave_handoff)
    lds_put(&marks[lane], (uint8_t)0);
    wave_handoff();  // every clear before any lane's mark
    const uint32_t rel = pos - base;
    if (n && rel < 64u) lds_put(&marks[rel], (uint8_t)(lane + 1u));
    wave_handoff();  // every mark before any lane's read
    const uint32_t v = lds_get(&marks[lane]);
    const unsigned long long m = __ballot(v != 0u) & (lane == 63u ? ~0ull : (2ull << lane) - 1ull);
    const uint32_t s = m ? 63u - (uint32_t)__builtin_clzll(m) : 0u;
    const uint32_t sv = lane_read(v, s);
    own = m ? sv - 1u : carry;
    carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
    const uint32_t gi = base + lane;
    owner_delta = lane_read(delta, own);
    const uint32_t k = owner_delta + gi;
    return gi < total ? k : 0u;
  }
  uint32_t owner_delta = 0;  // the last slot()'s owner's delta (its bit 31: the record flag, world_hit_bounce_wq)
};

// A bounce lane's direction cell: its band list's first entry b0 and length n.  With per-cell records
// (TraceParams::bvh_band_rec: 8 dwords per cell -- the list's start, its length, then its first
// kBandInline entries as half-words) one 8-byte load gives both, and a list that fits the record is read
// from it: b0 = the record's first entry as a half-word index of the records, with bit 31 set (the
// slots then load from the line the owner just brought in instead of a second random line).
// Otherwise the offsets (two words of one line) and the list.
constexpr uint32_t kBandInline = 12;
__device__ __forceinline__ void band_cell(const KArgs K, f3 d, uint32_t& b0, uint32_t& n) {
  const uint32_t cell = dir_cell(d, K->bvh_dir_res);
  if (const uint32_t* rec = K->bvh_band_rec) {
    const uint2 h = *reinterpret_cast<const uint2*>(rec + (size_t)cell * 8u);
    n = h.y;
    b0 = n <= kBandInline ? (cell * 16u + 4u) | 0x80000000u : h.x;
  } else {
    const uint32_t* band_off = K->bvh_band_off;
    b0 = band_off[cell];
    n = band_off[cell + 1] - b0;
  }
}

template <bool D, bool NodeR>
__device__ __forceinline__ void world_hit_bounce_wq(const Scene& sc, const TraceParams& P, const WqLds& wq, bool sec,
                                                    f3 o, f3 d, uint32_t& tests, Closest& c, Diag& dg) {
  const hrt_push_constants& pc = P.pc;
  const uint32_t lane = threadIdx.x & 63;
  // the batch's constants, read here (kargs): live for the batch only
  const KArgs K = kargs();
  const float4* prims = K->bvh_prims;
  const float rel_t = K->bvh_rel_t, abs_coef = K->bvh_abs_coef;
  const uint32_t tcap = K->wq_tcap;
#if HRT_WQ_BAND_EARLY
  // the lane's direction-cell offsets requested first: the band rounds' first dependent global read (a
  // random line of a structure far larger than an XCD's L2) then overlaps the spheres, the reciprocals,
  // the meshes' AABB tests and the irregular list instead of starting after them
  uint32_t cb0 = 0, cb1 = 0;
  if (sec) band_cell(K, d, cb0, cb1);
#endif
  spheres_first(sc, pc, sec, o, d, c);
  const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);  // the meshes' AABB tests and the traversal
  unsigned long long mask = 0ull;
  if (sec) {
    for (int m = 0; m < pc.num_meshes; ++m) {
      const hrt_mesh& mesh = sc.meshes[m];
      if (aabb_pass_inv(mesh, o, inv)) {
        mask |= 1ull << m;
        tests += mesh.len;
      }
    }
  }
  // the irregular list: per lane, as in BUNDLE_BVH
  uint32_t bkey = 0;
  float best_k = c.t * kOnePlus;
  const uint32_t n_irr = K->bvh_n_irregular;
  const float4* irr = K->bvh_irregular;
  for (uint32_t k = 0; k < n_irr; ++k)
    if (sec) bvh_prim_test(irr, k, mask, o, d, c, bkey, best_k);
  float R;
  {  // farthest root-box corner from the origin, rounded up
    const float4 R0 = wq.nodes[0], R1 = wq.nodes[1];
    const float fx = fmaxf(fabsf(o.x - R0.x), fabsf(R1.x - o.x)), fy = fmaxf(fabsf(o.y - R0.y), fabsf(R1.y - o.y));
    const float fz = fmaxf(fabsf(o.z - R0.z), fabsf(R1.z - o.z));
    R = __builtin_amdgcn_sqrtf(fx * fx + fy * fy + fz * fz) * 1.0001f;  // 1 ulp, inside the x1.0001
  }
  const float abs_t = abs_coef * R;
  uint32_t band_tests = 0, band_lmax = 0;
  // the ray's closest hit so far (spheres, the irregular list) seeds its slot
  const uint32_t id0 = c.kind == 2 ? ((c.mesh << 26) | c.idx) + 1u : 0u;
  wq_slot_seed(wq.slot, lane, ((unsigned long long)__float_as_uint(c.t) << 32) | id0);
  wave_handoff();  // seeds before any lane's read or lowering
  uint32_t tc = 0, tri_pairs = 0, steps = 0;
  // one step of 64 waiting triangle pairs (the band rounds' overflow guard)
  auto tri_step64 = [&]() {
    tc -= 64u;
    wave_handoff();
    const uint32_t e = lds_get(&wq.ts[tc + lane]), r = e & 63u;
    const unsigned long long rm = mask_read(mask, r, K->pc.num_meshes);
    wq_leaf_prim(prims, wq, e >> 6, r, rm, shfl3(o, r), shfl3(d, r));
    wave_handoff();  // these pops before the round's pushes into their words
    tri_pairs += 64u;
    ++steps;
  };
  // Grazing band, flattened over the wave: the bounce lanes' direction-cell lists laid end to end
  // (exclusive prefix pos of their lengths), 64 entries per round whatever the lists' lengths (the
  // per-lane scan ran as long as the batch's longest list: 33 entries against 9.3 per lane on
  // island).  Slot g's list is the last lane with pos <= g; an entry that passes its ray's pre-check
  // becomes a (ray, prim) pair of the triangle steps, whose slot minimum is the per-lane scan's result.
  // r03: the scan is a chain of latencies, not VALU (without it -- wrong frames -- island 2.26 -> 1.99,
  // cave 6.41 -> 5.42 ms): 2-byte entries with the prims' normals in a table (fetched bytes 1.08 ->
  // 0.36 GB per island frame), rounds pipelined one ahead, ballot prefix and start marks instead of
  // 6-step shuffle scans and binary searches: island 2.257 -> 2.154, cave 6.411 -> 6.066 ms
  // (profiles/r03/r03i..r03l; a two-stage pipeline and offsets requested at the bounce's start were
  // no faster).
  if (__any(sec && mask)) {
    const BandCheck bc(d, -K->bvh_band_tau - 2e-5f, 3e-5f);  // see world_hit_bounce_bvh
#if HRT_WQ_BAND_PLANE
    // Plane-side filter: an entry whose plane the ray starts behind, s = n^.o - n^.a < -ptol, cannot be
    // accepted.  The reference's num_t = dot(o - a, n) is within 4 eps (|o|_1 + |a|_1) |n| of |n| times
    // the exact n^.(o - a), and s within 6 eps (|o|_1 + |a|_1) of it (n^ within 2^-24 per component, the
    // fma chain, the host's rounding of n^.a, the subtraction), so s < -1e-5 (|o|_1 + max |a|_1) means
    // num_t < 0: dist <= 0, rejected (raytracing.glsl:233-238).  NaN -> kept.
    const float ptol = 1e-5f * (fabsf(o.x) + fabsf(o.y) + fabsf(o.z) + K->bvh_band_a1);
#endif
    uint32_t b0 = 0, n = 0;
#if HRT_WQ_BAND_EARLY
    if (sec && mask) {
      b0 = cb0;
      n = cb1;
    }
#else
    if (sec && mask) band_cell(K, d, b0, n);
#endif
    if (D && P.diag) {
      dg.band_len += n;
      band_lmax = n;
    }
    // exclusive prefix pos of the lengths and their total (wave_scan_excl; r03 used bit-plane ballots --
    // bvh_band_bits = the bit width of the scene's longest list; a 6-step shuffle scan was slower)
    uint32_t total;
    const uint32_t pos = wave_scan_excl(n, total, K->bvh_band_bits);
    const void* band = K->bvh_band;
    const uint32_t wide = K->bvh_band_wide;
    const float4* nhat = K->bvh_band_nhat;
    uint8_t* const marks = reinterpret_cast<uint8_t*>(wq.ns);  // (the node stack's words: empty until the root is tested)
    // (with records, b0 of a list kept in its record is a half-word index of the records with bit 31 set,
    // band_cell: the delta keeps that flag and is taken mod 2^31)
    const uint32_t* rec = K->bvh_band_rec;
    BandFlat bf{marks, lane, n, pos, total, rec ? (b0 & 0x80000000u) | ((b0 - pos) & 0x7FFFFFFFu) : b0 - pos, 0u};
    auto fetch = [&](uint32_t base, uint32_t& own, uint32_t& q) {
      const uint32_t k = bf.slot(base, own);
      if (rec) {  // (kernel argument: wave-uniform) one dword load from the record or the list, no branch
        const uint32_t i = k & 0x7FFFFFFFu;
        const uint32_t* w = (bf.owner_delta >> 31) ? rec : static_cast<const uint32_t*>(band);
        q = (w[i >> 1] >> ((i & 1u) << 4)) & 0xFFFFu;
      } else {
        q = band_entry(band, wide, k);  // (slots past the end: entry 0, unused)
      }
    };
    // Software-pipelined rounds: the next round's owner search and entry load are issued after this
    // round's normal load and before its check, so a round waits for the (cache-resident) normal
    // alone while the next round's (mostly L2-missing) entry load is in flight.  (The last round
    // fetches a round past the end too: a conditional load would make the normal's wait a full drain.)
#if HRT_WQ_BAND_AHEAD > 1
    // (A/B) the entry loads of the first HRT_WQ_BAND_AHEAD rounds issued together, then each round
    // fetches the round that far ahead: the lists' random lines (a 74 MB structure no L2 holds) wait
    // in parallel instead of one round at a time
    uint32_t own_r[HRT_WQ_BAND_AHEAD], q_r[HRT_WQ_BAND_AHEAD];
#pragma unroll
    for (int i = 0; i < HRT_WQ_BAND_AHEAD; ++i) {
      own_r[i] = 0u;
      q_r[i] = 0u;
      if (total > 64u * (uint32_t)i) fetch(64u * (uint32_t)i, own_r[i], q_r[i]);
    }
    for (uint32_t base = 0; base < total; base += 64u) {
      if (tc + 64u > tcap) tri_step64();  // room for this round's pairs
      const uint32_t own = own_r[0], q = q_r[0];
      const float4 nh = nhat[q];
#pragma unroll
      for (int i = 0; i + 1 < HRT_WQ_BAND_AHEAD; ++i) {
        own_r[i] = own_r[i + 1];
        q_r[i] = q_r[i + 1];
      }
      uint32_t own_n, q_n;
      fetch(base + 64u * HRT_WQ_BAND_AHEAD, own_n, q_n);
      own_r[HRT_WQ_BAND_AHEAD - 1] = own_n;
      q_r[HRT_WQ_BAND_AHEAD - 1] = q_n;
#else
    uint32_t own = 0, q = 0;
    if (total) fetch(0u, own, q);
    for (uint32_t base = 0; base < total; base += 64u) {
      if (tc + 64u > tcap) tri_step64();  // room for this round's pairs
      const float4 nh = nhat[q];
      uint32_t own_n, q_n;
      fetch(base + 64u, own_n, q_n);
#endif
      BandCheck oc = bc;
      oc.d = shfl3(bc.d, own);
#if HRT_WQ_BAND_PLANE
      const f3 oo = shfl3(o, own);
      const float ot = lane_read(ptol, own);
      const float sp = __builtin_fmaf(oo.z, nh.z, __builtin_fmaf(oo.y, nh.y, oo.x * nh.x)) - nh.w;
      const bool push = base + lane < total && oc.in(nh) && !(sp < -ot);
#else
      const bool push = base + lane < total && oc.in(nh);
#endif
      const unsigned long long pb = __ballot(push);
#if HRT_WQ_PUSH_DUMP
      // (non-pushing lanes store into the node stack's last word: empty during the band rounds)
      lds_put(push ? &wq.ts[tc + lanes_below(pb)] : &wq.ns[wq.ncap - 1u], (q << 6) | own);
#else
      if (push) lds_put(&wq.ts[tc + lanes_below(pb)], (q << 6) | own);
#endif
      tc += (uint32_t)__popcll(pb);
      band_tests += push ? 1u : 0u;
#if HRT_WQ_BAND_AHEAD <= 1
      own = own_n;
      q = q_n;
#endif
    }
  }
  // pair traversal: the root is tested per lane, then (ray, node group) / (ray, triangle) pairs
  uint32_t rinfo = 0;
  bool rvis = false;
  if (sec && mask) {
    float tn;
    rinfo = wq_info(wq.nodes, 0);
    rvis = wq_node_visit(wq.nodes, o, d, inv, R, abs_t, c.t * (1.0f + rel_t) + abs_t, tn);
  }
  const uint32_t rcnt = rvis ? rinfo >> 27 : 0u;
  const unsigned long long rb = __ballot(rvis && rcnt == 0u);
  wave_handoff();  // the band rounds' marks (in the node stack's words) before the root pushes
  if (rvis && rcnt == 0u) lds_put(&wq.ns[lanes_below(rb)], (rinfo << 6) | lane);  // inner root: its children's group
  uint32_t nc = (uint32_t)__popcll(rb);
  {  // leaf root (a scene of at most leaf-size triangles): its triangles, after any band pairs
    uint32_t tot;
    const uint32_t pre = tc + wave_scan_excl(rcnt, tot, 5u);
    for (uint32_t j = 0; j < rcnt; ++j) lds_put(&wq.ts[pre + j], (((rinfo & 0x07FFFFFFu) + j) << 6) | lane);
    tc += tot;
  }
  const uint32_t width = K->bvh_wq_width;  // the image's largest group
  uint32_t node_pairs = 0;
  while (nc | tc) {
    ++steps;
    // Step composition (wave-uniform): triangle pairs when >= 64 wait or no node pair is left; when
    // both stacks are short, one mixed step takes them all (lanes [0, nn) node pairs, then triangles).
    // (Measured, r02: filling a short node step's idle lanes with triangle pairs, or running triangle
    // steps from 32 waiting pairs, was no faster: 3.699 / 3.722 vs 3.692 ms, profiles/r02g_ab.txt.)
    const bool tri_step = tc >= HRT_WQ_TRI_MIN || nc == 0u;
    const bool mixed = HRT_WQ_MIXED && !tri_step && tc > 0u && nc + tc <= 64u;
    const uint32_t tn = tri_step ? min(64u, tc) : (mixed ? tc : 0u);
    const uint32_t nn = tri_step ? 0u : min(64u, nc);
    tc -= tn;
    nc -= nn;
    node_pairs += nn;
    tri_pairs += tn;
    const bool overflow = nc + width * nn > wq.ncap - (HRT_WQ_PUSH_DUMP ? 1u : 0u);  // wave-uniform
    const bool is_node = lane < nn, is_tri = lane >= nn && lane < nn + tn;
    if (D && P.diag && nn) ++dg.wq_fill[(nn - 1u) >> 4];
    wave_handoff();  // the last step's pushes and slot lowerings before this step's pops and reads
    const uint32_t e = is_node ? lds_get(&wq.ns[nc + lane]) : is_tri ? lds_get(&wq.ts[tc + lane - nn]) : lane;
    const uint32_t r = e & 63u;
    const f3 ro = shfl3(o, r), rd = shfl3(d, r);
    const unsigned long long rm = mask_read(mask, r, K->pc.num_meshes);
    if (is_tri) wq_leaf_prim(prims, wq, e >> 6, r, rm, ro, rd);
    if (nn == 0u) continue;
    // node pairs (ray r, group fc .. fc + cnt - 1): test every member.  Slot k: member k's push entry
    // (its info word << 6 | r when a kept inner node, else ~0u), sort key (minus its box entry
    // distance when pushed, else -inf), and its triangle count when a kept leaf.
    // (r03, measured slower: fetching the mesh filter only for steps with triangle pairs and abs_t as
    // abs_coef * R instead of a shuffle -- island 2.271 -> 2.276, cave 7.248 -> 7.310 ms)
    const f3 rinv = shfl3(inv, r);
    const float rR = lane_read(R, r), rabs = lane_read(abs_t, r);
    const WqRay rq = wq_ray(ro, rd, rinv, rR, rabs);
    uint32_t pe[kWqSlots], li[kWqSlots];
    float pk[kWqSlots];
#pragma unroll
    for (int k = 0; k < (int)kWqSlots; ++k) {
      pe[k] = ~0u;
      li[k] = 0u;
      pk[k] = -kFltMax;
    }
    if (is_node) {
      const uint32_t g = e >> 6, fc = g & 0xFFFFu, gcnt = (g >> 16) + 1u;
      if (D && P.diag) dg.wq_members += gcnt;
      if (!overflow) {
#if HRT_WQ_EARLY_REC
        // the first member pair's records are requested before the slot read: that read is an atomic
        // (lds_get), which the scheduler keeps every other memory access on its side of, so requested
        // after it they waited for the ray shuffles and the slot before being issued
        const float4* na0 = wq.nodes + 3 * fc;
        const float4* nb0 = wq.nodes + 3 * (fc + min(1u, gcnt - 1u));
        const float4 A00 = na0[0], A01 = na0[1], A02 = na0[2], B00 = nb0[0], B01 = nb0[1], B02 = nb0[2];
        // (both pairs up front: 24 more live VGPRs, scratch 92 -> 160 B with spills in the fused loop)
#endif
        const float t_hi = wq_slot_t(wq, r) * (1.0f + rel_t) + rabs;
        auto member = [&](const float4& N0, const float4& N1, const float4& N2, int k, bool valid = true) {
          float tnear;
          const uint32_t inf = __builtin_bit_cast(uint32_t, N2.w);
#if HRT_WQ_SELECT
          // the outcome as selects: no branch, and the info word arrives with the record (a branch let
          // hipcc sink its LDS read into the kept path: one more dependent round trip per member)
          const bool vis = wq_member_visit<NodeR>(N0, N1, N2, rq, t_hi, tnear) & valid;
          const bool leaf = (inf >> 27) != 0u;
          li[k] = (vis & leaf) ? inf : 0u;
          pe[k] = (vis & !leaf) ? ((inf << 6) | r) : ~0u;
          pk[k] = (vis & !leaf) ? -tnear : -kFltMax;
#else
          if (wq_member_visit<NodeR>(N0, N1, N2, rq, t_hi, tnear) & valid) {
            if (inf >> 27) {
              li[k] = inf;
            } else {
              pe[k] = (inf << 6) | r;
              pk[k] = -tnear;
            }
          }
#endif
        };
        // members two at a time, both records read up front (six LDS reads in flight); every group
        // has >= 2 members, and an odd count reads its last member twice and keeps one
#if HRT_WQ_ALL4
        // (A/B) every slot tested, the ones past the group's count masked (no per-pair branch)
#pragma unroll
        for (int h = 0; h < (int)kWqSlots / 2; ++h) {
#if HRT_WQ_EARLY_REC
          if (h == 0) {
            member(A00, A01, A02, 0);
            member(B00, B01, B02, 1);
            continue;
          }
#endif
          const float4* na = wq.nodes + 3 * (fc + min(2u * h, gcnt - 1u));
          const float4* nb = wq.nodes + 3 * (fc + min(2u * h + 1u, gcnt - 1u));
          const float4 A0 = na[0], A1 = na[1], A2 = na[2], B0 = nb[0], B1 = nb[1], B2 = nb[2];
          member(A0, A1, A2, 2 * h, h == 0 || 2u * h < gcnt);
          member(B0, B1, B2, 2 * h + 1, h == 0 || 2u * h + 1u < gcnt);
        }
#else
#pragma unroll
        for (int h = 0; h < (int)kWqSlots / 2; ++h) {
          if (h == 0 || 2u * h < gcnt) {
            const float4* na = wq.nodes + 3 * (fc + 2u * h);
            const float4* nb = wq.nodes + 3 * (fc + min(2u * h + 1u, gcnt - 1u));
            const float4 A0 = na[0], A1 = na[1], A2 = na[2], B0 = nb[0], B1 = nb[1], B2 = nb[2];
            member(A0, A1, A2, 2 * h);
            if (h == 0 || 2u * h + 1u < gcnt) member(B0, B1, B2, 2 * h + 1);
          }
        }
#endif
        // the nearest member in the last slot (pushed last = popped first)
#pragma unroll
        for (int st = 1; st < (int)kWqSlots; st *= 2)
#pragma unroll
          for (int k = st - 1; k + st < (int)kWqSlots; k += 2 * st) wq_order(pk[k], pe[k], pk[k + st], pe[k + st]);
      } else {  // finish the group's subtrees with a stackless walk (escape links)
        const uint32_t end = wq_escape(wq.nodes, fc + gcnt - 1u);
        uint32_t cur = fc;
        while (cur != end) {
          const uint32_t inf = wq_info(wq.nodes, cur), cnt = inf >> 27;
          float tnear;
          const float t_hi = wq_slot_t(wq, r) * (1.0f + rel_t) + rabs;
          const bool v = wq_node_visit(wq.nodes + 3 * cur, ro, rd, rinv, rR, rabs, t_hi, tnear);
          if (v && cnt) {
            const uint32_t first = inf & 0x07FFFFFFu;
            for (uint32_t k = first; k < first + cnt; ++k) wq_leaf_prim(prims, wq, k, r, rm, ro, rd);
          }
          cur = (v && !cnt) ? (inf & 0xFFFFu) : wq_escape(wq.nodes, cur);  // inner: its first child
        }
      }
    }
    // kept inner members: slot-major (every lane's slot 0, then slot 1, ...; the ordering may have
    // moved a member to any slot)
    wave_handoff();  // this step's pops before the pushes that reuse their words
#pragma unroll
    for (int k = 0; k < (int)kWqSlots; ++k) {
      const bool push = pe[k] != ~0u;
      const unsigned long long bk = __ballot(push);
#if HRT_WQ_PUSH_DUMP
      // every lane stores (no branch): the others into the stack's last word, which no entry reaches
      // (the overflow test keeps nc + width nn below ncap)
      lds_put(&wq.ns[push ? nc + lanes_below(bk) : wq.ncap - 1u], pe[k]);
#else
      if (push) lds_put(&wq.ns[nc + lanes_below(bk)], pe[k]);
#endif
      nc += (uint32_t)__popcll(bk);
    }
    // kept leaves' triangles: exclusive prefix of the per-lane counts (0..16)
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < (int)kWqSlots; ++k) cnt += li[k] >> 27;
    uint32_t tot;
    const uint32_t pre = wave_scan_excl(cnt, tot, 5u);
    if (tc + tot <= tcap) {  // wave-uniform
      uint32_t at = tc + pre;
#if HRT_WQ_LEAF_FLAT
      // one loop over the lane's kept triangles (slot of entry j by its running start, selects),
      // instead of a loop per slot
      const uint32_t c0 = li[0] >> 27, c1 = li[1] >> 27, c2 = li[2] >> 27;
      const uint32_t s1 = c0, s2 = s1 + c1, s3 = s2 + c2;
      const uint32_t f0 = li[0] & 0x07FFFFFFu, f1 = (li[1] & 0x07FFFFFFu) - s1, f2 = (li[2] & 0x07FFFFFFu) - s2,
                     f3 = (li[3] & 0x07FFFFFFu) - s3;
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t f = j >= s3 ? f3 : j >= s2 ? f2 : j >= s1 ? f1 : f0;
        lds_put(&wq.ts[at + j], ((f + j) << 6) | r);
      }
#else
#pragma unroll
      for (int k = 0; k < (int)kWqSlots; ++k) {
        const uint32_t c = li[k] >> 27, first = li[k] & 0x07FFFFFFu;
        for (uint32_t j = 0; j < c; ++j) lds_put(&wq.ts[at + j], ((first + j) << 6) | r);
        at += c;
      }
#endif
      tc += tot;
    } else {  // a burst of kept leaves beyond the triangle stack: each lane tests its own in place
#pragma unroll
      for (int k = 0; k < (int)kWqSlots; ++k) {
        const uint32_t c = li[k] >> 27, first = li[k] & 0x07FFFFFFu;
        for (uint32_t j = 0; j < c; ++j) wq_leaf_prim(prims, wq, first + j, r, rm, ro, rd);
      }
    }
  }
  wave_handoff();  // every lowering before the owners' reads
  if (sec) {
    const unsigned long long s = lds_get(&wq.slot[lane]);
    const uint32_t id = (uint32_t)s;
    if (id != 0u) c = Closest{__uint_as_float((uint32_t)(s >> 32)), 2, (id - 1u) & 0x03FFFFFFu, (id - 1u) >> 26};
  }
  if (D && P.diag) {  // wave totals, held by lane 0 (the tile record sums lanes)
    if (lane == 0) {
      dg.bvh_visits += node_pairs;
      dg.bvh_prims += tri_pairs;
      dg.bvh_trips += steps;
    }
    dg.bvh_band += band_tests;
    const uint32_t bm = wave_max_u(band_lmax);
    if (lane == 0) dg.band_max += bm;
  }
}

// Fused loop of BUNDLE / BUNDLE_CULL / BUNDLE_BVH.  Every lane stays in the loop until the whole wave is done, so
// the loop top is a full-wave region (lane-parallel culls and shuffles need all 64 lanes).  Primary
// segments take the bundle path; a lane whose next segment is a bounce waits (state untouched) until
// at least sec_batch lanes wait or no primary segment is left in the wave, then all waiting lanes run
// their bounce segment together.  Per-pixel order of work (and so every result) is unchanged.

// Sky items.  A wave whose primary list is empty (tl.ok, tl.n == 0) in a scene without spheres tests
// nothing in world_hit_tile, so each primary segment of its lanes is a miss: raytracing.glsl:318-346's
// miss branch (environment light, path ends, no RNG draw after get_ray_dir) and the lane's next sample
// starts at once.  The fused loop then spends its whole trip on bookkeeping (ballots, the bounce-batch
// vote, the list loop's set-up, shade_step's branches) around one ray generation.  sky_samples runs the
// lanes' num_samples such segments as a plain loop instead, two samples per trip (once each sample's
// three hashes are drawn, their ray generations are independent), with the fused loop's per-pixel
// arithmetic in the same order: the same colour, RNG state, segment and test counts.
#ifndef HRT_SKY_LOOP
#define HRT_SKY_LOOP 1
#endif
#ifndef HRT_SKY_UNROLL
#define HRT_SKY_UNROLL 1  // samples per trip of the sky loop (r04i/j: 1 beats 2 by ~1% on island; 3, 4 no better)
#endif
template <bool Zero>
__device__ __forceinline__ void sky_segment(const KArgs K, const TileList& tl, bool active, f3 centre, uint32_t& state,
                                            f3& colour, uint32_t& tests) {
  const auto& pc = K->pc;
  const f3 dir = get_ray_dir_sky<Zero>(pc, centre, state);
  // unit: the wave's second normalize took its fast path, so |d.c| <= 1 + 2^-23 in every lane (normalize_wu)
  bool unit = false;
  const f3 d = HRT_NORM_UNIFORM ? normalize_wu(dir, unit) : normalize(dir);
  // world_hit_tile's test count: the octant table (one lane read, all 64 lanes run this), or the
  // literal AABB test off its domain (|d.c| <= 1.5: implied by unit)
  // (the octant's byte address for ds_bpermute directly: __shfl added the lane's 64-lane segment base)
  const uint32_t oct4 = ((fbits(d.x) >> 31) << 2) | ((fbits(d.y) >> 31) << 3) | ((fbits(d.z) >> 31) << 4);
  const uint32_t oct_tests = (uint32_t)__builtin_amdgcn_ds_bpermute((int)oct4, (int)tl.tsum);
  if (__builtin_expect(tl.aabb_ok && (unit || (fabsf(d.x) <= 1.5f && fabsf(d.y) <= 1.5f && fabsf(d.z) <= 1.5f)), 1)) {
    tests += oct_tests;
  } else if (active) {
    const f3 o = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
    for (int m = 0; m < pc.num_meshes; ++m)
      if (aabb_pass(K->meshes[m], o, d)) tests += K->meshes[m].len;
  }
  // shade_step's miss (p.light = 0 + environment light) and the caller's colour += light * (1, 1, 1).
  // With |d.y| <= 1 + 2^-23 each light component is (1 - a) + a k with a = (d.y + 1) / 2 in
  // [-2^-24, 1 + 2^-24] and k in [0.5, 1]: at least 0.5 - 2^-23, never a zero, so 0 + light == light
  // (and without the environment light it is +0 either way).
  f3 light = environment_light(pc, d);
  if (!unit) light = mk(0.0f, 0.0f, 0.0f) + light;
  colour = colour + light * mk(1.0f, 1.0f, 1.0f);
}
// The lanes' whole pixels.  ALL 64 lanes run it (wave-uniform condition; the idle lanes' results are
// dropped); tl holds the wave's octant table.
__device__ __forceinline__ void sky_samples(const TileList& tl, bool active, f3 centre, uint32_t& state, f3& colour,
                                            uint32_t& segs, uint32_t& tests) {
  const KArgs K = kargs();
  const int ns = K->pc.num_samples;
  uint32_t t = 0;
  int s = 0;
  if (HRT_SKY_ZERO && fabsf(K->pc.jitter_size) < __builtin_inff() &&
      __all(!active || (centre.x != 0.0f && centre.y != 0.0f && fabsf(centre.x) < __builtin_inff() &&
                        fabsf(centre.y) < __builtin_inff()))) {  // get_ray_dir_sky<true>'s premises
    for (; s + HRT_SKY_UNROLL <= ns; s += HRT_SKY_UNROLL) {
#pragma unroll
      for (int u = 0; u < HRT_SKY_UNROLL; ++u) sky_segment<true>(K, tl, active, centre, state, colour, t);
    }
    for (; s < ns; ++s) sky_segment<true>(K, tl, active, centre, state, colour, t);
  } else {
    for (; s + HRT_SKY_UNROLL <= ns; s += HRT_SKY_UNROLL) {
#pragma unroll
      for (int u = 0; u < HRT_SKY_UNROLL; ++u) sky_segment<false>(K, tl, active, centre, state, colour, t);
    }
    for (; s < ns; ++s) sky_segment<false>(K, tl, active, centre, state, colour, t);
  }
  if (active) {
    segs += ns > 0 ? (uint32_t)ns : 0u;
    tests += t;
  }
}

// Issue priorities (s_setprio): heavy items' waves run at 3 (tile_loop), a light item's wave at 0 and
// at HRT_BOUNCE_PRIO during its bounce traversals -- the dependent LDS / L2 chains go first and the
// other waves' ALU work fills in behind them (r04z: cave 5.508 -> 5.433 ms per frame, island unchanged;
// light items at 1 or 2 with sky waves at 0, or bounce priority 2 or 3, no better;
// profiles/r04/r04z*_ab_*.jsonl)
#ifndef HRT_BOUNCE_PRIO
#define HRT_BOUNCE_PRIO 1
#endif
// kBounceWqR: BUNDLE_WQ with node margins from each member's own R (HRT_OPT_WQ_NODE_RADIUS = 2)
enum BounceMode { kBounceBrute = 0, kBounceCull = 1, kBounceBvh = 2, kBounceWq = 3, kBounceWqR = 4 };
constexpr bool is_wq(int b) { return b == kBounceWq || b == kBounceWqR; }

#ifndef HRT_PIXEL_POOL
#define HRT_PIXEL_POOL 1
#endif
template <int Bounce, bool D, class CullSrc, class BvhSrc = BvhGlobal>
__device__ __forceinline__ void trace_fused_split(const TraceParams& P, uint32_t x, uint32_t lr, const CullSrc& csrc,
                                                  const BvhSrc& bsrc, uint32_t* list_lds, Coop& co,
                                                  uint32_t frame = 0, uint32_t nrun = 1) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes, P.tri_nhat};
  const hrt_push_constants& pc = P.pc;
  const GlobalTris src{reinterpret_cast<const float4*>(P.tris)};
  uint32_t y = global_row(lr, P);
  uint32_t segs = 0, tests = 0;
  const bool active = x < pc.width && lr < kargs()->local_rows && y < pc.height;
  uint32_t id = active ? x + y * pc.width : 0u;
  const uint64_t tile_t0 = (D && P.tile_cycles) ? __builtin_readcyclecounter() : 0;
  f3 colour = mk(0.0f, 0.0f, 0.0f);
  uint32_t state = (pc.rng_offset + frame) * 719393u + id;  // raytracing.glsl:376, frame f of the launch
  f3 centre = mk(0.0f, 0.0f, 0.0f);
  if (active) {
    const float4 rc = kargs()->rays[id];
    centre = mk(rc.x, rc.y, rc.z);
  }
#if !HRT_RAYGEN_KARGS
  const f3 root = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
#endif
#if HRT_TL_PREPASS
  // a whole tile's item: the list the launch's tile_lists kernel built for the tile (the same function of
  // the same inputs -- camera, the tile's ray centres, the camera lists -- as building it here, which the
  // launch's other frames of the tile would repeat; r05c timelines: ~11 us of dependent L2 round trips
  // per item, 6 wave-us per tile-frame on island, 13 on a rank of 8)
  TileList tl;
  if (co.cache_tile != 0xFFFFFFFFu && !list_lds) {
    const uint32_t* rec = kargs()->tl_cache + (size_t)co.cache_tile * kTlRecWords;
    const uint32_t lane = threadIdx.x & 63;
    tl.v = rec[lane];
    tl.tsum = rec[64 + lane];
    tl.lds = nullptr;
    tl.n = __builtin_amdgcn_readfirstlane(rec[128]);
    tl.ok = __builtin_amdgcn_readfirstlane(rec[129]) != 0u;
    tl.aabb = (unsigned long long)__builtin_amdgcn_readfirstlane(rec[130]) |
              ((unsigned long long)__builtin_amdgcn_readfirstlane(rec[131]) << 32);
    tl.aabb_ok = __builtin_amdgcn_readfirstlane(rec[132]) != 0u;
  } else {
    tl = build_tile_list(P, active, centre, list_lds);
  }
#else
  const TileList tl = build_tile_list(P, active, centre, list_lds);
#endif
#if HRT_TIMELINE
  co.t_setup = __builtin_amdgcn_s_memrealtime();
  co.t_sky = tl.ok && tl.n == 0u && pc.num_spheres == 0;
#endif
  // bounce batch threshold scaled to the item's active lanes (a split tile's row group has 8/k rows):
  // a batch of few lanes then runs alongside the other lanes' primary segments instead of after them
  const uint32_t sec_thresh = max(1u, (kargs()->sec_batch * (uint32_t)__popcll(__ballot(active)) + 63u) / 64u);
  int sample = 0;
  Path p;
  p.bounce = pc.max_bounces + 1;
  bool done = !active;
  Diag dg;
  // Frame runs (tile_loop): the item's frames frame .. frame + nrun - 1 of a multi-frame launch, one
  // after the other per lane -- a lane that finishes its pixel in one frame starts the pixel's next
  // frame (rng_offset + f, its own image) at once instead of idling until the wave's slowest lane ends.
  uint32_t fr = 0;
  // Pixel pool (HRT_PIXEL_POOL, a whole tile's frame run with every lane active): the run's 64 x nrun
  // pixel-frames are one pool, frame-major, and a lane that finishes a pixel-frame takes the pool's next
  // one -- any pixel of the tile, not only its own pixel's next frame -- so the wave ends one pixel-frame
  // after the pool empties instead of after its slowest pixel's nrun frames.  A pixel-frame's work is
  // the same whichever lane runs it (its RNG seed, centre, samples in order, its own image), so every
  // frame is unchanged.  A lane that takes another pixel reloads its ray centre (a line the item's
  // start brought into the cache); fr = nrun once the pool is empty and the lane's last pixel-frame is
  // stored.
  const bool pool = HRT_PIXEL_POOL && nrun > 1u && __all(active);
  uint32_t pool_next = 64u;  // (wave-uniform)
  if (HRT_SKY_LOOP && tl.ok && tl.n == 0u && pc.num_spheres == 0) {  // wave-uniform: every segment a miss
    const uint64_t s0 = (D && P.diag) ? __builtin_readcyclecounter() : 0;
    for (;; ++fr) {
      sky_samples(tl, active, centre, state, colour, segs, tests);
      if (fr + 1u >= nrun) break;
      if (active) store_pixel(P, x, lr, div3(colour, (float)pc.num_samples), frame + fr);
      colour = mk(0.0f, 0.0f, 0.0f);
      state = (pc.rng_offset + frame + fr + 1u) * 719393u + id;
    }
    const uint32_t ns = pc.num_samples > 0 ? (uint32_t)pc.num_samples : 0u;
    if (co.w == 0) co.work += (2u + 3u * ns) * nrun;  // the fused loop's work units for these trips
    if (D && P.diag) {
      dg.prim_iters += ns * nrun;
      dg.sky_items += nrun;
      dg.cyc_sky += __builtin_readcyclecounter() - s0;
    }
    done = true;
  }
  while (__any(!done)) {
    // (a loop: with num_samples <= 0 a new pixel-frame ends at once too, and each must still be stored)
    while (pool) {
      const bool need = !done && p.bounce > pc.max_bounces && sample >= pc.num_samples;
      const unsigned long long nb = __ballot(need);
      if (!nb) break;
      {
        if (need) store_pixel(P, x, lr, div3(colour, (float)pc.num_samples), frame + fr);
        const uint32_t idx = pool_next + lanes_below(nb);
        pool_next += (uint32_t)__popcll(nb);
        if (need) {
          if (idx < 64u * nrun) {
            const uint32_t px = idx & 63u;
            fr = idx >> 6;
            x = (x & ~7u) + (px & 7u);
            lr = (lr & ~7u) + (px >> 3);
            y = global_row(lr, P);
            id = x + y * pc.width;
            const float4 rc = kargs()->rays[id];
            centre = mk(rc.x, rc.y, rc.z);
            colour = mk(0.0f, 0.0f, 0.0f);
            sample = 0;
            state = (pc.rng_offset + frame + fr) * 719393u + id;
          } else {
            done = true;
            fr = nrun;
          }
        }
      }
    }
    if (!done && p.bounce > pc.max_bounces) {
      // (a while: with num_samples <= 0 every frame of the run ends at once and each must still be stored)
      while (!pool && sample >= pc.num_samples && fr + 1u < nrun) {  // the pixel's next frame of the run
        store_pixel(P, x, lr, div3(colour, (float)pc.num_samples), frame + fr);
        ++fr;
        colour = mk(0.0f, 0.0f, 0.0f);
        sample = 0;
        state = (pc.rng_offset + frame + fr) * 719393u + id;
      }
      if (sample >= pc.num_samples) {
        done = true;
      } else {
        ++sample;
#if HRT_RAYGEN_KARGS
        // the camera (matrix, jitter, position) read at the sample's start (kargs): 13 values not held
        // in SGPRs across the loop
        const KArgs K = kargs();
        const f3 dir = get_ray_dir(K->pc, centre, state);
        p = Path{mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), mk(K->pc.cam_pos[0], K->pc.cam_pos[1], K->pc.cam_pos[2]),
                 normalize_fl(dir), 0, true};
#else
        const f3 dir = get_ray_dir(pc, centre, state);
        p = Path{mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), root, normalize_fl(dir), 0, true};
#endif
      }
    }
    const bool ready = !done && p.bounce == 0;  // a primary segment to run
    const bool waiting = !done && p.bounce != 0;
    const uint32_t nwait = (uint32_t)__popcll(__ballot(waiting));
    // (r04d, measured and dropped: primary segments waiting too while a bounce batch runs and fewer than
    // 8 lanes have one -- island 1.859 -> 1.878 ms)
    const bool prim = ready;
    const bool any_prim = __any(prim);
    const bool run_sec = nwait > 0 && (nwait >= sec_thresh || !any_prim);
    const bool sec = waiting && run_sec;
    Closest c{kFltMax, 0, 0u, 0u};
    uint64_t t0 = 0, t1 = 0, t2 = 0;
    if (D && P.diag) {
      dg.prim_iters += any_prim ? 1u : 0u;
      dg.sec_iters += run_sec ? 1u : 0u;
      dg.sec_lanes += run_sec ? nwait : 0u;
      dg.prim_lanes += (uint32_t)__popcll(__ballot(prim));
      dg.loop_iters += 1u;
      dg.live_lanes += (uint32_t)__popcll(__ballot(!done));
      t0 = __builtin_readcyclecounter();
    }
    if (co.w == 0) co.work += 2u + (any_prim ? 1u + (tl.ok ? tl.n : 64u) : 0u);  // shading, primary list
    if (any_prim) {
      if (tl.ok) {
        const uint32_t tested = world_hit_tile(HRT_SHADE_KARGS ? kscene() : sc, P, tl, prim, p.pos, p.dir, tests, c);
        if (D && P.diag) {
          dg.prim_considered += tl.n;
          dg.prim_survivors += tested;
        }
      } else {
        world_hit_bundle<D>(sc, P, prim, p.pos, p.dir, tests, c, dg);
      }
    }
    if (D && P.diag) t1 = __builtin_readcyclecounter();
    if (run_sec) {
      if (HRT_BOUNCE_PRIO && !co.hot) __builtin_amdgcn_s_setprio(HRT_BOUNCE_PRIO);
      if constexpr (is_wq(Bounce)) {
        world_hit_bounce_wq<D, Bounce == kBounceWqR>(HRT_SHADE_KARGS ? kscene() : sc, P, bsrc, sec, p.pos, p.dir, tests,
                                                     c, dg);
      } else if constexpr (Bounce == kBounceBvh) {
        world_hit_bounce_bvh<D>(sc, P, bsrc, sec, p.pos, p.dir, tests, c, dg);
      } else if constexpr (Bounce == kBounceCull) {
        world_hit_bounce_cull<D>(sc, P, csrc, sec, p.pos, p.dir, tests, c, dg, co);
      } else {
        if (sec) c = world_hit_brute(sc, src, pc, p.pos, p.dir, tests);
      }
    }
    if (HRT_BOUNCE_PRIO && run_sec && !co.hot) __builtin_amdgcn_s_setprio(0);
    if (D && P.diag) t2 = __builtin_readcyclecounter();
    if (prim || sec) {
      ++segs;
      const bool ended = shade_step(HRT_SHADE_KARGS ? kscene() : sc, pc, p, c, state);
      ++p.bounce;
      if (ended || p.bounce > pc.max_bounces) {
        colour = colour + p.light * p.colour;
        p.bounce = pc.max_bounces + 1;
      }
    }
    if (D && P.diag) {
      const uint64_t t3 = __builtin_readcyclecounter();
      dg.cyc_prim += t1 - t0;
      dg.cyc_sec += t2 - t1;
      dg.cyc_shade += t3 - t2;
    }
  }
  if (co.w != 0) return;  // cooperative tile: wave 0 of the group writes the results
  if (active && fr < nrun) {
    colour = div3(colour, (float)pc.num_samples);
    store_pixel(P, x, lr, colour, frame + fr);
  }
  if (co.defer) {
    unsigned long long s, t;
    uint32_t mx;
    wave_counters(segs, tests, s, t, mx);
    co.acc_s += s;
    co.acc_t += t;
    co.acc_m += mx;
  } else {
    flush_counters(P, segs, tests);
  }
  if (D && P.tile_cycles && (threadIdx.x & 63) == 0) {  // lane 0 sits at the tile's (0, 0)
    const uint32_t tiles_x = (pc.width + 7) / 8;
    unsigned long long* rec = P.tile_cycles + 4 * ((lr / 8) * tiles_x + x / 8);
    atomicMax(&rec[0], (unsigned long long)(__builtin_readcyclecounter() - tile_t0));  // slowest item of a split tile
    // bounce batches | (BUNDLE_WQ) pair steps << 32
    atomicAdd(&rec[1], (unsigned long long)dg.sec_iters |
                           (is_wq(Bounce) ? (unsigned long long)dg.bvh_trips << 32 : 0ull));
    if (Bounce != kBounceBvh && !is_wq(Bounce)) atomicAdd(&rec[2], (unsigned long long)dg.sec_survivors);
    atomicAdd(&rec[3], (unsigned long long)dg.cyc_sec);
  }
  if (D && P.tile_cycles && (Bounce == kBounceBvh || is_wq(Bounce)) && active) {
    // BUNDLE_BVH: the tile's per-lane node visits, summed | (leaf + band triangle tests) << 32
    const uint32_t tiles_x = (pc.width + 7) / 8;
    atomicAdd(P.tile_cycles + 4 * ((lr / 8) * tiles_x + x / 8) + 2,
              (unsigned long long)dg.bvh_visits + ((unsigned long long)(dg.bvh_prims + dg.bvh_band) << 32));
  }
  if (D && P.diag && (threadIdx.x & 63) == 0) {
    atomicAdd(&P.diag[10], (unsigned long long)dg.cyc_prim);
    atomicAdd(&P.diag[11], (unsigned long long)dg.cyc_sec);
    atomicAdd(&P.diag[12], (unsigned long long)dg.cyc_shade);
    atomicAdd(&P.diag[13], (unsigned long long)dg.sec_stage2);
    atomicAdd(&P.diag[14], (unsigned long long)dg.sec_front);
    atomicAdd(&P.diag[15], (unsigned long long)dg.bvh_trips);
    atomicAdd(&P.diag[16], (unsigned long long)dg.bvh_leaf_trips);
    atomicAdd(&P.diag[17], (unsigned long long)dg.band_max);
    atomicAdd(&P.diag[0], (unsigned long long)dg.prim_iters);
    atomicAdd(&P.diag[1], (unsigned long long)dg.prim_considered);
    atomicAdd(&P.diag[2], (unsigned long long)dg.prim_survivors);
    atomicAdd(&P.diag[3], (unsigned long long)dg.sec_iters);
    atomicAdd(&P.diag[4], (unsigned long long)dg.sec_considered);
    atomicAdd(&P.diag[5], (unsigned long long)dg.sec_survivors);
    atomicAdd(&P.diag[6], (unsigned long long)dg.sec_lanes);
    if (dg.sky_items) {
      atomicAdd(&P.diag[19], (unsigned long long)dg.sky_items);
      atomicAdd(&P.diag[20], (unsigned long long)dg.cyc_sky);
    }
    atomicAdd(&P.diag[21], (unsigned long long)dg.prim_lanes);
    atomicAdd(&P.diag[22], (unsigned long long)dg.loop_iters);
    atomicAdd(&P.diag[23], (unsigned long long)dg.live_lanes);
    if (is_wq(Bounce)) {
#pragma unroll
      for (int b = 0; b < 4; ++b) atomicAdd(&P.diag[24 + b], (unsigned long long)dg.wq_fill[b]);
    }
  }
  if (D && P.diag && is_wq(Bounce) && dg.wq_members) atomicAdd(&P.diag[28], (unsigned long long)dg.wq_members);
  if (D && P.diag && (Bounce == kBounceBvh || is_wq(Bounce))) {
    atomicAdd(&P.diag[7], (unsigned long long)dg.bvh_visits);
    atomicAdd(&P.diag[8], (unsigned long long)dg.bvh_prims);
    atomicAdd(&P.diag[9], (unsigned long long)dg.bvh_band);
    atomicAdd(&P.diag[18], (unsigned long long)dg.band_len);
  }
}

template <bool D>
__global__ __launch_bounds__(256) void trace_bundle(TraceParams P) {
  __shared__ uint32_t lists[4 * kTileCapLds];
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  const float4* T = reinterpret_cast<const float4*>(P.tris);
  Coop solo{0u, 1u, nullptr, 0u, 0u};
  trace_fused_split<kBounceBrute, D>(P, x, lr, CullGlobal{T, to_const(T)}, BvhGlobal{},
                                     lists + (threadIdx.x >> 6) * kTileCapLds, solo);
}

#ifndef HRT_CULL_WAVES
#define HRT_CULL_WAVES 1
#endif
template <bool D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HRT_CULL_WAVES))) void trace_bundle_cull(
    TraceParams P) {
  __shared__ uint32_t lists[4 * kTileCapLds];
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  const float4* T = reinterpret_cast<const float4*>(P.tris);
  Coop solo{0u, 1u, nullptr, 0u, 0u};
  trace_fused_split<kBounceCull, D>(P, x, lr, CullGlobal{T, to_const(T)}, BvhGlobal{},
                                    lists + (threadIdx.x >> 6) * kTileCapLds, solo);
}

template <bool D>
__global__ __launch_bounds__(256) void trace_bundle_bvh(TraceParams P) {
  __shared__ uint32_t lists[4 * kTileCapLds];
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  const float4* T = reinterpret_cast<const float4*>(P.tris);
  Coop solo{0u, 1u, nullptr, 0u, 0u};
  trace_fused_split<kBounceBvh, D>(P, x, lr, CullGlobal{T, to_const(T)}, BvhGlobal{P.bvh_nodes, P.bvh_prims},
                                   lists + (threadIdx.x >> 6) * kTileCapLds, solo);
}


// Stage the triangle buffer into LDS in the BRUTE_LDS image (3 float4 per triangle).
__device__ __forceinline__ void stage_tris(const TraceParams& P, float4* dst, uint32_t block) {
  const uint32_t n = P.n_tris;
  for (uint32_t k = threadIdx.x; k < 3 * n; k += block) {
    const uint32_t i = k / 3, part = k - 3 * i;
    const hrt_triangle& t = P.tris[i];
    float4 v;
    if (part == 0) v = make_float4(t.a[0], t.a[1], t.a[2], t.normal[0]);
    else if (part == 1) v = make_float4(t.normal[1], t.normal[2], t.edge_one[0], t.edge_one[1]);
    else v = make_float4(t.edge_one[2], t.edge_two[0], t.edge_two[1], t.edge_two[2]);
    dst[k] = v;
  }
}

// Persistent tile loop of the LDS-resident variants: the workgroups stay resident (one or two per CU,
// the scene staged once) and each wave takes 8x8 pixel tiles from a global counter until the image
// is done, so no wave idles while a slower wave of its workgroup finishes.  Every wave leaves the
// loop once the counter passes the tile count.
//
// Work items (P.items, built by plan_fill from the previous trace's per-tile costs): tile | log2 K << 22
// | s << 25 | heavy << 31.  K == 1 is a whole tile; otherwise item s (0..K-1) covers the tile's pixels
// [s * 64/K, (s+1) * 64/K) in row-major order with 64/K lanes (the rest idle); K (2..64) grows with
// the tile's cost.  A heavy tile's pixels run as K shorter sample chains in parallel
// with lighter batches, and the planner puts them first.  Every pixel is computed exactly once and
// independently of which wave runs it, so the bytes do not depend on the plan.  Each item's cost goes
// to P.tile_cost[tile] for the next plan: deterministic work units (Coop::work: survivor tests,
// culled chunks, primary list entries, iterations; the same with or without cooperation) in
// BUNDLE_CULL_LDS, shader clocks / 16 in BUNDLE_BVH_LDS.
constexpr uint32_t kItemTileMask = (1u << 22) - 1u;  // planned traces need fewer than 2^22 tiles
template <int BLOCK, bool CoopOk, class Body>
__device__ __forceinline__ void tile_loop(const TraceParams& P, unsigned long long* ex, uint32_t* s_item, Body&& body) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tiles_x = (P.pc.width + 7) / 8, tiles = tiles_x * ((P.local_rows + 7) / 8);
  // A launch of nf frames runs every item once per frame: work index t is item t / nf of frame t % nf,
  // so each item's frames follow each other and the plan's longest-first order holds across frames.
  const uint32_t nf = P.n_frames > 1 ? P.n_frames : 1u;
  const uint32_t n = (P.items ? P.sched[1] : tiles) * nf;
  uint32_t first = 0;
  // Phase 1 (a plan with cooperative heavy tiles): the workgroup takes the heavy items [0, H) one
  // at a time, all its waves on the same tile (Coop).  The item index goes through LDS; at the loop
  // head each wave's lane 0 publishes its share of the previous tile's work units.
  if (CoopOk && P.items && P.coop) {
    const uint32_t H = P.sched[2] * nf;
    first = H;
    Coop co{threadIdx.x >> 6, (uint32_t)BLOCK / 64, ex, 0u, 0u};
    uint32_t prev_tile = 0xFFFFFFFFu, prev_cost = 0;
    for (;;) {
      if (lane == 0) {
        if (prev_tile != 0xFFFFFFFFu) {
          atomicAdd(&P.tile_cost[prev_tile], prev_cost);
          atomicAdd(reinterpret_cast<unsigned long long*>(P.sched + 6), (unsigned long long)prev_cost);
        }
        if (threadIdx.x == 0) *s_item = atomicAdd(&P.sched[5], 1u);
      }
      __syncthreads();
      const uint32_t h = __builtin_amdgcn_readfirstlane(*s_item);
      __syncthreads();
      if (h >= H) break;
      const uint32_t hi = h / nf, hf = h - hi * nf;
      const uint32_t tile = __builtin_amdgcn_readfirstlane(P.items[hi]) & kItemTileMask;
      const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
      co.work = 0;
      body(tx * 8 + (lane & 7), ty * 8 + (lane >> 3), co, hf, 1u);
      prev_cost = __builtin_amdgcn_readfirstlane(co.work);
      prev_tile = tile;
    }
    if (lane == 0 && prev_tile != 0xFFFFFFFFu) {
      atomicAdd(&P.tile_cost[prev_tile], prev_cost);
      atomicAdd(reinterpret_cast<unsigned long long*>(P.sched + 6), (unsigned long long)prev_cost);
    }
  }
  // Phase 2: every wave on its own.  The loop's only lane-divergent block is at its head (lane 0
  // publishes the previous item's cost and takes the next item).  A second lane-0 block at the latch
  // let the compiler thread lanes 1-63 straight back to the body past the head, where they spun on
  // a stale item: keep it this way.
  Coop solo{0u, 1u, nullptr, 0u, 0u};
  solo.defer = true;
  uint32_t prev_tile = 0xFFFFFFFFu, prev_cost = 0, prev_lk = 0;
  // Items are taken kGrab at a time while far from the end (one same-address atomic per kGrab items;
  // the plan's longest-first order is kept, and the last HRT_GRAB_TAIL items per resident wave go singly).
  // The threshold sum of the planner (sched[6]) is summed per wave and added once.
#ifndef HRT_GRAB
#define HRT_GRAB 4u
#endif
#ifndef HRT_FRAME_RUN
#define HRT_FRAME_RUN 1
#endif
  constexpr uint32_t kGrab = HRT_GRAB;
#ifndef HRT_GRAB_TAIL
#define HRT_GRAB_TAIL 64u  // items per resident wave taken singly at the end (16 x the r01s grab of 4)
#endif
  const uint32_t resident = gridDim.x * (BLOCK / 64);
  uint32_t cur = first, end = first;
#ifndef HRT_GRAB_HEAVY
#define HRT_GRAB_HEAVY 0  // 1: heavy items grabbed kGrab at a time like the others (r03)
#endif
  const uint32_t heavy_end = (HRT_GRAB_HEAVY || !P.items) ? 0u : P.sched[4] * nf;
  unsigned long long cost_sum = 0;
  for (;;) {
    const bool refill = cur >= end;  // wave-uniform
    // (singly, too, while in the plan's heavy prefix: grabbed together, a heavy item's frames queue behind
    // each other on one wave -- HRT_GRAB_HEAVY)
    const uint32_t g = (kargs()->grab_always ||
                        ((uint64_t)cur + (uint64_t)HRT_GRAB_TAIL * resident < n && cur >= heavy_end)) ? kGrab : 1u;
    uint32_t t = 0;
    const KArgs K = kargs();  // (per work item: not held across the item's fused loop)
    if (lane == 0) {
      // a tile's cost: its items' summed clocks; the heavy threshold's sum counts an item by its
      // share of the tile's lanes (its work), so splitting does not raise the threshold (with summed
      // clocks there too, borderline tiles flipped between split and whole: 7.4 / 8.4 ms frames)
      if (prev_tile != 0xFFFFFFFFu) atomicAdd(&K->tile_cost[prev_tile], prev_cost);
      if (refill) t = first + atomicAdd(&K->sched[0], g);
    }
    if (prev_tile != 0xFFFFFFFFu) cost_sum += prev_cost >> prev_lk;
    if (refill) {
      cur = __builtin_amdgcn_readfirstlane(t);
      end = cur + g;
    }
    t = cur;
    if (t >= n) break;
    const uint32_t ti = t / nf, tf = t - ti * nf;
    const uint32_t* items = K->items;
    const uint32_t item = items ? __builtin_amdgcn_readfirstlane(items[ti]) : 0u;
    const uint32_t tile = items ? item & kItemTileMask : ti, lk = (item >> 22) & 7u, sub = (item >> 25) & 63u;
    const bool hot = item >> 31;  // heavy last time: issue priority over the light tiles' waves
    // The grabbed indices of a light item's next frames run as one body (frame runs, trace_fused_split).
    // A heavy item (split, or marked hot) takes its frames one at a time: its pixel chains are the
    // launch's longest, and a run of them in one wave would outlast the launch (runs of 8 frames for
    // every item: island 1.903 -> 2.208 ms per frame, profiles/r04/r04b_ab_island.jsonl).
#ifndef HRT_RUN_HEAVY
#define HRT_RUN_HEAVY 0
#endif
    const uint32_t run = (HRT_FRAME_RUN && (HRT_RUN_HEAVY || (!hot && lk == 0u))) ? min(min(end, n) - t, nf - tf) : 1u;
    cur += run;
    const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const uint32_t j = (sub << (6u - lk)) + lane;  // the tile pixel (row-major) of this lane
    uint32_t x = tx * 8 + (j & 7u), lr = ty * 8 + (j >> 3);
    if (lane >= (64u >> lk)) x = 0xFFFFFFFFu;  // idle lane of a split item
    const uint64_t t0 = __builtin_readcyclecounter();
#if HRT_TIMELINE
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (hot) __builtin_amdgcn_s_setprio(3);
    solo.hot = hot;
    solo.work = 0;
    solo.cache_tile = (HRT_TL_PREPASS && K->tl_cache && lk == 0u) ? tile : 0xFFFFFFFFu;
    body(x, lr, solo, tf, run);
    if (hot) __builtin_amdgcn_s_setprio(0);
#if HRT_TIMELINE
    if (P.timeline && lane == 0) {  // (timeline builds only: the product kernel has no such branch)
      const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
      const uint32_t slot = atomicAdd(P.timeline_count, 1u);
      if (slot < P.timeline_cap) {
        const uint32_t wave = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
        P.timeline[4 * (size_t)slot] = rt0;
        P.timeline[4 * (size_t)slot + 1] = solo.t_setup;
        P.timeline[4 * (size_t)slot + 2] = rt1;
        P.timeline[4 * (size_t)slot + 3] = (unsigned long long)(tile | (lk << 22) | (sub << 25) | ((uint32_t)hot << 31)) |
                                           ((unsigned long long)(tf & 0xFFu) << 32) |
                                           ((unsigned long long)(run & 0x7Fu) << 40) |
                                           ((unsigned long long)(solo.t_sky & 1u) << 47) |
                                           ((unsigned long long)(wave & 0xFFFFu) << 48);
      }
    }
#endif
    // cost: the work count where the body keeps one (BUNDLE_CULL_LDS), else shader clocks / 16
    const uint64_t c = CoopOk ? (uint64_t)solo.work : (__builtin_readcyclecounter() - t0) >> 4;
    prev_cost = __builtin_amdgcn_readfirstlane(c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c);
    prev_tile = tile;
    prev_lk = lk;
  }
  if (lane == 0 && prev_tile != 0xFFFFFFFFu) atomicAdd(&P.tile_cost[prev_tile], prev_cost);
  if (prev_tile != 0xFFFFFFFFu) cost_sum += prev_cost >> prev_lk;
  if (lane == 0 && cost_sum) atomicAdd(reinterpret_cast<unsigned long long*>(P.sched + 6), cost_sum);
  add_counters(P, solo.acc_s, solo.acc_t, solo.acc_m);
}

// Planner (after a trace of an LDS variant, before the next).  Items go in decreasing order of the
// tile's last cost (longest first: a long tile started late is what sets a frame's end), by a
// 64-bucket half-octave histogram and a descending scan; heavy tiles are the top buckets: cost >=
// factor x (sum of costs / resident waves), to the bucket, i.e. a tile that alone would take `factor`
// times a wave's fair share of the frame; each runs as 2, 4 or 8 items (bucket_items, <= split_k).  sched[8..71] histogram, [72..135] bucket offsets,
// [136..199] bucket cursors, [3] first heavy bucket.
#ifndef HRT_PLAN_SUB
// log2 of the planner's cost buckets per octave: eighth-octave buckets put a rank's long items nearer to
// their exact longest-first order (r06p: the slowest of ranks 3 and 6 -1.7% per run on island, -1.1% on
// cave; half-octave buckets left tiles up to 1.41x apart in arbitrary order)
#define HRT_PLAN_SUB 3
#endif
constexpr uint32_t kPlanSub = HRT_PLAN_SUB, kPlanBuckets = 32u << kPlanSub;
__device__ __forceinline__ uint32_t cost_bucket(unsigned long long c) {
  if (c < (2u << kPlanSub)) return (uint32_t)c;  // (floor(log2 c) <= kPlanSub: the value itself)
  if (c > 0xFFFFFFFFull) return kPlanBuckets;
  const uint32_t v = (uint32_t)c, l = 31 - __clz(v);  // floor(log2 c) > kPlanSub
  return min((l << kPlanSub) + ((v >> (l - kPlanSub)) & ((1u << kPlanSub) - 1u)), kPlanBuckets - 1);
}
// sched words: [8, 8 + B) histogram, [8 + B, 8 + 2B) bucket offsets, [8 + 2B, 8 + 3B) cursors
constexpr uint32_t kSchedHist = 8, kSchedOff = 8 + kPlanBuckets, kSchedCur = 8 + 2 * kPlanBuckets;
static_assert(kSchedCur + kPlanBuckets <= kSchedWords, "sched buffer");
// Both passes count in LDS first: a frame's tiles crowd a few buckets, and per-tile global atomics
// on those few words serialize (0.3 ms per pass at 1080p).
__global__ __launch_bounds__(256) void plan_hist(uint32_t* sched, const uint32_t* cost, uint32_t tiles) {
  __shared__ uint32_t h[kPlanBuckets];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (threadIdx.x < kPlanBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  if (i < tiles) atomicAdd(&h[cost_bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x < kPlanBuckets && h[threadIdx.x]) atomicAdd(&sched[kSchedHist + threadIdx.x], h[threadIdx.x]);
}
// Items of a heavy tile in bucket b >= hb: doubling per octave above the threshold (costs [1, 2) x
// threshold: 2 items, [2, 4): 4, ... up to 64 single pixels), at most kmax; kmax = 1: never split.
__device__ __forceinline__ uint32_t bucket_items(uint32_t b, uint32_t hb, uint32_t kmax) {
  return b < hb ? 1u : min(kmax, 2u << min((b - hb) >> kPlanSub, 5u));
}
// factor4: the heavy threshold in quarters of a resident wave's share of the launch's work
__global__ __launch_bounds__(64) void plan_scan(uint32_t* sched, uint32_t waves, uint32_t factor4, uint32_t kmax,
                                                uint32_t prio) {
  if (threadIdx.x != 0) return;
  const unsigned long long sum = *reinterpret_cast<const unsigned long long*>(sched + 6);
  const uint32_t hb = cost_bucket((unsigned long long)factor4 * sum / (4ull * (waves ? waves : 1u)));
  uint32_t pos = 0, heavy = 0, heavy_items = 0;
  for (int b = (int)kPlanBuckets - 1; b >= 0; --b) {
    const uint32_t cnt = sched[kSchedHist + b], hv = (uint32_t)b >= hb, k = bucket_items((uint32_t)b, hb, kmax);
    sched[kSchedOff + b] = pos;
    pos += cnt * k;
    heavy += hv ? cnt : 0u;
    heavy_items += hv ? cnt * k : 0u;
  }
  sched[1] = prio > 1 ? heavy_items : pos;  // prio 2: heavy items only (diagnostics)
  sched[2] = heavy;
  sched[4] = heavy_items;  // the plan's first heavy_items items are the heavy tiles' (tile_loop grabs them singly)
  sched[3] = hb;
}

// Item word: tile | log2(items of the tile) << 22 | item index s << 25 | heavy << 31 (tile_loop).
__global__ __launch_bounds__(256) void plan_fill(uint32_t* sched, const uint32_t* cost, uint32_t tiles, uint32_t kmax,
                                                 uint32_t prio, uint32_t* items) {
  __shared__ uint32_t cnt[kPlanBuckets], base[kPlanBuckets];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (threadIdx.x < kPlanBuckets) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t hb = sched[3];
  const uint32_t b = i < tiles ? cost_bucket(cost[i]) : 0u;
  const bool heavy = b >= hb;
  const uint32_t k = bucket_items(b, hb, kmax);
  const uint32_t local = i < tiles ? atomicAdd(&cnt[b], k) : 0u;
  __syncthreads();
  if (threadIdx.x < kPlanBuckets && cnt[threadIdx.x])
    base[threadIdx.x] = sched[kSchedOff + threadIdx.x] + atomicAdd(&sched[kSchedCur + threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (i >= tiles) return;
  const uint32_t at = base[b] + local;
  if (!heavy) {
    items[at] = i;
  } else {
    const uint32_t flag = prio ? 0x80000000u : 0u;
    if (k == 1) {
      items[at] = i | flag;
    } else {
      const uint32_t lk = (uint32_t)__builtin_ctz(k);
      for (uint32_t s = 0; s < k; ++s) items[at + s] = i | (lk << 22) | (s << 25) | flag;
    }
  }
}

// BUNDLE_CULL with the triangles resident in LDS (bounce survivors are read at LDS rather than L2
// latency).  Dynamic LDS: n_tris x 48 B triangles.
template <int BLOCK, bool D>
__global__ __launch_bounds__(BLOCK) void trace_bundle_cull_lds(TraceParams P) {
  __shared__ uint32_t s_item;
  stage_tris(P, lds_tris, BLOCK);
  // cooperative-tile exchange slots (Coop) after the triangle image, all clear
  unsigned long long* ex = reinterpret_cast<unsigned long long*>(lds_tris + 3 * P.n_tris);
  for (uint32_t k = threadIdx.x; k < 3 * 64; k += BLOCK) ex[k] = ~0ull;
  __syncthreads();
  tile_loop<BLOCK, true>(P, ex, &s_item, [&](uint32_t x, uint32_t lr, Coop& co, uint32_t f, uint32_t nr) {
    trace_fused_split<kBounceCull, D>(P, x, lr, CullLds{lds_tris}, BvhGlobal{}, nullptr, co, f, nr);
  });
}

// BUNDLE_WQ: the hierarchy's nodes in LDS, one pair-stack region per wave after them (persistent
// 1024-thread workgroups).  Dynamic LDS: [nodes x 48 B][16 x (64 slots x 8 B, wq_ncap + wq_tcap words)].
// (one body, two kernels: a __device__ wrapper taking P by reference changes the island kernel's
// register allocation and cost 0.6%)
#define HRT_WQ_KERNEL_BODY(BOUNCE)                                                                              \
  {                                                                                                             \
    const uint32_t nn = P.bvh_wq_n_nodes;                                                                       \
    float4* nodes = lds_tris;                                                                                   \
    for (uint32_t k = threadIdx.x; k < 3 * nn; k += 1024) nodes[k] = P.bvh_wq_nodes[k];                         \
    char* base =                                                                                                \
        reinterpret_cast<char*>(nodes + 3 * nn) + (size_t)(threadIdx.x >> 6) * (512 + 4 * (P.wq_ncap + P.wq_tcap)); \
    const WqLds wq{nodes, reinterpret_cast<unsigned long long*>(base), reinterpret_cast<uint32_t*>(base + 512),  \
                   reinterpret_cast<uint32_t*>(base + 512) + P.wq_ncap, P.wq_ncap};                            \
    __syncthreads();                                                                                            \
    const float4* T = reinterpret_cast<const float4*>(P.tris);                                                  \
    tile_loop<1024, false>(P, nullptr, nullptr, [&](uint32_t x, uint32_t lr, Coop& co, uint32_t f, uint32_t nr) { \
      trace_fused_split<BOUNCE, D>(P, x, lr, CullGlobal{T, to_const(T)}, wq, nullptr, co, f, nr);               \
    });                                                                                                         \
  }
template <bool D>
__global__ __launch_bounds__(1024) void trace_bundle_wq(TraceParams P) HRT_WQ_KERNEL_BODY(kBounceWq)
// the same with per-member R in the node margins (TraceParams::bvh_node_r, HRT_OPT_WQ_NODE_RADIUS)
template <bool D>
__global__ __launch_bounds__(1024) void trace_bundle_wq_nr(TraceParams P) HRT_WQ_KERNEL_BODY(kBounceWqR)
#undef HRT_WQ_KERNEL_BODY

// BUNDLE_BVH with the hierarchy and the triangle image in LDS (persistent 1024-thread workgroups).
// Dynamic LDS: [n_tris x 48 B triangles][nodes x 64 B][prims x 4 B entries][meshes x 4 B key bases].
template <bool D>
__global__ __launch_bounds__(1024) void trace_bundle_bvh_lds(TraceParams P) {
  const uint32_t n = P.n_tris, nn = P.bvh_n_nodes, np = P.bvh_n_prims, nm = P.bvh_n_meshes;
  stage_tris(P, lds_tris, 1024);
  float4* nodes = lds_tris + 3 * n;
  for (uint32_t k = threadIdx.x; k < 4 * nn; k += 1024) nodes[k] = P.bvh_nodes[k];
  uint32_t* entries = reinterpret_cast<uint32_t*>(nodes + 4 * nn);
  for (uint32_t k = threadIdx.x; k < np; k += 1024) entries[k] = P.bvh_entries[k];
  uint32_t* kbase = entries + np;
  for (uint32_t k = threadIdx.x; k < nm; k += 1024) kbase[k] = P.bvh_keybase[k];
  __syncthreads();
  const float4* T = reinterpret_cast<const float4*>(P.tris);
  tile_loop<1024, false>(P, nullptr, nullptr, [&](uint32_t x, uint32_t lr, Coop& co, uint32_t f, uint32_t nr) {
    trace_fused_split<kBounceBvh, D>(P, x, lr, CullGlobal{T, to_const(T)}, BvhLds{nodes, lds_tris, entries, kbase},
                                     nullptr, co, f, nr);
  });
}

// The persistent kernels' whole-tile lists (HRT_TL_PREPASS): one wave per 8x8 tile builds exactly what
// trace_fused_split's build_tile_list would for the tile's whole-tile items (the same pixels, the same
// function) and stores it in the tile's record; the launch's items of the tile then read it back (every
// frame of a multi-frame launch shares the camera and the camera lists).
__global__ __launch_bounds__(256) void tile_lists(TraceParams P) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tiles_x = (P.pc.width + 7) / 8, tiles = tiles_x * ((P.local_rows + 7) / 8);
  const uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= tiles) return;  // wave-uniform
  const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const uint32_t x = tx * 8 + (lane & 7), lr = ty * 8 + (lane >> 3);
  const uint32_t y = global_row(lr, P);
  const bool active = x < P.pc.width && lr < P.local_rows && y < P.pc.height;
  f3 centre = mk(0.0f, 0.0f, 0.0f);
  if (active) {
    const float4 rc = P.rays[x + y * P.pc.width];
    centre = mk(rc.x, rc.y, rc.z);
  }
  const TileList t = build_tile_list(P, active, centre, nullptr);
  uint32_t* rec = P.tl_cache + (size_t)tile * kTlRecWords;
  rec[lane] = t.v;
  rec[64 + lane] = t.tsum;
  if (lane == 0) {
    rec[128] = t.n;
    rec[129] = t.ok ? 1u : 0u;
    rec[130] = (uint32_t)t.aabb;
    rec[131] = (uint32_t)(t.aabb >> 32);
    rec[132] = t.aabb_ok ? 1u : 0u;
  }
}

// Per-frame prep for the bundle variants: one workgroup per mesh, order-preserving compaction of the
// mesh's camera-facing triangles (num_t(cam_pos) > 0, computed exactly as the trace kernel does).
__global__ __launch_bounds__(256) void camera_lists(TraceParams P) {
  const uint32_t m = blockIdx.x;
  const hrt_mesh& mesh = P.meshes[m];
  __shared__ uint32_t wave_counts[4];
  __shared__ uint32_t base_s;
  uint32_t start = 0;
  for (uint32_t j = 0; j < m; ++j) start += P.meshes[j].len;
  if (threadIdx.x == 0) base_s = 0;
  const f3 o = mk(P.pc.cam_pos[0], P.pc.cam_pos[1], P.pc.cam_pos[2]);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t c0 = 0; c0 < mesh.len; c0 += 256) {
    const uint32_t k = c0 + threadIdx.x;
    bool keep = false;
    f3 ao = mk(0.0f, 0.0f, 0.0f);
    float nt = 0.0f;
    if (k < mesh.len) {
      const hrt_triangle& t = P.tris[mesh.first_index + k];
      ao = o - ld3(t.a);
      nt = dot(ao, ld3(t.normal));
      keep = nt > 0.0f;
    }
    const unsigned long long ballot = __ballot(keep);
    const uint32_t prefix = __popcll(ballot & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) wave_counts[wave] = __popcll(ballot);
    __syncthreads();
    uint32_t off = base_s;
    for (uint32_t w = 0; w < wave; ++w) off += wave_counts[w];
    if (keep) {
      const uint32_t dst = start + off + prefix, idx = mesh.first_index + k;
      const hrt_triangle& t = P.tris[idx];
      const f3 n = ld3(t.normal), e1 = ld3(t.edge_one), e2 = ld3(t.edge_two);
      float4* out = P.cam_tris + 4 * (size_t)dst;
      out[0] = make_float4(ao.x, ao.y, ao.z, nt);
      out[1] = make_float4(e1.x, e1.y, e1.z, __builtin_bit_cast(float, idx));
      out[2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
      out[3] = make_float4(n.x, n.y, n.z, 0.0f);
      // bundle-cull record: the linear forms' coefficients and their margins
      const f3 gu = cross(e2, ao), h = cross(e1, ao);
      const f3 kw = (gu - h) + n;
      auto nrm = [](f3 v) { return __builtin_sqrtf(v.x * v.x + v.y * v.y + v.z * v.z) * 1.0001f; };
      const float pn = nrm(n), pao = nrm(ao), pu = nrm(e2) * pao, pv = nrm(e1) * pao;
      const float tiny = pn * 9.094947017729282e-13f;  // 2^-40 |n|
      float4* cc = P.cam_cull + 5 * (size_t)dst;
      cc[0] = make_float4(n.x, n.y, n.z, 1e-5f * pn);
      cc[1] = make_float4(gu.x, gu.y, gu.z, 1e-5f * pu + tiny);
      cc[2] = make_float4(h.x, h.y, h.z, 1e-5f * pv + tiny);
      cc[3] = make_float4(kw.x, kw.y, kw.z, 1e-5f * (pu + pv + pn) + pn * 6.103515625e-05f);
      cc[4] = make_float4(pn, fmaxf(nrm(gu), pu), fmaxf(nrm(h), pv), nrm(kw) + 1e-5f * (pu + pv + pn));
    }
    __syncthreads();
    if (threadIdx.x == 0) base_s += wave_counts[0] + wave_counts[1] + wave_counts[2] + wave_counts[3];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    P.cam_start[m] = start;
    P.cam_count[m] = base_s;
  }
}

// ---- ray centres (create_ray_subbuffer's loop, src/raytrace_pipeline.rs:319-326) ------------------
// (first + px * x) + py * y per component, each product and sum rounded as written (-ffp-contract=off):
// the same bits as hrt_host_create_rays.
// normalize(triangle normal) once per scene, as resolve_hit would per hit (raytracing.glsl:282 hit_normal)
// One thread per direction cell: the cell's band record (band_cell) -- its list's start and length, then
// the list's first kBandInline entries as half-words (unused ones 0) -- as two 16 B stores.
__global__ __launch_bounds__(256) void band_records(const uint32_t* __restrict__ off, const uint32_t* __restrict__ band16,
                                                    uint4* __restrict__ rec, uint32_t cells) {
  const uint32_t c = blockIdx.x * 256u + threadIdx.x;
  if (c >= cells) return;
  const uint32_t b0 = off[c], n = off[c + 1] - b0;
  uint32_t w[8] = {b0, n, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t j = 0; j < kBandInline; ++j) {
    const uint32_t k = b0 + j;
    if (j < n) w[2 + j / 2] |= ((band16[k >> 1] >> ((k & 1u) << 4)) & 0xFFFFu) << ((j & 1u) << 4);
  }
  rec[2 * (size_t)c] = make_uint4(w[0], w[1], w[2], w[3]);
  rec[2 * (size_t)c + 1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ __launch_bounds__(256) void tri_normals(const hrt_triangle* tris, float4* nhat, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const f3 v = normalize(ld3(tris[i].normal));
  nhat[i] = make_float4(v.x, v.y, v.z, 0.0f);
}

__global__ __launch_bounds__(256) void make_rays(float4* rays, uint32_t width, uint32_t height, float fx, float fy,
                                                 float fz, float pxx, float pxy, float pxz, float pyx, float pyy,
                                                 float pyz) {
  const uint32_t x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= width || y >= height) return;
  const float xf = (float)x, yf = (float)y;
  rays[(size_t)y * width + x] = make_float4((fx + pxx * xf) + pyx * yf, (fy + pxy * xf) + pyy * yf,
                                            (fz + pxz * xf) + pyz * yf, 1.0f);
}

// ---- init clear (raytracing.glsl:363-366) and image_combiner.glsl (:22-43) ----------------------
__global__ __launch_bounds__(256) void clear_kernel(uint32_t* img8, float4* img32, size_t npix) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  if (img8) img8[i] = 255u << 24;
  if (img32) img32[i] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
}

// image_combiner.glsl:22-43 for one pixel: frame 0 clears, frame k folds the new frame in.
__device__ __forceinline__ uint32_t combine_rgba8(uint32_t pv, uint32_t nv, uint32_t frame) {
  if (frame == 0) return 255u << 24;
  const float ff = (float)frame, ff1 = (float)(frame + 1u);
  uint32_t out = 255u << 24;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float prev = unorm8_to_float((pv >> (8 * ch)) & 255u);
    const float nc = unorm8_to_float((nv >> (8 * ch)) & 255u);
    out |= unorm8((nc + prev * ff) / ff1) << (8 * ch);
  }
  return out;
}
__device__ __forceinline__ float4 combine_rgba32f(float4 p, float4 n, uint32_t frame) {
  if (frame == 0) return make_float4(0.0f, 0.0f, 0.0f, 1.0f);
  const float ff = (float)frame, ff1 = (float)(frame + 1u);
  return make_float4((n.x + p.x * ff) / ff1, (n.y + p.y * ff) / ff1, (n.z + p.z * ff) / ff1, 1.0f);
}
// combine_rgba8 with its nine IEEE divisions replaced by the same quotients (r05): the six UNORM8 loads
// k / 255 from a 256-entry table of those quotients (unorm8_to_float, built once per workgroup in LDS),
// and the three divisions by frame + 1 through that denominator's reciprocal, shared by the channels
// (div_core: rcp_core is RN(1 / b) on [2^-40, 2^40], every numerator here is 0 or in [2^-8, 2^33], so
// Markstein's correction gives the correctly rounded quotient; a zero numerator gives +0 as the IEEE
// division does).  combine_rgba8 stays the reference spelling (tests/test_gpu_parity.py holds every
// accumulator to the oracle's combiner).
__device__ __forceinline__ uint32_t combine_rgba8_fast(uint32_t pv, uint32_t nv, uint32_t frame, const float* tab) {
  if (frame == 0) return 255u << 24;
  const float ff = (float)frame, ff1 = (float)(frame + 1u), y = rcp_core(ff1);
  uint32_t out = 255u << 24;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float prev = tab[(pv >> (8 * ch)) & 255u];
    const float nc = tab[(nv >> (8 * ch)) & 255u];
    out |= unorm8(div_core(nc + prev * ff, ff1, y)) << (8 * ch);
  }
  return out;
}
#ifndef HRT_COMBINE_FAST
#define HRT_COMBINE_FAST 1
#endif
__device__ __forceinline__ void unorm8_table(float* tab) {  // blockDim.x == 256
  tab[threadIdx.x] = unorm8_to_float(threadIdx.x);
  __syncthreads();
}
__global__ __launch_bounds__(256) void accumulate_rgba8(uint32_t* cur, const uint32_t* nw, size_t npix, uint32_t frame) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#if HRT_COMBINE_FAST
  __shared__ float tab[256];
  unorm8_table(tab);
  if (i >= npix) return;
  cur[i] = combine_rgba8_fast(frame == 0 ? 0u : cur[i], nw[i], frame, tab);
#else
  if (i >= npix) return;
  cur[i] = combine_rgba8(frame == 0 ? 0u : cur[i], nw[i], frame);
#endif
}
// hrt_compute_n: the nf frames of one launch folded in frame order in one pass (frame frame0 + f is
// image f of the stack): the per-frame combiner's arithmetic, pixel by pixel, with the accumulator
// read and written once instead of once per frame.
__global__ __launch_bounds__(256) void accumulate_frames_rgba8(uint32_t* cur, const uint32_t* stack, size_t npix,
                                                             uint32_t nf, uint32_t frame0) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#if HRT_COMBINE_FAST
  __shared__ float tab[256];
  unorm8_table(tab);
#endif
  if (i >= npix) return;
  uint32_t v = cur[i];
#if HRT_COMBINE_FAST
  for (uint32_t f = 0; f < nf; ++f) v = combine_rgba8_fast(v, stack[f * npix + i], frame0 + f, tab);
#else
  for (uint32_t f = 0; f < nf; ++f) v = combine_rgba8(v, stack[f * npix + i], frame0 + f);
#endif
  cur[i] = v;
}
__global__ __launch_bounds__(256) void accumulate_frames_rgba32f(float4* cur, const float4* stack, size_t npix,
                                                               uint32_t nf, uint32_t frame0) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  float4 v = cur[i];
  for (uint32_t f = 0; f < nf; ++f) v = combine_rgba32f(v, stack[f * npix + i], frame0 + f);
  cur[i] = v;
}

__global__ __launch_bounds__(256) void accumulate_rgba32f(float4* cur, const float4* nw, size_t npix, uint32_t frame) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  cur[i] = combine_rgba32f(frame == 0 ? make_float4(0.0f, 0.0f, 0.0f, 1.0f) : cur[i], nw[i], frame);
}

// format conversion for hrt_read_image
__global__ __launch_bounds__(256) void rgba8_to_f32(const uint32_t* src, float4* dst, size_t npix) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint32_t v = src[i];
  dst[i] = make_float4(unorm8_to_float(v & 255u), unorm8_to_float((v >> 8) & 255u), unorm8_to_float((v >> 16) & 255u),
                       unorm8_to_float(v >> 24));
}
__global__ __launch_bounds__(256) void f32_to_rgba8(const float4* src, uint32_t* dst, size_t npix) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const float4 v = src[i];
  dst[i] = unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | (unorm8(v.w) << 24);
}

// Row-tile framebuffer assembly after the gather: global row y lives in part
// (y / row_tile) % parts at local row (y / row_tile / parts) * row_tile + y % row_tile.  One 4-byte word
// per lane; grid.y = rows, so the row arithmetic is wave-uniform and both sides stream coalesced.
__global__ __launch_bounds__(256) void assemble_rows(const uint32_t* __restrict__ gathered, uint32_t* __restrict__ frame,
                                                     uint32_t row_words, uint32_t local_rows, uint32_t row_tile,
                                                     uint32_t parts) {
  const uint32_t y = blockIdx.y;
  const uint32_t t = y / row_tile;
  const uint32_t part = t % parts;
  const uint32_t lr = (t / parts) * row_tile + y % row_tile;
  const uint32_t* src = gathered + ((size_t)part * local_rows + lr) * row_words;
  uint32_t* dst = frame + (size_t)y * row_words;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < row_words; i += gridDim.x * 256) dst[i] = src[i];
}

// Self-check of hrt_math.h's shared-reciprocal division and sqrt paths against the compiler's IEEE
// sequences, bit for bit, on hashed inputs (exponents over the whole range for a third of the
// threads, the fast-path range for the rest).  out[0..3]: normalize, div3, sqrt mismatches, fast cases.
__device__ __forceinline__ float math_check_value(uint32_t& st, bool wide) {
  const uint32_t h = hash(st), g = hash(st);
  if (wide) return __builtin_bit_cast(float, h);  // any bit pattern: NaN, inf, denormals, zeros
  const int e = (int)(g % 100u) - 50;             // |v| in [2^-50, 2^50)
  const float m = __builtin_bit_cast(float, 0x3f800000u | (h & 0x007fffffu));
  const float v = __builtin_ldexpf(m, e);
  return (g >> 31) ? -v : v;
}
// Exhaustive over the 2^32 values of a u01 draw (k = base + thread): sqrt_rng against the compiler's
// sqrt on u01(k) and on -2 log(u01(k)), and spec_sincos_angle against spec_sincos on the two angle
// forms of raytracing.glsl (u * 2 * pi and 6.2831852 * u); and adjust_dir's Lambertian shortcut
// premise: a normal_dist radius sqrt(-2 log u) is finite and nonzero iff u is neither 0 nor 1, and the
// cosine of 6.2831852 u is never 0 (and spec_log_u01 equals spec_log on every u01 value); and
// rcp_core's reciprocal is correctly rounded on div_core's range (k read as a float).
// out[0..2]: violations of each.
__global__ __launch_bounds__(256) void math_check_rng(uint32_t base, unsigned long long* out) {
  const uint32_t k = base + blockIdx.x * 256u + threadIdx.x;
  const float u = u01(k);
  const float l = -2.0f * spec_log(u);
  const bool bad_sqrt = fbits(sqrt_rng(u)) != fbits(__builtin_sqrtf(u)) ||
                        fbits(sqrt_rng(l)) != fbits(__builtin_sqrtf(l));
  float s0, c0, s1, c1, s2, c2, s3, c3;
  const float r = (u * 2.0f) * 3.14159265358979323846f, th = 6.2831852f * u;
  spec_sincos(r, s0, c0);
  spec_sincos_angle(r, s1, c1);
  spec_sincos(th, s2, c2);
  spec_sincos_angle(th, s3, c3);
  const bool bad_sc = fbits(s0) != fbits(s1) || fbits(c0) != fbits(c1) || fbits(s2) != fbits(s3) ||
                      fbits(c2) != fbits(c3);
  const float rho = sqrt_rng(l);
  const bool rho_nz = fabsf(rho) < __builtin_inff() && rho != 0.0f;
  const bool bad_fast = rho_nz != (u != 0.0f && u != 1.0f) || c3 == 0.0f ||
                        (k - 1u < 0xFFFFFF7Fu) != (u != 0.0f && u != 1.0f);  // adjust_dir's HRT_FUZZ_INT test
  const bool bad_log = fbits(spec_log_u01(u)) != fbits(spec_log(u));
  // the folded u01 scalings of get_ray_dir and normal_dist (u01_mul), exact by construction
  const bool bad_mul = fbits(u01_mul(k, 3.14159265358979323846f * 0x1p-31f)) != fbits(r) ||
                       fbits(u01_mul(k, 6.2831852f * 0x1p-32f)) != fbits(th);
  if (bad_sqrt) atomicAdd(&out[0], 1ull);
  // the hardware square root alone against the correctly rounded one on both domains (out[3], out[4]):
  // where it never differs, sqrt_rng needs no correction steps
  if (fbits(__builtin_amdgcn_sqrtf(u)) != fbits(__builtin_sqrtf(u))) atomicAdd(&out[3], 1ull);
  if (fbits(__builtin_amdgcn_sqrtf(l)) != fbits(__builtin_sqrtf(l))) atomicAdd(&out[4], 1ull);
  if (bad_sc) atomicAdd(&out[1], 1ull);
  // rcp_core(b) = RN(1/b) for every float b in [2^-40, 2^40] (k read as a float), the premise of
  // div_core's one correction
  const float bk = bitsf(k);
  const bool bad_rcp = bk >= 0x1p-40f && bk <= 0x1p40f && fbits(rcp_core(bk)) != fbits(1.0f / bk);
  if (bad_fast || bad_log || bad_rcp || bad_mul) atomicAdd(&out[2], 1ull);
}
// hrt_debug_band_flatten: BandFlat on 64 given lists (n[l], b0[l]); out[(r * 64 + l) * 2 + {0, 1}] = the
// owner and entry of slot r * 64 + l for each round r < rounds, and out[rounds * 128] = total.
__global__ __launch_bounds__(64) void band_flatten_check(const uint32_t* n_in, const uint32_t* b0_in, uint32_t rounds,
                                                         uint32_t* out) {
  __shared__ uint8_t marks[64];
  const uint32_t lane = threadIdx.x & 63u, n = n_in[lane], b0 = b0_in[lane];
  uint32_t total;
  const uint32_t pos = wave_scan_excl(n, total);  // (the kernel's scan, checked here on given counts)
  BandFlat bf{marks, lane, n, pos, total, b0 - pos, 0u};
  for (uint32_t r = 0; r < rounds; ++r) {
    uint32_t own;
    const uint32_t k = bf.slot(r * 64u, own);
    out[(r * 64u + lane) * 2u] = own;
    out[(r * 64u + lane) * 2u + 1u] = k;
  }
  if (lane == 0) out[rounds * 128u] = total;
}

// hrt_debug_wq_protocol: the pair traversal's LDS handoffs on a scripted run of one wave -- per round,
// the top take[r] entries popped (lane l < take reads entry n - take + l), each lane's slot read and
// lowering of slot tgt (tgt >= 64: none), then the lanes' pushes (lane l pushes cnt[r][l] <= 4 entries
// (r << 16 | l << 8 | k), slot-major as the node steps push) -- in the product kernel's order, with
// its helpers (wq_push, lds_get, wq_slot_*, wave_handoff).
constexpr uint32_t kProtoCap = 8192;
__global__ __launch_bounds__(64) void wq_protocol_check(uint32_t rounds, const uint32_t* cnt, const uint32_t* take,
                                                        const uint32_t* tgt, const unsigned long long* val,
                                                        const unsigned long long* seed, uint32_t* popped,
                                                        unsigned long long* seen, unsigned long long* slots_out,
                                                        uint32_t* depth_out) {
  __shared__ unsigned long long slot[64];
  __shared__ uint32_t st[kProtoCap];
  const uint32_t lane = threadIdx.x & 63u;
  wq_slot_seed(slot, lane, seed[lane]);
  wave_handoff();
  uint32_t n = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t tk = min(take[r], n);
    n -= tk;
    wave_handoff();
    popped[r * 64u + lane] = lane < tk ? lds_get(&st[n + lane]) : ~0u;
    const uint32_t t = tgt[r * 64u + lane];
    if (t < 64u) {
      seen[r * 64u + lane] = lds_get(&slot[t]);
      wq_slot_lower(slot, t, val[r * 64u + lane]);
    }
    const uint32_t c = cnt[r * 64u + lane];
    wave_handoff();
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) wq_push(st, n, c > k && n + 256u <= kProtoCap, (r << 16) | (lane << 8) | k);
  }
  wave_handoff();
  slots_out[lane] = lds_get(&slot[lane]);
  if (lane == 0) *depth_out = n;
}

__global__ __launch_bounds__(256) void math_check(uint32_t n, uint32_t seed, unsigned long long* out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t st = seed * 2654435761u + i;
  const bool wide = (i % 3u) == 0u;
  const f3 a = mk(math_check_value(st, wide), math_check_value(st, wide), math_check_value(st, wide));
  const f3 x = normalize(a), y = normalize_ieee(a);
  const bool bad_n = fbits(x.x) != fbits(y.x) || fbits(x.y) != fbits(y.y) || fbits(x.z) != fbits(y.z);
  const float sv = __builtin_fabsf(math_check_value(st, wide));
  const f3 p = div3(a, sv);
  const bool bad_d = sv > 0.0f && (fbits(p.x) != fbits(a.x / sv) || fbits(p.y) != fbits(a.y / sv) ||
                                   fbits(p.z) != fbits(a.z / sv));
  const float q = __builtin_fabsf(math_check_value(st, wide));
  const bool in = q >= 0x1p-96f && q <= 0x1p80f;
  const bool bad_s = in && fbits(sqrt_core(q)) != fbits(__builtin_sqrtf(q));
  const float d2 = dot(a, a);
  const bool fast = d2 >= 0x1p-80f && d2 <= 0x1p78f;
  if (bad_n) atomicAdd(&out[0], 1ull);
  if (bad_d) atomicAdd(&out[1], 1ull);
  if (bad_s) atomicAdd(&out[2], 1ull);
  if (fast) atomicAdd(&out[3], 1ull);
}

}  // namespace hrt

// ---- launch wrappers (host) ----------------------------------------------------------------------
namespace hrt {

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + 255) / 256); }
constexpr size_t kMaxLdsScene = 160 * 1024 - 64;  // dynamic LDS per CU, leaving room for the kernels' static LDS
constexpr uint32_t kAutoCullTris = 256;   // BUNDLE_CULL from this many mesh triangles, BUNDLE below
constexpr uint32_t kAutoBvhTris = 4096;   // BUNDLE_BVH from this many (profiles/r01d_bvh_scaling.log)
constexpr uint32_t kAutoWqStack = 384;    // BUNDLE_WQ when its per-wave node stacks hold this many entries

// BUNDLE_BVH_LDS footprint: triangles + nodes + entries + key bases.
size_t bvh_lds_bytes(const TraceParams& p) {
  return (size_t)p.n_tris * 48 + (size_t)p.bvh_n_nodes * 64 + (size_t)p.bvh_n_prims * 4 + (size_t)p.bvh_n_meshes * 4;
}
bool bvh_lds_fits(const TraceParams& p) { return p.bvh_nodes && p.bvh_entries && bvh_lds_bytes(p) <= kMaxLdsScene; }

// BUNDLE_CULL_LDS workgroup size for a scene of n triangles (0 = does not fit): two 512-thread
// workgroups per CU when twice the footprint fits the 160 KiB, else one of 1024.
constexpr size_t kCoopLds = 3 * 64 * 8;  // cooperative-tile exchange slots
uint32_t lds_block(uint32_t n) {
  const size_t tri = (size_t)n * 48 + kCoopLds;
  return tri <= kMaxLdsScene / 2 ? 512u : tri <= kMaxLdsScene ? 1024u : 0u;
}

// BUNDLE_WQ per-wave pair stacks: triangle stack 64 x (1 + 2 x largest leaf), node stack what is left of
// the 160 KiB after the nodes (at most 1024 pairs, at least 128).  Returns the LDS bytes, 0 = no fit.
// Triangle stack: 64 x (1 + 2 x largest leaf) pairs -- a node step's pushes onto < 64 waiting ones
// when each lane keeps at most two leaves; a larger burst of a grouped step is tested in place.
constexpr uint32_t wq_tri_cap(uint32_t max_leaf) { return 64u * (1u + 2u * max_leaf); }
uint32_t wq_stack_cap(uint32_t n_nodes, uint32_t width, uint32_t max_leaf) {
  if (max_leaf > 4 || width > kWqSlots || width < 2) return 0;
  const size_t nodes = (size_t)n_nodes * 48, t = wq_tri_cap(max_leaf);
  if (nodes + 16 * (512 + 4 * (t + 128)) > kMaxLdsScene) return 0;
  const size_t per_wave = (kMaxLdsScene - nodes) / 16;
  return (uint32_t)std::min<size_t>(1024, ((per_wave - 512 - 4 * t) / 4) & ~(size_t)63);
}

size_t wq_lds_bytes(const TraceParams& p, uint32_t* ncap, uint32_t* tcap) {
  if (!p.bvh_nodes || !p.bvh_wq_nodes) return 0;
  const uint32_t n = wq_stack_cap(p.bvh_wq_n_nodes, p.bvh_wq_width, p.bvh_max_leaf);
  if (n == 0) return 0;
  const size_t t = wq_tri_cap(p.bvh_max_leaf);
  if (ncap) *ncap = n;
  if (tcap) *tcap = (uint32_t)t;
  return (size_t)p.bvh_wq_n_nodes * 48 + 16 * (512 + 4 * ((size_t)n + t));
}

int resolve_variant(const TraceParams& p, int variant) {
  if (variant == HRT_KERNEL_AUTO) {
    // profiles/r01g_*: island 21.4 (LDS) vs 23.7 ms, cave 112 vs 120 ms; BVH from ~4K triangles.
    // BUNDLE_WQ when its node stacks get >= kAutoWqStack entries (r02, node groups: island 2.84 vs
    // ~15 ms for BUNDLE_CULL_LDS; cave 17.3 ms at 384-entry stacks vs 20.2, profiles/r02p_cave_wq.txt)
    // A poor hierarchy (large overlapping triangles, HRT_SCENE_BVH_SAH_MILLI > 100) is left to the
    // wave-level culls: triangle soups of 256 / 1K / 4K / 16K run 2.5-5x faster culled
    // (profiles/r01p_soup_sweep.log).
    uint32_t ncap = 0;
    const bool good_bvh = p.bvh_nodes && p.bvh_sah_milli <= 100;
    const bool wq = good_bvh && wq_lds_bytes(p, &ncap, nullptr) && ncap >= kAutoWqStack && p.pc.num_meshes <= 64;
    variant = p.cam_list_capacity < kAutoCullTris                   ? HRT_KERNEL_BUNDLE
              : wq                                                 ? HRT_KERNEL_BUNDLE_WQ
              : p.cam_list_capacity >= kAutoBvhTris && good_bvh    ? HRT_KERNEL_BUNDLE_BVH
              : lds_block(p.n_tris) != 0                ? HRT_KERNEL_BUNDLE_CULL_LDS
                                                                 : HRT_KERNEL_BUNDLE_CULL;
  }
  if (variant == HRT_KERNEL_BRUTE_LDS && (size_t)p.n_tris * 48 > kMaxLdsScene) variant = HRT_KERNEL_BRUTE;
  if (variant == HRT_KERNEL_BUNDLE_BVH && (!p.bvh_nodes || p.pc.num_meshes > 64)) variant = HRT_KERNEL_BUNDLE_CULL;
  if (variant == HRT_KERNEL_BUNDLE_CULL_LDS && lds_block(p.n_tris) == 0) variant = HRT_KERNEL_BUNDLE_CULL;
  if (variant == HRT_KERNEL_BUNDLE_WQ && (wq_lds_bytes(p, nullptr, nullptr) == 0 || p.pc.num_meshes > 64))
    variant = HRT_KERNEL_BUNDLE_BVH_LDS;
  if (variant == HRT_KERNEL_BUNDLE_BVH_LDS && !bvh_lds_fits(p)) variant = HRT_KERNEL_BUNDLE_BVH;
  if (variant == HRT_KERNEL_BUNDLE_BVH_LDS && (!p.bvh_nodes || p.pc.num_meshes > 64)) variant = HRT_KERNEL_BUNDLE_CULL;
  if (p.pc.max_bounces < 0) variant = HRT_KERNEL_LITERAL;  // the fused loops assume >= 1 segment per path
  return variant;
}

static uint32_t tiles_of(const TraceParams& p) { return ((p.pc.width + 7) / 8) * ((p.local_rows + 7) / 8); }

// Persistent kernels: plan this trace from the last one's tile costs (when p.plan_valid and
// splitting is on), then reset the counters the trace fills.  q.items = nullptr: plain tile order.
static hipError_t prepare_schedule(TraceParams& q, hipStream_t stream) {
  const uint32_t tiles = ((q.pc.width + 7) / 8) * ((q.local_rows + 7) / 8);
  // longest-first order whenever last trace's costs are known (and tile indices fit the item word)
  const bool plan = q.plan_valid && tiles > 0 && tiles <= kItemTileMask;
  q.items = plan ? q.item_buf : nullptr;
  hipError_t e;
  if (plan) {
    if ((e = hipMemsetAsync(q.sched + kSchedHist, 0, 3 * kPlanBuckets * 4, stream)) != hipSuccess) return e;  // histogram, cursors
    plan_hist<<<(tiles + 255) / 256, 256, 0, stream>>>(q.sched, q.tile_cost, tiles);
    // factor auto (-1): 3 when a resident wave gets more than 4 tiles, else 1 (profiles/r01k_schedule_sweep)
    // a launch of nf frames: a resident wave's fair share is nf frames' work, i.e. waves / nf per frame
    const uint32_t nf = q.n_frames > 1 ? q.n_frames : 1u;
    const uint32_t waves = std::max(1u, q.num_cus * 16u / nf);
    const uint32_t factor4 =
        q.split_factor4 ? q.split_factor4 : 4u * (q.split_factor >= 0 ? (uint32_t)q.split_factor : tiles > 4 * waves ? 3u : 1u);
    plan_scan<<<1, 64, 0, stream>>>(q.sched, waves, factor4, q.split_k, q.split_prio);
    plan_fill<<<(tiles + 255) / 256, 256, 0, stream>>>(q.sched, q.tile_cost, tiles, q.split_k, q.split_prio,
                                                       q.item_buf);
  }
  if ((e = hipMemsetAsync(q.tile_cost, 0, (size_t)tiles * 4, stream)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(q.sched + 5, 0, 12, stream)) != hipSuccess) return e;  // coop counter, cost sum
  return hipMemsetAsync(q.sched, 0, 4, stream);
}

// The persistent kernels' dynamic-LDS limits, set once per device (hrt_create calls this for its device;
// the attribute is per device, so every device a context lives on gets its own call).
hipError_t ensure_kernel_attributes(int device) {
  static std::mutex mu;
  static std::vector<char> done;
  std::lock_guard<std::mutex> lock(mu);
  if (device < 0) return hipErrorInvalidDevice;
  if ((size_t)device < done.size() && done[(size_t)device]) return hipSuccess;
  const void* brute[] = {reinterpret_cast<const void*>(&trace_brute_lds)};
  const void* half_cu[] = {reinterpret_cast<const void*>(&trace_bundle_cull_lds<512, false>),
                           reinterpret_cast<const void*>(&trace_bundle_cull_lds<512, true>)};
  const void* whole_cu[] = {reinterpret_cast<const void*>(&trace_bundle_cull_lds<1024, false>),
                            reinterpret_cast<const void*>(&trace_bundle_cull_lds<1024, true>),
                            reinterpret_cast<const void*>(&trace_bundle_bvh_lds<false>),
                            reinterpret_cast<const void*>(&trace_bundle_bvh_lds<true>),
                            reinterpret_cast<const void*>(&trace_bundle_wq<false>),
                            reinterpret_cast<const void*>(&trace_bundle_wq<true>),
                            reinterpret_cast<const void*>(&trace_bundle_wq_nr<false>),
                            reinterpret_cast<const void*>(&trace_bundle_wq_nr<true>)};
  hipError_t e;
  for (const void* f : brute)
    if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene)) != hipSuccess)
      return e;
  for (const void* f : half_cu)
    if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kMaxLdsScene / 2))) !=
        hipSuccess)
      return e;
  for (const void* f : whole_cu)
    if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene)) != hipSuccess)
      return e;
  if (done.size() <= (size_t)device) done.resize((size_t)device + 1, 0);
  done[(size_t)device] = 1;
  return hipSuccess;
}

hipError_t launch_trace(const TraceParams& p0, int variant, hipStream_t stream, int* ran, int* block_out) {
  TraceParams p = p0;
  variant = resolve_variant(p, variant);
  *ran = variant;
  // bounce batch threshold, auto: the pair traversal's step cost scales with its rays, so BUNDLE_WQ
  // batches earlier (28 of 64 lanes); the cull kernels test every survivor for the whole wave (48)
  // (profiles/r01q_sec_batch_sweep.jsonl, frames in 16-frame launches); 36 for the per-node-radius
  // kernel, whose scenes bounce far more (cave 20 / 28 / 36 / 44 / 56: 7.43 / 7.38 / 7.31 / 7.32 /
  // 7.45 ms; island stays best at 28: profiles/r02v_ab.txt)
  if (p.sec_batch == 0) p.sec_batch = variant == HRT_KERNEL_BUNDLE_WQ ? (p.bvh_node_r ? 36u : 28u) : 48u;
  *block_out = variant == HRT_KERNEL_BRUTE_LDS ? 1024 : 256;
  const dim3 grid((p.pc.width + 15) / 16, (p.local_rows + 15) / 16, 1);
  switch (variant) {
    case HRT_KERNEL_LITERAL:
      trace_literal<<<grid, 256, 0, stream>>>(p);
      break;
    case HRT_KERNEL_BRUTE_LDS: {
      const dim3 g32((p.pc.width + 31) / 32, (p.local_rows + 31) / 32, 1);
      trace_brute_lds<<<g32, 1024, (size_t)p.n_tris * 48, stream>>>(p);
      break;
    }
    case HRT_KERNEL_BUNDLE_BVH_LDS: {
      if (p.pc.num_meshes > 0 && !p.cam_lists_ready) camera_lists<<<p.pc.num_meshes, 256, 0, stream>>>(p);
      if (HRT_TL_PREPASS && p.tl_cache && !p.tl_lists_ready) tile_lists<<<(tiles_of(p) + 3) / 4, 256, 0, stream>>>(p);
      TraceParams q = p;
      q.coop = 0;
      if (q.split_k == 0) q.split_k = 1;
      const size_t lds = bvh_lds_bytes(p);
      if (hipError_t e = prepare_schedule(q, stream); e != hipSuccess) return e;
      if (p.diag || p.probe)
        trace_bundle_bvh_lds<true><<<p.num_cus, 1024, lds, stream>>>(q);
      else
        trace_bundle_bvh_lds<false><<<p.num_cus, 1024, lds, stream>>>(q);
      *block_out = 1024;
      break;
    }
    case HRT_KERNEL_BUNDLE_WQ: {
      if (p.pc.num_meshes > 0 && !p.cam_lists_ready) camera_lists<<<p.pc.num_meshes, 256, 0, stream>>>(p);
      if (HRT_TL_PREPASS && p.tl_cache && !p.tl_lists_ready) tile_lists<<<(tiles_of(p) + 3) / 4, 256, 0, stream>>>(p);
      TraceParams q = p;
      q.coop = 0;
      // auto: a pair step's work scales with the rays in the batch, so heavy tiles (> factor x a
      // resident wave's fair share of the work) run as 2, 4 or 8 items by cost; factor 2 when a
      // resident wave gets more than 6 tiles (the full frame), else 3 (row partitions at N > 1)
      // (profiles/r01o_lane_weighted_sum_factor_sweep.jsonl)
      if (q.split_k == 0) q.split_k = 8;
      // A launch of several frames (hrt_compute_n) splits a tile from 1.25 x a wave's share of the launch:
      // a rank of 8 holds 1/8 of the rows but the same pixel chains, and one cave tile's frame took 18 ms
      // against a 15 ms share, unsplit at 2 x (profiles/r06/r06aa/).  Cave's slowest rank of 8 0.88 ->
      // 0.80 ms per frame; island, 2 and 4 ranks and whole frames within noise (r06ac, r06ad).
      if (q.split_factor < 0 && p.n_frames > 1)
        q.split_factor4 = 5;
      else if (q.split_factor < 0)
        q.split_factor = (uint64_t)tiles_of(p) * std::max(1u, p.n_frames) > 6ull * p.num_cus * 16u ? 2 : 3;
      const size_t lds = wq_lds_bytes(p, &q.wq_ncap, &q.wq_tcap);
      if (p.wq_ncap) q.wq_ncap = std::min(q.wq_ncap, std::max(128u, p.wq_ncap & ~63u));  // HRT_OPT_WQ_NODE_CAP
      if (p.wq_tcap) q.wq_tcap = std::min(q.wq_tcap, std::max(128u, p.wq_tcap & ~63u));  // HRT_DEBUG_OPT_WQ_TRI_CAP
      if (hipError_t e = prepare_schedule(q, stream); e != hipSuccess) return e;
      if (p.bvh_node_r) {
        if (p.diag || p.probe)
          trace_bundle_wq_nr<true><<<p.num_cus, 1024, lds, stream>>>(q);
        else
          trace_bundle_wq_nr<false><<<p.num_cus, 1024, lds, stream>>>(q);
      } else if (p.diag || p.probe) {
        trace_bundle_wq<true><<<p.num_cus, 1024, lds, stream>>>(q);
      } else {
        trace_bundle_wq<false><<<p.num_cus, 1024, lds, stream>>>(q);
      }
      *block_out = 1024;
      break;
    }
    case HRT_KERNEL_BUNDLE_CULL_LDS: {
      if (p.pc.num_meshes > 0 && !p.cam_lists_ready) camera_lists<<<p.pc.num_meshes, 256, 0, stream>>>(p);
      if (HRT_TL_PREPASS && p.tl_cache && !p.tl_lists_ready) tile_lists<<<(tiles_of(p) + 3) / 4, 256, 0, stream>>>(p);
      TraceParams q = p;
      const uint32_t block = lds_block(p.n_tris);
      *block_out = (int)block;
      const size_t lds = (size_t)p.n_tris * 48 + kCoopLds;
      if (q.split_k == 0) q.split_k = 1;  // auto: cooperative heavy tiles instead
      q.coop = p.coop && q.split_k == 1 && p.pc.num_meshes <= 62 ? 1u : 0u;
      if (hipError_t e = prepare_schedule(q, stream); e != hipSuccess) return e;
      if (block == 512) {
        if (p.diag || p.probe)
          trace_bundle_cull_lds<512, true><<<2 * p.num_cus, 512, lds, stream>>>(q);
        else
          trace_bundle_cull_lds<512, false><<<2 * p.num_cus, 512, lds, stream>>>(q);
      } else {
        if (p.diag || p.probe)
          trace_bundle_cull_lds<1024, true><<<p.num_cus, 1024, lds, stream>>>(q);
        else
          trace_bundle_cull_lds<1024, false><<<p.num_cus, 1024, lds, stream>>>(q);
      }
      break;
    }
    case HRT_KERNEL_BUNDLE:
    case HRT_KERNEL_BUNDLE_CULL:
    case HRT_KERNEL_BUNDLE_BVH:
      if (p.pc.num_meshes > 0 && !p.cam_lists_ready) camera_lists<<<p.pc.num_meshes, 256, 0, stream>>>(p);
      if (variant == HRT_KERNEL_BUNDLE)
        p.diag ? trace_bundle<true><<<grid, 256, 0, stream>>>(p) : trace_bundle<false><<<grid, 256, 0, stream>>>(p);
      else if (variant == HRT_KERNEL_BUNDLE_CULL)
        p.diag ? trace_bundle_cull<true><<<grid, 256, 0, stream>>>(p)
               : trace_bundle_cull<false><<<grid, 256, 0, stream>>>(p);
      else
        p.diag ? trace_bundle_bvh<true><<<grid, 256, 0, stream>>>(p)
               : trace_bundle_bvh<false><<<grid, 256, 0, stream>>>(p);
      break;
    default:
      trace_brute<<<grid, 256, 0, stream>>>(p);
      break;
  }
  return hipGetLastError();
}

hipError_t launch_make_rays(float4* rays, uint32_t width, uint32_t height, const float first[3], const float px[3],
                            const float py[3], hipStream_t stream) {
  if (width == 0 || height == 0) return hipSuccess;
  const dim3 g((width + 15) / 16, (height + 15) / 16, 1);
  make_rays<<<g, 256, 0, stream>>>(rays, width, height, first[0], first[1], first[2], px[0], px[1], px[2], py[0],
                                   py[1], py[2]);
  return hipGetLastError();
}

hipError_t launch_accumulate_frames(uint32_t* cur8, const uint32_t* stack8, float4* cur32, const float4* stack32,
                                   size_t npix, uint32_t nf, uint32_t frame0, hipStream_t stream) {
  if (npix == 0 || nf == 0) return hipSuccess;
  if (cur8)
    accumulate_frames_rgba8<<<blocks_for(npix), 256, 0, stream>>>(cur8, stack8, npix, nf, frame0);
  else
    accumulate_frames_rgba32f<<<blocks_for(npix), 256, 0, stream>>>(cur32, stack32, npix, nf, frame0);
  return hipGetLastError();
}

hipError_t launch_band_records(const uint32_t* off, const uint32_t* band16, uint32_t* rec, uint32_t cells,
                               hipStream_t stream) {
  if (cells == 0) return hipSuccess;
  band_records<<<(cells + 255) / 256, 256, 0, stream>>>(off, band16, reinterpret_cast<uint4*>(rec), cells);
  return hipGetLastError();
}

hipError_t launch_tri_normals(const hrt_triangle* tris, float4* nhat, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  tri_normals<<<(n + 255) / 256, 256, 0, stream>>>(tris, nhat, n);
  return hipGetLastError();
}

hipError_t launch_clear(uint32_t* img8, float4* img32, size_t npix, hipStream_t stream) {
  if (npix == 0) return hipSuccess;
  clear_kernel<<<blocks_for(npix), 256, 0, stream>>>(img8, img32, npix);
  return hipGetLastError();
}

hipError_t launch_accumulate(uint32_t* cur8, const uint32_t* new8, float4* cur32, const float4* new32, size_t npix,
                             uint32_t frame, hipStream_t stream) {
  if (npix == 0) return hipSuccess;
  if (cur8)
    accumulate_rgba8<<<blocks_for(npix), 256, 0, stream>>>(cur8, new8, npix, frame);
  else
    accumulate_rgba32f<<<blocks_for(npix), 256, 0, stream>>>(cur32, new32, npix, frame);
  return hipGetLastError();
}

hipError_t launch_assemble_rows(const uint32_t* gathered, uint32_t* frame, uint32_t row_words, uint32_t height,
                                uint32_t local_rows, uint32_t row_tile, uint32_t parts, hipStream_t stream) {
  if (row_words == 0 || height == 0) return hipSuccess;
  if (parts == 0 || row_tile == 0 || (uint64_t)((height - 1) / row_tile / parts + 1) * row_tile > local_rows)
    return hipErrorInvalidValue;  // some global row would read outside its part's local rows
  const dim3 g(std::min<uint32_t>((row_words + 255) / 256, 64), height, 1);
  assemble_rows<<<g, 256, 0, stream>>>(gathered, frame, row_words, local_rows, row_tile, parts);
  return hipGetLastError();
}

hipError_t launch_wq_protocol_check(uint32_t rounds, const uint32_t* cnt, const uint32_t* take, const uint32_t* tgt,
                                    const unsigned long long* val, const unsigned long long* seed, uint32_t* popped,
                                    unsigned long long* seen, unsigned long long* slots, uint32_t* depth,
                                    hipStream_t stream) {
  wq_protocol_check<<<1, 64, 0, stream>>>(rounds, cnt, take, tgt, val, seed, popped, seen, slots, depth);
  return hipGetLastError();
}
hipError_t launch_band_flatten_check(const uint32_t* n, const uint32_t* b0, uint32_t rounds, uint32_t* out,
                                     hipStream_t stream) {
  band_flatten_check<<<1, 64, 0, stream>>>(n, b0, rounds, out);
  return hipGetLastError();
}
hipError_t launch_math_check_rng(unsigned long long* out, hipStream_t stream) {
  for (uint64_t base = 0; base < (1ull << 32); base += (1ull << 28)) {  // 16 launches of 2^28 states
    math_check_rng<<<(1u << 28) / 256u, 256, 0, stream>>>((uint32_t)base, out);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_math_check(uint32_t n, uint32_t seed, unsigned long long* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  math_check<<<(n + 255) / 256, 256, 0, stream>>>(n, seed, out);
  return hipGetLastError();
}

hipError_t launch_convert(const uint32_t* src8, float4* dst32, const float4* src32, uint32_t* dst8, size_t npix,
                          hipStream_t stream) {
  if (npix == 0) return hipSuccess;
  if (src8)
    rgba8_to_f32<<<blocks_for(npix), 256, 0, stream>>>(src8, dst32, npix);
  else
    f32_to_rgba8<<<blocks_for(npix), 256, 0, stream>>>(src32, dst8, npix);
  return hipGetLastError();
}

}  // namespace hrt
