// hrt_kernels.hip -- gfx950 kernels for the path-trace dispatch (assets/raytracing.glsl) and the
// progressive accumulator (assets/image_combiner.glsl).
//
// Geometry of a launch: 256-thread workgroups = 4 waves; each wave owns an 8x8 pixel tile (coherent
// primary rays share triangle-rejection outcomes), a workgroup a 16x16 tile.  Scene records are
// read with wave-uniform addresses, so hipcc streams triangles through SGPRs (s_load_dwordx16) --
// every lane of the wave tests the same triangle against its own ray.
//
// Two trace variants with identical results (tests/test_gpu_parity.py holds both to the oracle):
//   trace_literal  per-sample / per-bounce loops shaped like raytracing.glsl:308-389;
//   trace_tuned    the same arithmetic with (a) the sample and bounce loops fused into one
//                  per-lane segment loop, so a lane whose path ended starts its next sample
//                  instead of idling until the wave's longest path ends, and (b) a division-free
//                  conservative pre-test per triangle; the correctly rounded 1/det path runs only
//                  when some lane of the wave may accept the triangle (DESIGN.md "exact cull").
#include <hip/hip_runtime.h>

#include "hip_raytrace.h"
#include "hrt_kernels.h"
#include "hrt_math.h"

namespace hrt {

// Read-only views of the uploaded std430 records.
struct Scene {
  const float4* __restrict__ rays;
  const hrt_sphere* __restrict__ spheres;
  const hrt_triangle* __restrict__ tris;
  const hrt_mesh* __restrict__ meshes;
};

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 ray_at(f3 o, f3 d, float t) { return o + d * t; }  // :158-160

// local (compacted) row -> global row, hrt_create_info partition.
__device__ __forceinline__ uint32_t global_row(uint32_t lr, const TraceParams& p) {
  if (p.part_count <= 1) return lr;
  const uint32_t tile = lr / p.row_tile, r = lr - tile * p.row_tile;
  return (tile * p.part_count + p.part_index) * p.row_tile + r;
}

// get_ray_dir, raytracing.glsl:162-166 (u1, u2, u3 in that order)
__device__ __forceinline__ f3 get_ray_dir(const hrt_push_constants& pc, f3 c, uint32_t& state) {
  const float r = (u01(hash(state)) * 2.0f) * 3.14159265358979323846f;
  float sr, cr;
  spec_sincos(r, sr, cr);
  const float j = pc.jitter_size;
  const float s2 = __builtin_sqrtf(u01(hash(state)));
  const f3 t1 = ((mk(0.0f, 0.0f, 1.0f) * cr) * j) * s2;
  const float s3 = __builtin_sqrtf(u01(hash(state)));
  const f3 t2 = ((mk(0.0f, 1.0f, 0.0f) * sr) * j) * s3;
  const f3 nc = (c + t1) + t2;
  const float* M = pc.cam_alignment_mat;
  const f3 w = mk(__builtin_fmaf(M[8], nc.z, __builtin_fmaf(M[4], nc.y, M[0] * nc.x)),
                  __builtin_fmaf(M[9], nc.z, __builtin_fmaf(M[5], nc.y, M[1] * nc.x)),
                  __builtin_fmaf(M[10], nc.z, __builtin_fmaf(M[6], nc.y, M[2] * nc.x)));
  return normalize(w);
}

// intersecting_aabb, raytracing.glsl:192-210, restated with its min/max quirks (:202, :206).
__device__ __forceinline__ bool aabb_pass(const hrt_mesh& m, f3 o, f3 d) {
  const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
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
    h.normal = normalize(ld3(sc.tris[c.idx].normal));
    h.mat = &sc.meshes[c.mesh].material;
  }
  return h;
}

// environment_light, raytracing.glsl:290-294
__device__ __forceinline__ f3 environment_light(const hrt_push_constants& pc, f3 d) {
  if (!pc.use_environment_light) return mk(0.0f, 0.0f, 0.0f);
  const float a = 0.5f * (d.y + 1.0f);
  const float oma = 1.0f - a;
  return mk(oma * 1.0f + a * 0.5f, oma * 1.0f + a * 0.7f, oma * 1.0f + a * 1.0f);
}

// adjust_dir, raytracing.glsl:297-305 (both unit-sphere draws always happen: 12 hashes)
__device__ __forceinline__ f3 adjust_dir(f3 d, f3 n, const hrt_material& mat, bool specular, uint32_t& state) {
  const f3 diffuse_dir = normalize(n + unit_sphere(state));
  const float k = 2.0f * dot(n, d);
  const f3 specular_dir = d - n * k;
  const f3 fuzz = unit_sphere(state) * mat.settings[2];
  const float a = mat.settings[1] * (float)(int)specular;
  const float oma = 1.0f - a;
  const f3 mixed = mk(diffuse_dir.x * oma + specular_dir.x * a, diffuse_dir.y * oma + specular_dir.y * a,
                      diffuse_dir.z * oma + specular_dir.z * a);
  return normalize(mixed + fuzz);
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
    p.colour = p.colour / prob;
    return false;
  }
  p.light = p.light + environment_light(pc, p.dir);
  return true;
}

__device__ __forceinline__ void store_pixel(const TraceParams& P, uint32_t x, uint32_t lr, f3 col) {
  const size_t idx = (size_t)lr * P.pc.width + x;
  if (P.img8) {
    P.img8[idx] = unorm8(col.x) | (unorm8(col.y) << 8) | (unorm8(col.z) << 16) | (255u << 24);
  }
  if (P.img32) P.img32[idx] = make_float4(col.x, col.y, col.z, 1.0f);
}

// wave-level sums of the per-lane counters (+ the wave's longest lane), one atomic each per wave.
__device__ __forceinline__ void flush_counters(const TraceParams& P, uint32_t segs, uint32_t tests) {
  if (!P.counters) return;
  unsigned long long s = segs, t = tests;
  uint32_t mx = segs;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    t += __shfl_xor(t, off, 64);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&P.counters[0], s);
    atomicAdd(&P.counters[1], t);
    atomicAdd(&P.counters[2], (unsigned long long)mx);
  }
}

__device__ __forceinline__ void lane_pixel(const TraceParams& P, uint32_t& x, uint32_t& lr) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
  lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
}

// ---- literal variant: raytracing.glsl main (:355-389) with trace_ray's loop as written ----------
__global__ __launch_bounds__(256) void trace_literal(TraceParams P) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes};
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
    colour = colour / (float)pc.num_samples;
    store_pixel(P, x, lr, colour);
  }
  flush_counters(P, segs, tests);
}

// ---- tuned variant -----------------------------------------------------------------------------
//
// Exact cull (proof in DESIGN.md): with det = -dot(d,n) > 0 and inv = RN(1/det) > 0, the reference
// can only accept a triangle if none of these division-free rejections holds (when det >= 2^-60):
//   R6  num_t <  RN(det * 0.000999)           (then dist < 0.001)
//   R3  num_u < -RN(det * 2^-60)              (then u = RN(num_u*inv) < 0, no underflow to -0)
//   R4  num_v >  RN(det * 2^-60)              (then v < 0)
//   R5  RN(num_u - num_v) > RN(det * (1+2^-16))   (then w = 1-u-v < 0)
//   R7  num_t >  RN(best_k * det), best_k = RN(best * (1+2^-16))   (then dist >= best)
// A lane that passes the pre-test is only a candidate; the exact reference expression decides.
constexpr float kTiny = 8.673617379884035e-19f;   // 2^-60
constexpr float kOnePlus = 1.0000152587890625f;   // 1 + 2^-16
constexpr float kTMin = 0.000999f;

// Division-free part of one triangle test for one lane (all quantities exactly as the reference
// computes them, so the exact path below can reuse them).
struct TriPre {
  float num_t, num_u, num_v, det;
  bool cand;
};

// The 12 floats of a triangle record the test reads.
struct TriData {
  f3 a, e1, e2, n;
};

// Triangle sources: the std430 buffer read with wave-uniform addresses (-> SGPRs), or the LDS copy.
struct GlobalTris {
  const hrt_triangle* __restrict__ t;
  __device__ __forceinline__ TriData operator()(uint32_t i) const {
    const hrt_triangle& r = t[i];
    return {ld3(r.a), ld3(r.edge_one), ld3(r.edge_two), ld3(r.normal)};
  }
};
struct GlobalTris4 {  // whole 64-byte records (lets hipcc use wide s_loads)
  const float4* __restrict__ t;
  __device__ __forceinline__ TriData operator()(uint32_t i) const {
    const float4 A = t[4 * i], B = t[4 * i + 1], C = t[4 * i + 2], N = t[4 * i + 3];
    return {mk(A.x, A.y, A.z), mk(B.x, B.y, B.z), mk(C.x, C.y, C.z), mk(N.x, N.y, N.z)};
  }
};
// LDS image: 3 float4 per triangle = (a.xyz, n.x) (n.yz, e1.xy) (e1.z, e2.xyz)
struct LdsTris {
  const float4* t;
  __device__ __forceinline__ TriData operator()(uint32_t i) const {
    const float4 p = t[3 * i], q = t[3 * i + 1], r = t[3 * i + 2];
    return {mk(p.x, p.y, p.z), mk(q.z, q.w, r.x), mk(r.y, r.z, r.w), mk(p.w, q.x, q.y)};
  }
};

__device__ __forceinline__ TriPre tri_pre(const TriData& tri, f3 o, f3 d, float best_k) {
  TriPre r;
  const f3 n = tri.n;
  const float dn = dot(d, n);
  const f3 ao = o - tri.a;
  r.num_t = dot(ao, n);
  const f3 dao = cross(ao, d);
  r.num_u = dot(tri.e2, dao);
  r.num_v = dot(tri.e1, dao);
  r.det = -dn;
  const float tiny = r.det * kTiny;
  const bool reject = (r.num_t < r.det * kTMin) | (r.num_u < -tiny) | (r.num_v > tiny) |
                      ((r.num_u - r.num_v) > r.det * kOnePlus) | (r.num_t > best_k * r.det);
  r.cand = (dn < 0.0f) & (!reject | (r.det < kTiny));
  return r;
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

// G consecutive triangles: G pre-tests, then one wave-uniform branch into the exact path.  Within
// the group the exact tests run in buffer order against the updated closest hit (ties: first wins);
// best_k is only tightened between groups, which keeps the pre-test conservative.
template <int G, class Src>
__device__ __forceinline__ void tri_group(const Src& tris, uint32_t i0, uint32_t m, f3 o, f3 d,
                                          Closest& c, float& best_k) {
  TriPre q[G];
  bool any = false;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    q[g] = tri_pre(tris(i0 + g), o, d, best_k);
    any |= q[g].cand;
  }
  if (__builtin_expect(__any(any), 0)) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (G == 1 || __any(q[g].cand)) {
        if (q[g].cand) tri_exact(q[g], i0 + g, m, c, best_k);
      }
    }
  }
}

// Two-stage variant: stage 1 computes only ao and num_t (7 VALU) and skips the triangle when no
// lane has num_t > 0 (necessary for dist > 0.001 since inv_det > 0).  For primary rays all lanes share
// the origin, so num_t is wave-uniform and every triangle facing away from the camera is rejected
// here; stage 2 completes the same pre-test as tri_pre.
template <class Src>
__device__ __forceinline__ void tri_two_stage(const Src& tris, uint32_t i, uint32_t m, f3 o, f3 d, Closest& c,
                                              float& best_k) {
  const TriData tri = tris(i);
  const f3 ao = o - tri.a;
  TriPre q;
  q.num_t = dot(ao, tri.n);
  if (!__any(q.num_t > 0.0f)) return;
  const float dn = dot(d, tri.n);
  const f3 dao = cross(ao, d);
  q.num_u = dot(tri.e2, dao);
  q.num_v = dot(tri.e1, dao);
  q.det = -dn;
  const float tiny = q.det * kTiny;
  const bool reject = (q.num_t < q.det * kTMin) | (q.num_u < -tiny) | (q.num_v > tiny) |
                      ((q.num_u - q.num_v) > q.det * kOnePlus) | (q.num_t > best_k * q.det);
  q.cand = (dn < 0.0f) & (q.num_t > 0.0f) & (!reject | (q.det < kTiny));
  if (__builtin_expect(__any(q.cand), 0)) {
    if (q.cand) tri_exact(q, i, m, c, best_k);
  }
}

template <class Src>
__device__ __forceinline__ Closest world_hit_two_stage(const Scene& sc, const Src& src, const hrt_push_constants& pc,
                                                       f3 o, f3 d, uint32_t& tests) {
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  float best_k = c.t * kOnePlus;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = aabb_pass(mesh, o, d);
    tests += pass ? mesh.len : 0u;
    if (!pass) continue;
    const uint32_t end = mesh.first_index + mesh.len;
    for (uint32_t i = mesh.first_index; i < end; ++i) tri_two_stage(src, i, (uint32_t)m, o, d, c, best_k);
  }
  return c;
}

template <int G, class Src>
__device__ __forceinline__ Closest world_hit_tuned(const Scene& sc, const Src& src, const hrt_push_constants& pc,
                                                   f3 o, f3 d, uint32_t& tests) {
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
    uint32_t i = mesh.first_index;
    for (; i + G <= end; i += G) tri_group<G, Src>(src, i, (uint32_t)m, o, d, c, best_k);
    if (G > 1)
      for (; i < end; ++i) tri_group<1, Src>(src, i, (uint32_t)m, o, d, c, best_k);
  }
  return c;
}

// Fused sample/bounce loop: each lane runs its pixel's num_samples paths back to back
// (RNG state chains through them exactly as raytracing.glsl:379-385); the wave iterates until
// every lane's last path has ended.
template <int G, class Src, bool TwoStage = false>
__device__ __forceinline__ void trace_fused(const TraceParams& P, const Src& src, uint32_t x, uint32_t lr) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes};
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
      const Closest c = TwoStage ? world_hit_two_stage(sc, src, pc, p.pos, p.dir, tests)
                                 : world_hit_tuned<G>(sc, src, pc, p.pos, p.dir, tests);
      ++segs;
      const bool ended = shade_step(sc, pc, p, c, state);
      ++p.bounce;
      if (ended || p.bounce > pc.max_bounces) {
        colour = colour + p.light * p.colour;
        p.bounce = pc.max_bounces + 1;
      }
    }
    colour = colour / (float)pc.num_samples;
    store_pixel(P, x, lr, colour);
  }
  flush_counters(P, segs, tests);
}

template <int G>
__global__ __launch_bounds__(256) void trace_tuned(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<G>(P, GlobalTris{P.tris}, x, lr);
}

__global__ __launch_bounds__(256) void trace_tuned_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

// Whole scene resident in LDS (3 float4 per triangle), 1024-thread workgroups (16 waves, a 32x32
// pixel tile of 8x8 wave tiles): the copy is paid once per workgroup, every wave then streams the
// triangles from LDS with broadcast reads instead of scalar loads.
extern __shared__ float4 lds_tris[];
template <bool TwoStage>
__global__ __launch_bounds__(1024) void trace_lds(TraceParams P) {
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
  trace_fused<1, LdsTris, TwoStage>(P, LdsTris{lds_tris}, x, lr);
}

__global__ __launch_bounds__(256) void trace_two_stage_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1, GlobalTris4, true>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

// ---- init clear (raytracing.glsl:363-366) and image_combiner.glsl (:22-43) ----------------------
__global__ __launch_bounds__(256) void clear_kernel(uint32_t* img8, float4* img32, size_t npix) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  if (img8) img8[i] = 255u << 24;
  if (img32) img32[i] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
}

__global__ __launch_bounds__(256) void accumulate_rgba8(uint32_t* cur, const uint32_t* nw, size_t npix, uint32_t frame) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  if (frame == 0) {
    cur[i] = 255u << 24;
    return;
  }
  const float ff = (float)frame, ff1 = (float)(frame + 1u);
  const uint32_t pv = cur[i], nv = nw[i];
  uint32_t out = 255u << 24;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float prev = unorm8_to_float((pv >> (8 * ch)) & 255u);
    const float nc = unorm8_to_float((nv >> (8 * ch)) & 255u);
    out |= unorm8((nc + prev * ff) / ff1) << (8 * ch);
  }
  cur[i] = out;
}

__global__ __launch_bounds__(256) void accumulate_rgba32f(float4* cur, const float4* nw, size_t npix, uint32_t frame) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  if (frame == 0) {
    cur[i] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    return;
  }
  const float ff = (float)frame, ff1 = (float)(frame + 1u);
  const float4 p = cur[i], n = nw[i];
  cur[i] = make_float4((n.x + p.x * ff) / ff1, (n.y + p.y * ff) / ff1, (n.z + p.z * ff) / ff1, 1.0f);
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

}  // namespace hrt

// ---- launch wrappers (host) ----------------------------------------------------------------------
namespace hrt {

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + 255) / 256); }
constexpr size_t kMaxLdsScene = 160 * 1024;

hipError_t launch_trace(const TraceParams& p, int variant, hipStream_t stream) {
  static bool lds_attr = false;
  if (!lds_attr) {
    lds_attr = true;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&trace_lds<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&trace_lds<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene);
  }
  const dim3 grid((p.pc.width + 15) / 16, (p.local_rows + 15) / 16, 1);
  const size_t lds_bytes = (size_t)p.n_tris * 48;
  if (variant == 0) variant = 6;  // auto: two-stage test, scene in LDS when it fits
  if ((variant == 5 || variant == 6) && lds_bytes > kMaxLdsScene) variant = (variant == 6) ? 7 : 3;
  switch (variant) {
    case 1: trace_literal<<<grid, 256, 0, stream>>>(p); break;
    case 3: trace_tuned_f4<<<grid, 256, 0, stream>>>(p); break;
    case 4: trace_tuned<2><<<grid, 256, 0, stream>>>(p); break;
    case 5:
    case 6: {
      const dim3 g32((p.pc.width + 31) / 32, (p.local_rows + 31) / 32, 1);
      if (variant == 5)
        trace_lds<false><<<g32, 1024, lds_bytes, stream>>>(p);
      else
        trace_lds<true><<<g32, 1024, lds_bytes, stream>>>(p);
      break;
    }
    case 7: trace_two_stage_f4<<<grid, 256, 0, stream>>>(p); break;
    default: trace_tuned<1><<<grid, 256, 0, stream>>>(p); break;  // 2
  }
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
