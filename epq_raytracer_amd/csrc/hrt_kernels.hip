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

// Primary segments (origin = cam_pos for every active lane of the wave): iterate each mesh's
// camera-facing list only.  A triangle left out has num_t = dot(cam_pos - a, n) <= 0 (or NaN) -- the
// same value every primary lane would compute -- so no primary lane can accept it.
template <class Src, class List>
__device__ __forceinline__ Closest world_hit_primary(const Scene& sc, const Src& src, const List& list,
                                                     const TraceParams& P, f3 o, f3 d, uint32_t& tests) {
  const hrt_push_constants& pc = P.pc;
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
    const uint32_t k0 = P.cam_start[m], k1 = k0 + P.cam_count[m];
    for (uint32_t k = k0; k < k1; ++k) {
      const uint32_t i = list(k);
      const TriPre q = tri_pre(src(i), o, d, best_k);
      if (__builtin_expect(__any(q.cand), 0)) {
        if (q.cand) tri_exact(q, i, (uint32_t)m, c, best_k);
      }
    }
  }
  return c;
}

// Primary segments over the compacted camera-facing records (sequential wave-uniform loads, the
// original triangle index travels in a.w).
__device__ __forceinline__ Closest world_hit_primary_compact(const Scene& sc, const TraceParams& P, f3 o, f3 d,
                                                             uint32_t& tests) {
  const hrt_push_constants& pc = P.pc;
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  float best_k = c.t * kOnePlus;
  const float4* __restrict__ ct = P.cam_tris;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = aabb_pass(mesh, o, d);
    tests += pass ? mesh.len : 0u;
    if (!pass) continue;
    const uint32_t k0 = P.cam_start[m], k1 = k0 + P.cam_count[m];
    for (uint32_t k = k0; k < k1; ++k) {
      const float4 A = ct[4 * k], B = ct[4 * k + 1], C = ct[4 * k + 2], N = ct[4 * k + 3];
      const TriData td{mk(A.x, A.y, A.z), mk(B.x, B.y, B.z), mk(C.x, C.y, C.z), mk(N.x, N.y, N.z)};
      const TriPre q = tri_pre(td, o, d, best_k);
      if (__builtin_expect(__any(q.cand), 0)) {
        if (q.cand) tri_exact(q, __builtin_bit_cast(uint32_t, A.w), (uint32_t)m, c, best_k);
      }
    }
  }
  return c;
}

struct CompactTag {
  __device__ __forceinline__ uint32_t operator()(uint32_t) const { return 0u; }
};
struct CompactAoTag {
  __device__ __forceinline__ uint32_t operator()(uint32_t) const { return 0u; }
};

// Primary segments over compacted records carrying the precomputed ao = cam_pos - a and num_t
// (wave-uniform for primary rays).  Stage A: dn = dot(d, n); a triangle no lane approaches from its
// front (dn < 0 fails for every lane) cannot be accepted.  Stage B: the rest of the pre-test.
__device__ __forceinline__ Closest world_hit_primary_ao(const Scene& sc, const TraceParams& P, f3 o, f3 d,
                                                        uint32_t& tests) {
  const hrt_push_constants& pc = P.pc;
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  float best_k = c.t * kOnePlus;
  const float4* __restrict__ ct = P.cam_tris;
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = aabb_pass(mesh, o, d);
    tests += pass ? mesh.len : 0u;
    if (!pass) continue;
    const uint32_t k0 = P.cam_start[m], k1 = k0 + P.cam_count[m];
    for (uint32_t k = k0; k < k1; ++k) {
      const float4 N = ct[4 * k + 3];
      const f3 n = mk(N.x, N.y, N.z);
      const float dn = dot(d, n);
      if (!__any(dn < 0.0f)) continue;
      const float4 A = ct[4 * k], B = ct[4 * k + 1], C = ct[4 * k + 2];
      const f3 ao = mk(A.x, A.y, A.z);
      TriPre q;
      q.num_t = A.w;
      const f3 dao = cross(ao, d);
      q.num_u = dot(mk(C.x, C.y, C.z), dao);
      q.num_v = dot(mk(B.x, B.y, B.z), dao);
      q.det = -dn;
      const float tiny = q.det * kTiny;
      const bool reject = (q.num_t < q.det * kTMin) | (q.num_u < -tiny) | (q.num_v > tiny) |
                          ((q.num_u - q.num_v) > q.det * kOnePlus) | (q.num_t > best_k * q.det);
      q.cand = (dn < 0.0f) & (!reject | (q.det < kTiny));
      if (__builtin_expect(__any(q.cand), 0)) {
        if (q.cand) tri_exact(q, __builtin_bit_cast(uint32_t, B.w), (uint32_t)m, c, best_k);
      }
    }
  }
  return c;
}

// Batched form of world_hit_primary_ao: the stage-A loads (normals) of 4 consecutive compacted
// records are issued together so their latency overlaps; each triangle then branches into stage B
// on its own wave vote.  Rec is an accessor for the compacted records (global or LDS).
template <class Rec>
__device__ __forceinline__ void primary_stage_b(const Rec& rec, uint32_t k, float dn, f3 d, uint32_t m, Closest& c,
                                                float& best_k) {
  const float4 A = rec(4 * k), B = rec(4 * k + 1), C = rec(4 * k + 2);
  const f3 ao = mk(A.x, A.y, A.z);
  TriPre q;
  q.num_t = A.w;
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  const float tiny = q.det * kTiny;
  const bool reject = (q.num_t < q.det * kTMin) | (q.num_u < -tiny) | (q.num_v > tiny) |
                      ((q.num_u - q.num_v) > q.det * kOnePlus) | (q.num_t > best_k * q.det);
  q.cand = (dn < 0.0f) & (!reject | (q.det < kTiny));
  if (__builtin_expect(__any(q.cand), 0)) {
    if (q.cand) tri_exact(q, __builtin_bit_cast(uint32_t, B.w), m, c, best_k);
  }
}

template <class Rec>
__device__ __forceinline__ Closest world_hit_primary_batch(const Scene& sc, const Rec& rec, const TraceParams& P,
                                                           f3 o, f3 d, uint32_t& tests) {
  const hrt_push_constants& pc = P.pc;
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
    const uint32_t k0 = P.cam_start[m], k1 = k0 + P.cam_count[m];
    uint32_t k = k0;
    for (; k + 4 <= k1; k += 4) {
      const float4 N0 = rec(4 * k + 3), N1 = rec(4 * k + 7), N2 = rec(4 * k + 11), N3 = rec(4 * k + 15);
      const float dn0 = dot(d, mk(N0.x, N0.y, N0.z)), dn1 = dot(d, mk(N1.x, N1.y, N1.z));
      const float dn2 = dot(d, mk(N2.x, N2.y, N2.z)), dn3 = dot(d, mk(N3.x, N3.y, N3.z));
      if (__any(dn0 < 0.0f)) primary_stage_b(rec, k, dn0, d, (uint32_t)m, c, best_k);
      if (__any(dn1 < 0.0f)) primary_stage_b(rec, k + 1, dn1, d, (uint32_t)m, c, best_k);
      if (__any(dn2 < 0.0f)) primary_stage_b(rec, k + 2, dn2, d, (uint32_t)m, c, best_k);
      if (__any(dn3 < 0.0f)) primary_stage_b(rec, k + 3, dn3, d, (uint32_t)m, c, best_k);
    }
    for (; k < k1; ++k) {
      const float4 N = rec(4 * k + 3);
      const float dn = dot(d, mk(N.x, N.y, N.z));
      if (__any(dn < 0.0f)) primary_stage_b(rec, k, dn, d, (uint32_t)m, c, best_k);
    }
  }
  return c;
}

struct GlobalRec {
  const float4* __restrict__ r;
  __device__ __forceinline__ float4 operator()(uint32_t j) const { return r[j]; }
};
struct LdsRec {
  const float4* r;
  __device__ __forceinline__ float4 operator()(uint32_t j) const { return r[j]; }
};
struct BatchGlobalTag {
  __device__ __forceinline__ uint32_t operator()(uint32_t) const { return 0u; }
};
struct BatchLdsTag {
  const float4* r;
  __device__ __forceinline__ uint32_t operator()(uint32_t) const { return 0u; }
};

struct GlobalList {
  const uint32_t* __restrict__ l;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return l[k]; }
};
struct LdsList {
  const uint32_t* l;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return l[k]; }
};

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
struct NoList {
  __device__ __forceinline__ uint32_t operator()(uint32_t) const { return 0u; }
};

template <int G, class Src, bool TwoStage = false, class List = NoList>
__device__ __forceinline__ void trace_fused(const TraceParams& P, const Src& src, uint32_t x, uint32_t lr,
                                            const List& list = List()) {
  constexpr bool kCamList = !__is_same(List, NoList);
  constexpr bool kCompact = __is_same(List, CompactTag);
  constexpr bool kCompactAo = __is_same(List, CompactAoTag);
  constexpr bool kBatchG = __is_same(List, BatchGlobalTag);
  constexpr bool kBatchL = __is_same(List, BatchLdsTag);
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
      Closest c;
      if constexpr (kBatchG) {
        if (__all(p.bounce == 0))
          c = world_hit_primary_batch(sc, GlobalRec{P.cam_tris}, P, p.pos, p.dir, tests);
        else
          c = world_hit_two_stage(sc, src, pc, p.pos, p.dir, tests);
      } else if constexpr (kBatchL) {
        if (__all(p.bounce == 0))
          c = world_hit_primary_batch(sc, LdsRec{list.r}, P, p.pos, p.dir, tests);
        else
          c = world_hit_two_stage(sc, src, pc, p.pos, p.dir, tests);
      } else if (kCompactAo && __all(p.bounce == 0))
        c = world_hit_primary_ao(sc, P, p.pos, p.dir, tests);
      else if (kCompact && __all(p.bounce == 0))
        c = world_hit_primary_compact(sc, P, p.pos, p.dir, tests);
      else if (kCamList && !kCompact && !kCompactAo && !kBatchG && !kBatchL && __all(p.bounce == 0))
        c = world_hit_primary(sc, src, list, P, p.pos, p.dir, tests);
      else if (TwoStage)
        c = world_hit_two_stage(sc, src, pc, p.pos, p.dir, tests);
      else
        c = world_hit_tuned<G>(sc, src, pc, p.pos, p.dir, tests);
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
template <bool TwoStage, bool CamList = false>
__global__ __launch_bounds__(1024) void trace_lds(TraceParams P) {
  const uint32_t n = P.n_tris;
  uint32_t* lds_list = reinterpret_cast<uint32_t*>(lds_tris + 3 * n);
  if (CamList)
    for (uint32_t k = threadIdx.x; k < P.cam_list_capacity; k += blockDim.x) lds_list[k] = P.cam_list[k];
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
  if (CamList)
    trace_fused<1, LdsTris, TwoStage, LdsList>(P, LdsTris{lds_tris}, x, lr, LdsList{lds_list});
  else
    trace_fused<1, LdsTris, TwoStage>(P, LdsTris{lds_tris}, x, lr);
}

__global__ __launch_bounds__(256) void trace_camlist_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1, GlobalTris4, true, GlobalList>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr,
                                                GlobalList{P.cam_list});
}

__global__ __launch_bounds__(256) void trace_camcompact_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1, GlobalTris4, true, CompactTag>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr,
                                                CompactTag{});
}

__global__ __launch_bounds__(256) void trace_camao_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1, GlobalTris4, true, CompactAoTag>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr,
                                                  CompactAoTag{});
}

__global__ __launch_bounds__(256) void trace_batch_f4(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused<1, GlobalTris4, true, BatchGlobalTag>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr,
                                                    BatchGlobalTag{});
}

// Compacted camera-facing records resident in LDS (64 B each), the generic path on scalar loads.
__global__ __launch_bounds__(1024) void trace_batch_lds(TraceParams P) {
  const uint32_t nrec = 4 * P.cam_list_capacity;
  for (uint32_t k = threadIdx.x; k < nrec; k += blockDim.x) lds_tris[k] = P.cam_tris[k];
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t x = blockIdx.x * 32 + (wave & 3) * 8 + (lane & 7);
  const uint32_t lr = blockIdx.y * 32 + (wave >> 2) * 8 + (lane >> 3);
  trace_fused<1, GlobalTris4, true, BatchLdsTag>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr,
                                                 BatchLdsTag{lds_tris});
}

// ---- variant 14: primary-ray bundle culling -------------------------------------------------------
//
// For a primary segment every lane's ray starts at cam_pos, so for a fixed triangle the reference's
// det = -d.n, num_u = d.(e2 x ao) and num_v = d.(e1 x ao) are LINEAR in the lane's direction d
// (ao = cam_pos - a is shared).  Bounding d over the wave's directions (axis a, cos range [c_lo,c_hi],
// sine bound s_hi) bounds each linear form; a triangle is rejected for the whole wave when
//   R1  min d.n            > m_n   (every lane: dn >= 0, raytracing.glsl:217)
//   R3  max d.(e2 x ao)    < -m_u  (every lane: u < 0)
//   R4  min d.(e1 x ao)    > m_v   (every lane: v < 0)
//   R5  min d.(g_u-h+n)    > m_w   (every lane: num_u - num_v > det(1+2^-16), so u, v or w < 0)
// with margins m_* = 1e-5 * (product norms) + 2^-40|n| (+2^-14|n| for R5) covering the rounding of the
// reference's own dot/cross sequence (<= ~10 eps * product norm) and of these bounds.  The cull runs
// lane-parallel: lane j bounds triangle base+j, so 64 triangles cost one pass.  Survivors (in buffer
// order) get the exact per-lane test.
struct Bundle {
  f3 a;
  float c_lo, c_hi, s_hi;
};

__device__ __forceinline__ float wave_min_all(float v) {  // all 64 lanes active
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ float lin_lower(float ga, float gn, const Bundle& b) {
  return fminf(b.c_lo * ga, b.c_hi * ga) - b.s_hi * gn;
}
__device__ __forceinline__ float lin_upper(float ga, float gn, const Bundle& b) {
  return fmaxf(b.c_lo * ga, b.c_hi * ga) + b.s_hi * gn;
}

// Primary segments of the lanes with prim == true.  Called with ALL 64 lanes of the wave active.
__device__ __forceinline__ void world_hit_bundle(const Scene& sc, const TraceParams& P, bool prim, f3 o, f3 d,
                                                 uint32_t& tests, Closest& c) {
  const hrt_push_constants& pc = P.pc;
  const unsigned long long pm = __ballot(prim);
  const int lead = __builtin_ctzll(pm);
  Bundle b;
  b.a = mk(__shfl(d.x, lead, 64), __shfl(d.y, lead, 64), __shfl(d.z, lead, 64));
  const float lam = prim ? dot(d, b.a) : 3.0f;
  b.c_lo = wave_min_all(lam) - 1e-5f;
  b.c_hi = 1.00001f;
  b.s_hi = (b.c_lo > 0.0f) ? __builtin_sqrtf(fmaxf(0.0f, 1.00002f - b.c_lo * b.c_lo)) * 1.00001f + 1e-6f : 1.00001f;
  if (prim) {
    c = Closest{kFltMax, 0, 0u, 0u};
    for (int i = 0; i < pc.num_spheres; ++i) {
      const float t = sphere_dist(sc.spheres[i], o, d);
      if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
    }
  }
  float best_k = c.t * kOnePlus;
  const float4* __restrict__ ct = P.cam_tris;
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
      while (mask) {
        const uint32_t j = __builtin_ctzll(mask);
        mask &= mask - 1ull;
        const uint32_t kk = base + j;
        if (pass) {
          const float4 N = ct[4 * kk + 3];
          const float dn = dot(d, mk(N.x, N.y, N.z));
          if (__any(dn < 0.0f)) primary_stage_b(GlobalRec{ct}, kk, dn, d, (uint32_t)m, c, best_k);
        }
      }
    }
  }
}

// Bounce-path world_hit with the next triangle's 64-byte record loaded (wave-uniform, into SGPRs)
// while the current one is tested: the loop no longer waits a full scalar-load latency per triangle.
__device__ __forceinline__ void tri_two_stage_rec(const float4& A, const float4& B, const float4& C, const float4& N,
                                                  uint32_t i, uint32_t m, f3 o, f3 d, Closest& c, float& best_k) {
  const f3 n = mk(N.x, N.y, N.z);
  const f3 ao = o - mk(A.x, A.y, A.z);
  TriPre q;
  q.num_t = dot(ao, n);
  if (!__any(q.num_t > 0.0f)) return;
  const float dn = dot(d, n);
  const f3 dao = cross(ao, d);
  q.num_u = dot(mk(C.x, C.y, C.z), dao);
  q.num_v = dot(mk(B.x, B.y, B.z), dao);
  q.det = -dn;
  const float tiny = q.det * kTiny;
  const bool reject = (q.num_t < q.det * kTMin) | (q.num_u < -tiny) | (q.num_v > tiny) |
                      ((q.num_u - q.num_v) > q.det * kOnePlus) | (q.num_t > best_k * q.det);
  q.cand = (dn < 0.0f) & (q.num_t > 0.0f) & (!reject | (q.det < kTiny));
  if (__builtin_expect(__any(q.cand), 0)) {
    if (q.cand) tri_exact(q, i, m, c, best_k);
  }
}

__device__ __forceinline__ Closest world_hit_prefetch(const Scene& sc, const hrt_push_constants& pc, f3 o, f3 d,
                                                      uint32_t& tests) {
  Closest c{kFltMax, 0, 0u, 0u};
  for (int i = 0; i < pc.num_spheres; ++i) {
    const float t = sphere_dist(sc.spheres[i], o, d);
    if (t > 0.001f && t < c.t) c = Closest{t, 1, (uint32_t)i, 0u};
  }
  float best_k = c.t * kOnePlus;
  const float4* __restrict__ T = reinterpret_cast<const float4*>(sc.tris);
  for (int m = 0; m < pc.num_meshes; ++m) {
    const hrt_mesh& mesh = sc.meshes[m];
    const bool pass = aabb_pass(mesh, o, d);
    tests += pass ? mesh.len : 0u;
    if (!pass) continue;
    const uint32_t first = mesh.first_index, end = first + mesh.len;
    if (first >= end) continue;
    float4 A = T[4 * first], B = T[4 * first + 1], C = T[4 * first + 2], N = T[4 * first + 3];
    for (uint32_t i = first; i < end; ++i) {
      const uint32_t nx = (i + 1 < end) ? i + 1 : i;  // in-bounds prefetch of the next record
      const float4 A1 = T[4 * nx], B1 = T[4 * nx + 1], C1 = T[4 * nx + 2], N1 = T[4 * nx + 3];
      tri_two_stage_rec(A, B, C, N, i, (uint32_t)m, o, d, c, best_k);
      A = A1; B = B1; C = C1; N = N1;
    }
  }
  return c;
}

template <class Src, bool Prefetch = false>
__device__ __forceinline__ void trace_fused_split(const TraceParams& P, const Src& src, uint32_t x, uint32_t lr) {
  const Scene sc{P.rays, P.spheres, P.tris, P.meshes};
  const hrt_push_constants& pc = P.pc;
  const uint32_t y = global_row(lr, P);
  uint32_t segs = 0, tests = 0;
  const bool active = x < pc.width && lr < P.local_rows && y < pc.height;
  const uint32_t id = active ? x + y * pc.width : 0u;
  f3 colour = mk(0.0f, 0.0f, 0.0f);
  uint32_t state = pc.rng_offset * 719393u + id;
  f3 centre = mk(0.0f, 0.0f, 0.0f);
  if (active) {
    const float4 rc = sc.rays[id];
    centre = mk(rc.x, rc.y, rc.z);
  }
  const f3 root = mk(pc.cam_pos[0], pc.cam_pos[1], pc.cam_pos[2]);
  int sample = 0;
  Path p;
  p.bounce = pc.max_bounces + 1;
  bool done = !active;
  // every lane stays in the loop until the whole wave is done (full-wave region at the loop top)
  while (__any(!done)) {
    if (!done && p.bounce > pc.max_bounces) {
      if (sample >= pc.num_samples) {
        done = true;
      } else {
        ++sample;
        const f3 dir = get_ray_dir(pc, centre, state);
        p = Path{mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), root, normalize(dir), 0, true};
      }
    }
    const bool prim = !done && p.bounce == 0;
    const bool sec_ready = !done && p.bounce != 0;
    // Deferred secondaries: a lane whose next segment is a bounce waits (its state untouched) until
    // at least sec_batch lanes are waiting or no primary lane is left, so the brute-force bounce
    // path runs on well-filled waves.  Per-pixel order of work is unchanged.
    const uint32_t nsec = (uint32_t)__popcll(__ballot(sec_ready));
    const bool any_prim = __any(prim);
    const bool run_sec = nsec > 0 && (nsec >= P.sec_batch || !any_prim);
    const bool sec = sec_ready && run_sec;
    Closest c{kFltMax, 0, 0u, 0u};
    if (any_prim) world_hit_bundle(sc, P, prim, p.pos, p.dir, tests, c);
    if (run_sec) {
      if (sec) {
        if constexpr (Prefetch)
          c = world_hit_prefetch(sc, pc, p.pos, p.dir, tests);
        else
          c = world_hit_two_stage(sc, src, pc, p.pos, p.dir, tests);
      }
    }
    if (prim || sec) {
      ++segs;
      const bool ended = shade_step(sc, pc, p, c, state);
      ++p.bounce;
      if (ended || p.bounce > pc.max_bounces) {
        colour = colour + p.light * p.colour;
        p.bounce = pc.max_bounces + 1;
      }
    }
  }
  if (active) {
    colour = colour / (float)pc.num_samples;
    store_pixel(P, x, lr, colour);
  }
  flush_counters(P, segs, tests);
}

__global__ __launch_bounds__(256) void trace_bundle(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused_split(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

__global__ __launch_bounds__(256) void trace_bundle_pf(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused_split<GlobalTris4, true>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

__global__ __launch_bounds__(256, 8) void trace_bundle_pf8(TraceParams P) {
  uint32_t x, lr;
  lane_pixel(P, x, lr);
  trace_fused_split<GlobalTris4, true>(P, GlobalTris4{reinterpret_cast<const float4*>(P.tris)}, x, lr);
}

// Per-frame prep for the camera-facing lists: one workgroup per mesh, order-preserving compaction
// of the mesh's triangles with num_t(cam_pos) > 0, computed exactly as the trace kernel does.
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
    if (k < mesh.len) {
      const hrt_triangle& t = P.tris[mesh.first_index + k];
      const f3 ao = o - ld3(t.a);
      keep = dot(ao, ld3(t.normal)) > 0.0f;
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
      P.cam_list[dst] = idx;
      if (P.cam_tris) {
        const float4* src = reinterpret_cast<const float4*>(P.tris) + 4 * (size_t)idx;
        float4* out = P.cam_tris + 4 * (size_t)dst;
        if (P.cam_layout == 1) {
          // (ao, num_t) (e1, idx) (e2, -) (n, -): ao and num_t exactly as a primary lane computes them
          const hrt_triangle& t = P.tris[idx];
          const f3 ao = o - ld3(t.a);
          const float nt = dot(ao, ld3(t.normal));
          out[0] = make_float4(ao.x, ao.y, ao.z, nt);
          float4 e1 = src[1];
          e1.w = __builtin_bit_cast(float, idx);
          out[1] = e1;
        } else {
          float4 a = src[0];
          a.w = __builtin_bit_cast(float, idx);
          out[0] = a;
          out[1] = src[1];
        }
        out[2] = src[2];
        out[3] = src[3];
        if (P.cam_cull) {
          const hrt_triangle& t = P.tris[idx];
          const f3 ao = o - ld3(t.a);
          const f3 n = ld3(t.normal), e1 = ld3(t.edge_one), e2 = ld3(t.edge_two);
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
      }
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
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&trace_lds<true, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&trace_batch_lds),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsScene);
  }
  const dim3 grid((p.pc.width + 15) / 16, (p.local_rows + 15) / 16, 1);
  const size_t lds_bytes = (size_t)p.n_tris * 48;
  if (variant == 0) variant = 14;  // auto: primary bundle cull + deferred two-stage bounce path
  const size_t lds_list_bytes = lds_bytes + (size_t)p.cam_list_capacity * 4;
  if (variant == 8 && lds_list_bytes > kMaxLdsScene) variant = 9;
  if ((variant == 5 || variant == 6) && lds_bytes > kMaxLdsScene) variant = (variant == 6) ? 7 : 3;
  const size_t lds_rec_bytes = (size_t)p.cam_list_capacity * 64;
  if (variant == 12 && lds_rec_bytes > kMaxLdsScene) variant = 13;
  if (variant >= 8 && variant <= 16 && p.pc.num_meshes > 0) {
    TraceParams q = p;
    if (variant == 8 || variant == 9) q.cam_tris = nullptr;
    q.cam_layout = (variant >= 11) ? 1u : 0u;
    if (variant < 14) q.cam_cull = nullptr;
    camera_lists<<<p.pc.num_meshes, 256, 0, stream>>>(q);
  }
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
    case 8: {
      const dim3 g32((p.pc.width + 31) / 32, (p.local_rows + 31) / 32, 1);
      trace_lds<true, true><<<g32, 1024, lds_list_bytes, stream>>>(p);
      break;
    }
    case 9: trace_camlist_f4<<<grid, 256, 0, stream>>>(p); break;
    case 10: trace_camcompact_f4<<<grid, 256, 0, stream>>>(p); break;
    case 11: trace_camao_f4<<<grid, 256, 0, stream>>>(p); break;
    case 12: {
      const dim3 g32((p.pc.width + 31) / 32, (p.local_rows + 31) / 32, 1);
      trace_batch_lds<<<g32, 1024, lds_rec_bytes, stream>>>(p);
      break;
    }
    case 13: trace_batch_f4<<<grid, 256, 0, stream>>>(p); break;
    case 14: trace_bundle<<<grid, 256, 0, stream>>>(p); break;
    case 15: trace_bundle_pf<<<grid, 256, 0, stream>>>(p); break;
    case 16: trace_bundle_pf8<<<grid, 256, 0, stream>>>(p); break;
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
