/*
 * oracle/rt_oracle.c -- CPU restatement of hindlet/EPQ_Raytracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (epq_raytracer_amd/, libhip_raytrace.so) never links it.
 *
 * PARITY STATUS: "parity unpinned" against the GLSL path itself.  The reference is
 * Rust + Vulkan (vulkano 0.33) and cannot be built or run in this container (no
 * cargo/rustc, no glslang, no Vulkan ICD; git deps rust_maths@992a952d and
 * rust_vulkan_graphics@b3c6a9c4 are not vendored -- SURVEY.md 8(c)).  The reference
 * ships no tests, golden images or fixtures.  What IS pinned:
 *   - the integer RNG (assets/raytracing.glsl:13-25) against the known-answer
 *     vectors derived in SURVEY.md 8(c) (tests/test_oracle.py);
 *   - analytic known-answer cases for every intersection routine;
 *   - the GLSL-unpinned floating-point choices, each fixed below and in DESIGN.md
 *     ("numerics spec"), so that the HIP kernels can be held to it bit for bit.
 *
 * Numerics spec (shared contract with the HIP kernels, restated independently there):
 *   S1  all arithmetic is IEEE binary32, round-to-nearest-even, denormals kept;
 *   S2  dot(a,b)   = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
 *       cross(a,b) = (fma(a.y,b.z,-(a.z*b.y)), fma(a.z,b.x,-(a.x*b.z)), fma(a.x,b.y,-(a.y*b.x)))
 *       mat3(M)*c  = per row i: fma(M[2][i],c.z, fma(M[1][i],c.y, M[0][i]*c.x))   (M column-major)
 *   S3  no other contraction: every other expression is evaluated exactly as written
 *       in the GLSL, left to right;
 *   S4  '/' and sqrt are correctly rounded; normalize(v) = v / sqrt(dot(v,v)) (3 divides);
 *   S5  log/sin/cos are the fixed polynomial algorithms spec_logf/spec_sinf/spec_cosf below;
 *   S6  GLSL min(x,y) = (y<x)?y:x, max(x,y) = (x<y)?y:x (GLSL 4.60 8.3 definitions);
 *       mix(x,y,a) = x*(1-a) + y*a; reflect(I,N) = I - (2*dot(N,I))*N;
 *   S7  rgba8 UNORM store: NaN and x<=0 -> 0, x>=1 -> 255, else rint(x*255) (RNE);
 *       UNORM load: k/255 (correctly rounded);
 *   S8  host-side (Rust) arithmetic has no contraction at all: Vector3::cross is
 *       a.y*b.z - a.z*b.y ..., magnitude = sqrt((x*x + y*y) + z*z), normalised = v / magnitude.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp).
 *
 * Parity-risk variants (oracle/Makefile liborc_drv_*.so; tests/test_parity_risk.py):
 * what a Vulkan driver typically emits where the GLSL leaves the choice open, one choice at a time --
 *   ORC_DRIVER_MATH      log/sin/cos from the C library (glibc logf/sinf/cosf) instead of S5;
 *   ORC_DRIVER_RSQ       normalize(v) = v * (1/sqrt(dot(v,v))) instead of S4's three divides;
 *   -ffp-contract=fast   the compiler fuses a*b+c wherever it likes (instead of S3).
 * They measure how far "bit-exact against this oracle" can sit from a real driver's frame; they
 * are never the checker.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_FLT_MAX 3.402823466e+38f /* assets/raytracing.glsl:2 */

/* ---------------------------------------------------------------------------------
 * std430 records (assets/raytracing.glsl:51-111), restated independently of include/.
 * ------------------------------------------------------------------------------- */
typedef struct { float colour[4], emission[4], settings[4]; } orc_material;          /* 48 B */
typedef struct { float sample_centre[4]; } orc_ray;                                  /* 16 B */
typedef struct { float centre[3]; float radius; orc_material material; } orc_sphere; /* 64 B */
typedef struct { float a[4], edge_one[4], edge_two[4], normal[4]; } orc_triangle;    /* 64 B */
typedef struct {
  float min_point[3]; uint32_t first_index;
  float max_point[3]; uint32_t len;
  orc_material material;
} orc_mesh;                                                                          /* 80 B */
/* push constants, assets/raytracing.glsl:135-153 / src/raytrace_pipeline.rs:125-139 (124 B) */
typedef struct {
  float cam_pos[4];
  float cam_alignment_mat[16]; /* column-major */
  int32_t num_rays, num_spheres, num_meshes, num_samples;
  float jitter_size;
  int32_t max_bounces;
  uint32_t use_environment_light, rng_offset, init, width, height;
} orc_push;

typedef struct { float x, y, z; } v3;

_Static_assert(sizeof(orc_material) == 48, "material");
_Static_assert(sizeof(orc_sphere) == 64, "sphere");
_Static_assert(sizeof(orc_triangle) == 64, "triangle");
_Static_assert(sizeof(orc_mesh) == 80, "mesh");
_Static_assert(sizeof(orc_push) == 124, "push");

static inline v3 mk3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls3(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
static inline v3 divs3(v3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
static inline v3 adds3(v3 a, float s) { return mk3(a.x + s, a.y + s, a.z + s); }
/* S2 */
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross3(v3 a, v3 b) {
  return mk3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
/* S4 */
#ifdef ORC_DRIVER_RSQ
static inline v3 normalize3(v3 a) { float r = 1.0f / sqrtf(dot3(a, a)); return muls3(a, r); }
#else
static inline v3 normalize3(v3 a) { float l = sqrtf(dot3(a, a)); return divs3(a, l); }
#endif
/* S6 */
static inline float glsl_min(float x, float y) { return (y < x) ? y : x; }
static inline float glsl_max(float x, float y) { return (x < y) ? y : x; }

/* ---------------------------------------------------------------------------------
 * S5: pinned transcendentals.  Range reduction + minimax polynomials (Cephes-style
 * coefficients), every step an explicit mul / add / fma so any IEEE binary32 machine
 * reproduces the bits.
 * ------------------------------------------------------------------------------- */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float spec_logf(float x) {
  uint32_t ix = f2u(x);
  if (x != x) return x;                     /* NaN */
  if (x == 0.0f) return -INFINITY;          /* log(+-0) = -inf */
  if (ix >> 31) return u2f(0x7fc00000u);    /* x < 0 -> NaN */
  if (ix == 0x7f800000u) return x;          /* +inf */
  int k = 0;
  if (ix < 0x00800000u) { x = x * 8388608.0f; ix = f2u(x); k = -23; } /* denormal: scale by 2^23 */
  ix += 0x3f800000u - 0x3f3504f3u;
  k += (int)(ix >> 23) - 0x7f;
  ix = (ix & 0x007fffffu) + 0x3f3504f3u;    /* m in [sqrt(1/2), sqrt(2)) */
  float f = u2f(ix) - 1.0f;                 /* exact (Sterbenz) */
  float z = f * f;
  float p = 7.0376836292e-2f;
  p = fmaf(p, f, -1.1514610310e-1f);
  p = fmaf(p, f, 1.1676998740e-1f);
  p = fmaf(p, f, -1.2420140846e-1f);
  p = fmaf(p, f, 1.4249322787e-1f);
  p = fmaf(p, f, -1.6668057665e-1f);
  p = fmaf(p, f, 2.0000714765e-1f);
  p = fmaf(p, f, -2.4999993993e-1f);
  p = fmaf(p, f, 3.3333331174e-1f);
  float y = (p * f) * z;
  float fk = (float)k;
  y = fmaf(fk, -2.12194440e-4f, y);
  y = fmaf(z, -0.5f, y);
  float r = f + y;
  return fmaf(fk, 0.693359375f, r);
}

/* shared range reduction for sin/cos: x = q*(pi/2) + r, |r| <= ~pi/4 */
static inline float spec_reduce(float x, int* q) {
  float j = rintf(x * 0.636619772367581343f);
  *q = (int)j;
  float r = fmaf(-j, 1.5703125f, x);
  r = fmaf(-j, 4.837512969970703125e-4f, r);
  r = fmaf(-j, 7.549789954891882e-8f, r);
  return r;
}
static inline float spec_sin_poly(float r) {
  float z = r * r;
  float p = -1.9515295891e-4f;
  p = fmaf(p, z, 8.3321608736e-3f);
  p = fmaf(p, z, -1.6666654611e-1f);
  return fmaf(p * z, r, r);
}
static inline float spec_cos_poly(float r) {
  float z = r * r;
  float p = 2.443315711809948e-5f;
  p = fmaf(p, z, -1.388731625493765e-3f);
  p = fmaf(p, z, 4.166664568298827e-2f);
  return fmaf(p * z, z, fmaf(z, -0.5f, 1.0f));
}
float spec_sinf(float x) {
  if (!(fabsf(x) <= 1.0e5f)) return (x != x) ? x : u2f(0x7fc00000u); /* NaN/inf/huge: NaN */
  int q; float r = spec_reduce(x, &q);
  switch (q & 3) {
    case 0: return spec_sin_poly(r);
    case 1: return spec_cos_poly(r);
    case 2: return -spec_sin_poly(r);
    default: return -spec_cos_poly(r);
  }
}
float spec_cosf(float x) {
  if (!(fabsf(x) <= 1.0e5f)) return (x != x) ? x : u2f(0x7fc00000u);
  int q; float r = spec_reduce(x, &q);
  switch (q & 3) {
    case 0: return spec_cos_poly(r);
    case 1: return -spec_sin_poly(r);
    case 2: return -spec_cos_poly(r);
    default: return spec_sin_poly(r);
  }
}

#ifdef ORC_DRIVER_MATH
#define ORC_LOGF logf
#define ORC_SINF sinf
#define ORC_COSF cosf
#else
#define ORC_LOGF spec_logf
#define ORC_SINF spec_sinf
#define ORC_COSF spec_cosf
#endif

/* ---------------------------------------------------------------------------------
 * RNG -- assets/raytracing.glsl:13-40
 * ------------------------------------------------------------------------------- */
/* hash, raytracing.glsl:13-21 */
static inline uint32_t orc_hash(uint32_t* state) {
  uint32_t s = *state;
  s ^= 2747636419u;
  s *= 2654435769u;
  s ^= s >> 16;
  s *= 2654435769u;
  s ^= s >> 16;
  s *= 2654435769u;
  *state = s;
  return s;
}
/* scaleToRange01, raytracing.glsl:23-25: state / float(4294967295.0) == float(state) / 2^32 */
static inline float orc_u01(uint32_t s) { return (float)s / 4294967296.0f; }
/* RandomValueNormalDistribution, raytracing.glsl:28-33 (u1 then u2) */
static inline float orc_normal(uint32_t* state) {
  float theta = 6.2831852f * orc_u01(orc_hash(state)); /* 2 * 3.1415926, folded exactly */
  float rho = sqrtf(-2.0f * ORC_LOGF(orc_u01(orc_hash(state))));
  return rho * ORC_COSF(theta);
}
/* RandomPointOnUnitSphere, raytracing.glsl:35-40 (x, y, z order) */
static inline v3 orc_unit_sphere(uint32_t* state) {
  float x = orc_normal(state);
  float y = orc_normal(state);
  float z = orc_normal(state);
  return normalize3(mk3(x, y, z));
}

/* exported for KATs */
uint32_t orc_hash_step(uint32_t* state) { return orc_hash(state); }
float orc_scale01(uint32_t s) { return orc_u01(s); }
float orc_normal_dist(uint32_t* state) { return orc_normal(state); }
void orc_point_on_sphere(uint32_t* state, float out[3]) {
  v3 p = orc_unit_sphere(state); out[0] = p.x; out[1] = p.y; out[2] = p.z;
}

/* ---------------------------------------------------------------------------------
 * Intersections -- assets/raytracing.glsl:158-288
 * ------------------------------------------------------------------------------- */
typedef struct {
  v3 hit_normal, hit_pos;
  float hit_dist;
  const orc_material* hit_mat; /* NULL = empty_mat() (raytracing.glsl:57-63) */
} orc_hit;

static inline orc_hit empty_hit(void) { /* raytracing.glsl:104-111 */
  orc_hit h; h.hit_normal = mk3(0, 0, 0); h.hit_pos = mk3(0, 0, 0); h.hit_dist = ORC_FLT_MAX; h.hit_mat = NULL;
  return h;
}

/* ray_at, raytracing.glsl:158-160 */
static inline v3 ray_at(v3 o, v3 d, float t) { return add3(o, muls3(d, t)); }

/* intersecting_sphere, raytracing.glsl:169-190 */
static orc_hit intersecting_sphere(const orc_sphere* s, v3 o, v3 d) {
  v3 l = sub3(o, ld3(s->centre));
  float a = dot3(d, d);
  float half_b = dot3(d, l);
  float c = dot3(l, l) - s->radius * s->radius;
  float disc = half_b * half_b - a * c;
  if (disc >= 0.0f) {
    float dist = (-half_b - sqrtf(disc)) / a;
    v3 pos = ray_at(o, d, dist);
    orc_hit h; h.hit_normal = normalize3(sub3(pos, ld3(s->centre))); h.hit_pos = pos;
    h.hit_dist = dist; h.hit_mat = &s->material;
    return h;
  }
  return empty_hit();
}

/* intersecting_aabb, raytracing.glsl:192-210 -- restated with its quirks (min/max mix-up at :202,:206) */
int orc_intersecting_aabb(const float mn[3], const float mx[3], const float op[3], const float dp[3]) {
  v3 o = ld3(op), d = ld3(dp);
  v3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float d_max, d_min;
  d_max = (((inv.x < 0.0f) ? mn[0] : mx[0]) - o.x) * inv.x;
  d_min = (((inv.x < 0.0f) ? mx[0] : mn[0]) - o.x) * inv.x;
  if (d_max > 0.0f || d_min > 0.0f) return 1;
  d_max = glsl_max(d_max, (((inv.y < 0.0f) ? mn[1] : mx[1]) - o.y) * inv.y);
  d_min = glsl_min(d_max, (((inv.y < 0.0f) ? mx[1] : mn[1]) - o.y) * inv.y);
  if (d_max > 0.0f || d_min > 0.0f) return 1;
  d_max = glsl_max(d_max, (((inv.z < 0.0f) ? mn[2] : mx[2]) - o.z) * inv.z);
  d_min = glsl_max(d_min, (((inv.z < 0.0f) ? mx[2] : mn[2]) - o.z) * inv.z);
  if (d_max > 0.0f || d_min > 0.0f) return 1;
  return 0;
}

/* intersecting_tri, raytracing.glsl:213-241; returns (normal, dist) in out[4] */
static inline void intersecting_tri(const orc_triangle* t, v3 o, v3 d, float out[4]) {
  v3 n = ld3(t->normal);
  if (dot3(d, n) >= 0.0f) { out[0] = out[1] = out[2] = 0.0f; out[3] = ORC_FLT_MAX; return; }
  v3 ao = sub3(o, ld3(t->a));
  v3 dao = cross3(ao, d);
  float det = -dot3(d, n);
  if (det == 0.0f) goto miss;
  float inv_det = 1.0f / det;
  float dist = dot3(ao, n) * inv_det;
  if (dist < 0.0f) goto miss;
  float u = dot3(ld3(t->edge_two), dao) * inv_det;
  if (u < 0.0f) goto miss;
  float v = -dot3(ld3(t->edge_one), dao) * inv_det;
  if (v < 0.0f) goto miss;
  float w = 1.0f - u - v;
  if (w < 0.0f) goto miss;
  { v3 nn = normalize3(n); out[0] = nn.x; out[1] = nn.y; out[2] = nn.z; out[3] = dist; }
  return;
miss:
  out[0] = out[1] = out[2] = out[3] = ORC_FLT_MAX;
}

void orc_intersecting_tri(const orc_triangle* t, const float o[3], const float d[3], float out[4]) {
  intersecting_tri(t, ld3(o), ld3(d), out);
}

typedef struct {
  const orc_sphere* spheres; int num_spheres;
  const orc_triangle* tris;
  const orc_mesh* meshes; int num_meshes;
  uint64_t segments, tri_tests;
} orc_world;

/* intersecting_mesh, raytracing.glsl:243-264 */
static orc_hit intersecting_mesh(orc_world* w, const orc_mesh* m, v3 o, v3 d) {
  float op[3] = {o.x, o.y, o.z}, dp[3] = {d.x, d.y, d.z};
  if (!orc_intersecting_aabb(m->min_point, m->max_point, op, dp)) return empty_hit();
  w->tri_tests += m->len;
  float closest[4] = {ORC_FLT_MAX, ORC_FLT_MAX, ORC_FLT_MAX, ORC_FLT_MAX};
  for (uint32_t i = 0; i < m->len; i++) {
    float hi[4];
    intersecting_tri(&w->tris[i + m->first_index], o, d, hi);
    if (hi[3] > 0.001f && hi[3] < closest[3]) memcpy(closest, hi, sizeof closest);
  }
  if (closest[3] == ORC_FLT_MAX) return empty_hit();
  orc_hit h; h.hit_normal = mk3(closest[0], closest[1], closest[2]);
  h.hit_pos = ray_at(o, d, closest[3]); h.hit_dist = closest[3]; h.hit_mat = &m->material;
  return h;
}

/* world_hit, raytracing.glsl:267-288 (spheres first, then meshes, strict '<') */
static orc_hit world_hit(orc_world* w, v3 o, v3 d) {
  w->segments++;
  orc_hit closest = empty_hit();
  for (int i = 0; i < w->num_spheres; i++) {
    orc_hit h = intersecting_sphere(&w->spheres[i], o, d);
    if (h.hit_dist > 0.001f && h.hit_dist < closest.hit_dist) closest = h;
  }
  for (int i = 0; i < w->num_meshes; i++) {
    orc_hit h = intersecting_mesh(w, &w->meshes[i], o, d);
    if (h.hit_dist > 0.001f && h.hit_dist < closest.hit_dist) closest = h;
  }
  return closest;
}

/* ---------------------------------------------------------------------------------
 * Shading -- assets/raytracing.glsl:290-352
 * ------------------------------------------------------------------------------- */
/* environment_light, raytracing.glsl:290-294 */
static inline v3 environment_light(const orc_push* pc, v3 d) {
  if (!pc->use_environment_light) return mk3(0, 0, 0);
  float a = 0.5f * (d.y + 1.0f);
  float oma = 1.0f - a;
  return mk3(oma * 1.0f + a * 0.5f, oma * 1.0f + a * 0.7f, oma * 1.0f + a * 1.0f);
}

/* adjust_dir, raytracing.glsl:297-305 (both unit-sphere draws always happen) */
static inline v3 adjust_dir(v3 d, v3 n, const orc_material* mat, int specular, uint32_t* state) {
  v3 diffuse_dir = normalize3(add3(n, orc_unit_sphere(state)));
  float k = 2.0f * dot3(n, d);                      /* reflect(I,N) = I - 2*dot(N,I)*N */
  v3 specular_dir = sub3(d, muls3(n, k));
  v3 fuzz = muls3(orc_unit_sphere(state), mat->settings[2]);
  float a = mat->settings[1] * (float)specular;     /* settings.y * int(specular) */
  float oma = 1.0f - a;
  v3 mixed = mk3(diffuse_dir.x * oma + specular_dir.x * a,
                 diffuse_dir.y * oma + specular_dir.y * a,
                 diffuse_dir.z * oma + specular_dir.z * a);
  return normalize3(add3(mixed, fuzz));
}

/* trace_ray, raytracing.glsl:308-352 (returns light*colour -- reference behaviour) */
static v3 trace_ray(orc_world* w, const orc_push* pc, v3 root, v3 dir, uint32_t* state) {
  v3 light = mk3(0, 0, 0), colour = mk3(1, 1, 1);
  int has_not_hit_visible = 1;
  v3 ray_pos = root, ray_dir = dir;
  for (int i = 0; i <= pc->max_bounces; i++) {
    orc_hit hit = world_hit(w, ray_pos, ray_dir);
    if (hit.hit_dist < ORC_FLT_MAX) {
      const orc_material* m = hit.hit_mat;
      int invis = (m->settings[3] == 1.0f);
      ray_pos = adds3(hit.hit_pos, (float)invis * 0.001f);
      if (invis && has_not_hit_visible) {
        ray_pos = add3(hit.hit_pos, muls3(ray_dir, 0.001f));
        continue;
      } else {
        has_not_hit_visible = 0;
      }
      int is_spec = orc_u01(orc_hash(state)) < m->settings[0];
      ray_dir = adjust_dir(ray_dir, hit.hit_normal, m, is_spec, state);
      v3 emitted = muls3(ld3(m->emission), m->emission[3]);
      light = add3(light, mul3(emitted, colour));
      colour = mul3(colour, ld3(m->colour));
      float p = glsl_max(colour.x, glsl_max(colour.y, colour.z));
      if (orc_u01(orc_hash(state)) >= p) break;
      colour = divs3(colour, p);
    } else {
      light = add3(light, environment_light(pc, ray_dir));
      break;
    }
  }
  return mul3(light, colour);
}

/* get_ray_dir, raytracing.glsl:162-166 (u1, u2, u3 in order; left-to-right evaluation) */
static inline v3 get_ray_dir(const orc_push* pc, v3 c, uint32_t* state) {
  float r = (orc_u01(orc_hash(state)) * 2.0f) * 3.14159265358979323846f;
  float cr = ORC_COSF(r);
  float j = pc->jitter_size;
  float s2 = sqrtf(orc_u01(orc_hash(state)));
  v3 t1 = muls3(muls3(muls3(mk3(0.0f, 0.0f, 1.0f), cr), j), s2);
  float sr = ORC_SINF(r);
  float s3 = sqrtf(orc_u01(orc_hash(state)));
  v3 t2 = muls3(muls3(muls3(mk3(0.0f, 1.0f, 0.0f), sr), j), s3);
  v3 nc = add3(add3(c, t1), t2);
  const float* M = pc->cam_alignment_mat; /* mat3(M) * nc, S2 row order */
  v3 wv = mk3(fmaf(M[8], nc.z, fmaf(M[4], nc.y, M[0] * nc.x)),
              fmaf(M[9], nc.z, fmaf(M[5], nc.y, M[1] * nc.x)),
              fmaf(M[10], nc.z, fmaf(M[6], nc.y, M[2] * nc.x)));
  return normalize3(wv);
}

/* S7 */
static inline uint8_t unorm8(float x) {
  if (!(x > 0.0f)) return 0;
  if (x >= 1.0f) return 255;
  return (uint8_t)(int)rintf(x * 255.0f);
}

/* main, raytracing.glsl:355-389 for one pixel.  out_rgb = colour/num_samples (pre-quantization). */
static void shade_pixel(orc_world* w, const orc_push* pc, const orc_ray* rays, uint32_t x, uint32_t y,
                        float out_rgb[3]) {
  uint32_t id = x + y * pc->width;
  v3 colour = mk3(0, 0, 0);
  uint32_t state = pc->rng_offset * 719393u + id;
  v3 root = ld3(pc->cam_pos);
  v3 centre = ld3(rays[id].sample_centre);
  for (int i = 0; i < pc->num_samples; i++) {
    v3 dir = get_ray_dir(pc, centre, &state);
    colour = add3(colour, trace_ray(w, pc, root, normalize3(dir), &state));
  }
  colour = divs3(colour, (float)pc->num_samples);
  out_rgb[0] = colour.x; out_rgb[1] = colour.y; out_rgb[2] = colour.z;
}

/*
 * Trace a frame (or the rows [y0, y1) of one).  rgba8 may be NULL; rgba32f may be NULL.
 * Both are indexed with the full-image row stride (W) and global row y.
 * segments / tri_tests (may be NULL) receive the exact counts.
 * nthreads <= 0 -> OpenMP default.
 */
void orc_trace_rows(const orc_push* pc, const orc_ray* rays, const orc_sphere* spheres,
                    const orc_triangle* tris, const orc_mesh* meshes, uint32_t y0, uint32_t y1,
                    uint8_t* rgba8, float* rgba32f, uint64_t* segments, uint64_t* tri_tests, int nthreads) {
  uint64_t seg = 0, tt = 0;
  uint32_t W = pc->width;
  if (y1 > pc->height) y1 = pc->height;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  if (pc->init) { /* raytracing.glsl:363-366 */
    for (uint32_t y = y0; y < y1; y++)
      for (uint32_t x = 0; x < W; x++) {
        size_t p = (size_t)y * W + x;
        if (rgba8) { rgba8[4 * p] = 0; rgba8[4 * p + 1] = 0; rgba8[4 * p + 2] = 0; rgba8[4 * p + 3] = 255; }
        if (rgba32f) { rgba32f[4 * p] = 0; rgba32f[4 * p + 1] = 0; rgba32f[4 * p + 2] = 0; rgba32f[4 * p + 3] = 1; }
      }
    if (segments) *segments = 0;
    if (tri_tests) *tri_tests = 0;
    return;
  }
  long npix = (long)(y1 > y0 ? y1 - y0 : 0) * (long)W;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : seg, tt)
  for (long q = 0; q < npix; q++) {
    uint32_t y = y0 + (uint32_t)(q / W), x = (uint32_t)(q % W);
    orc_world w = {spheres, pc->num_spheres, tris, meshes, pc->num_meshes, 0, 0};
    float rgb[3];
    shade_pixel(&w, pc, rays, x, y, rgb);
    size_t p = (size_t)y * W + x;
    if (rgba8) {
      rgba8[4 * p] = unorm8(rgb[0]); rgba8[4 * p + 1] = unorm8(rgb[1]);
      rgba8[4 * p + 2] = unorm8(rgb[2]); rgba8[4 * p + 3] = 255;
    }
    if (rgba32f) {
      rgba32f[4 * p] = rgb[0]; rgba32f[4 * p + 1] = rgb[1]; rgba32f[4 * p + 2] = rgb[2]; rgba32f[4 * p + 3] = 1.0f;
    }
    seg += w.segments; tt += w.tri_tests;
  }
  if (segments) *segments = seg;
  if (tri_tests) *tri_tests = tt;
}

/* Trace one pixel (per-pixel path KATs). */
void orc_trace_pixel(const orc_push* pc, const orc_ray* rays, const orc_sphere* spheres,
                     const orc_triangle* tris, const orc_mesh* meshes, uint32_t x, uint32_t y,
                     float out_rgb[3], uint64_t* segments, uint64_t* tri_tests) {
  orc_world w = {spheres, pc->num_spheres, tris, meshes, pc->num_meshes, 0, 0};
  shade_pixel(&w, pc, rays, x, y, out_rgb);
  if (segments) *segments = w.segments;
  if (tri_tests) *tri_tests = w.tri_tests;
}

/* A list of pixels (xy[2k], xy[2k+1]) of one frame: rgba8 out[4k..4k+3] (OpenMP over the list). */
void orc_trace_pixels(const orc_push* pc, const orc_ray* rays, const orc_sphere* spheres,
                      const orc_triangle* tris, const orc_mesh* meshes, const uint32_t* xy, uint32_t n,
                      uint8_t* out, uint64_t* segments, uint64_t* tri_tests, int nthreads) {
  uint64_t seg = 0, tt = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : seg, tt)
  for (long k = 0; k < (long)n; k++) {
    orc_world w = {spheres, pc->num_spheres, tris, meshes, pc->num_meshes, 0, 0};
    float rgb[3];
    shade_pixel(&w, pc, rays, xy[2 * k], xy[2 * k + 1], rgb);
    out[4 * k] = unorm8(rgb[0]); out[4 * k + 1] = unorm8(rgb[1]);
    out[4 * k + 2] = unorm8(rgb[2]); out[4 * k + 3] = 255;
    seg += w.segments; tt += w.tri_tests;
  }
  if (segments) *segments = seg;
  if (tri_tests) *tri_tests = tt;
}

/* image_combiner.glsl:22-43 on rgba8 images (npix pixels). */
void orc_accumulate_rgba8(uint32_t frame, uint8_t* current, const uint8_t* new_image, size_t npix) {
  for (size_t p = 0; p < npix; p++) {
    if (frame == 0) { current[4 * p] = 0; current[4 * p + 1] = 0; current[4 * p + 2] = 0; current[4 * p + 3] = 255; continue; }
    float ff = (float)frame, ff1 = (float)(frame + 1u);
    for (int c = 0; c < 3; c++) {
      float prev = (float)current[4 * p + c] / 255.0f;
      float nw = (float)new_image[4 * p + c] / 255.0f;
      float col = (nw + prev * ff) / ff1;
      current[4 * p + c] = unorm8(col);
    }
    current[4 * p + 3] = 255;
  }
}

/* fp32 accumulator mode (build extension): same formula, no quantization. */
void orc_accumulate_rgba32f(uint32_t frame, float* current, const float* new_image, size_t npix) {
  for (size_t p = 0; p < npix; p++) {
    if (frame == 0) { current[4 * p] = 0; current[4 * p + 1] = 0; current[4 * p + 2] = 0; current[4 * p + 3] = 1; continue; }
    float ff = (float)frame, ff1 = (float)(frame + 1u);
    for (int c = 0; c < 3; c++) current[4 * p + c] = (new_image[4 * p + c] + current[4 * p + c] * ff) / ff1;
    current[4 * p + 3] = 1.0f;
  }
}

uint8_t orc_unorm8(float x) { return unorm8(x); }

/* ---------------------------------------------------------------------------------
 * Host prep -- src/raytrace_pipeline.rs:269-428 (Rust arithmetic: S8, no contraction)
 * ------------------------------------------------------------------------------- */
static inline v3 rs_cross(v3 a, v3 b) {
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float rs_mag(v3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
static inline v3 rs_norm(v3 a) { float m = rs_mag(a); return mk3(a.x / m, a.y / m, a.z / m); }
static inline v3 rs_neg(v3 a) { return mk3(-a.x, -a.y, -a.z); }

/* get_view_matrix, src/raytrace_pipeline.rs:269-285.  out = column-major mat4 (rows of the
 * transposed from_columns matrix become the columns: M*(1,0,0) = normalised direction). */
void orc_view_matrix(const float dir[3], const float up[3], float out[16]) {
  v3 d = ld3(dir), u = ld3(up);
  v3 nx = rs_norm(d);
  v3 nz = rs_neg(rs_norm(rs_cross(d, u)));
  v3 ny = rs_neg(rs_norm(rs_cross(nx, nz)));
  float m[16] = {nx.x, nx.y, nx.z, 0.0f, ny.x, ny.y, ny.z, 0.0f, nz.x, nz.y, nz.z, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f};
  memcpy(out, m, sizeof m);
}

/* create_ray_subbuffer, src/raytrace_pipeline.rs:289-338.  Returns number of rays; writes
 * W*H records (w component 1.0, unused by the kernel) and the default jitter. */
uint32_t orc_create_rays(uint32_t W, uint32_t H, float focal, float vh, const float up[3], orc_ray* out,
                         float* default_jitter) {
  if (W == 0 || H == 0) { *default_jitter = 0.0f; return 0; }
  float vw = vh * ((float)W / (float)H);
  v3 X = mk3(1.0f, 0.0f, 0.0f);
  v3 vx = rs_norm(rs_cross(ld3(up), X));
  v3 vy = rs_norm(rs_cross(vx, X));
  v3 fx = mk3(X.x * focal, X.y * focal, X.z * focal);
  v3 ul = sub3(add3(mk3(0, 0, 0), fx), muls3(add3(muls3(vx, vw), muls3(vy, vh)), 0.5f));
  v3 px = divs3(muls3(vx, vw), (float)W);
  v3 py = divs3(muls3(vy, vh), (float)H);
  v3 first = add3(ul, muls3(add3(px, py), 0.5f));
  for (uint32_t y = 0; y < H; y++)
    for (uint32_t x = 0; x < W; x++) {
      v3 r = add3(add3(first, muls3(px, (float)x)), muls3(py, (float)y));
      orc_ray* o = &out[(size_t)y * W + x];
      o->sample_centre[0] = r.x; o->sample_centre[1] = r.y; o->sample_centre[2] = r.z; o->sample_centre[3] = 1.0f;
    }
  float mx = rs_mag(px), my = rs_mag(py);
  *default_jitter = ((mx < my) ? my : mx) * 0.5f; /* f32::max */
  return W * H;
}

/* transform_meshes, src/raytrace_pipeline.rs:377-428 for ONE mesh (caller loops meshes).
 * positions: nverts*3 floats; indices: nidx (multiple of 3).  Writes nidx/3 triangles and fills
 * min/max (the mesh record's first_index/len/material are the caller's). */
void orc_transform_mesh(const float* positions, const uint32_t* indices, uint32_t nidx, orc_triangle* tris,
                        float mn[3], float mx[3]) {
  float mnx = ORC_FLT_MAX, mny = ORC_FLT_MAX, mnz = ORC_FLT_MAX;
  float mxx = -ORC_FLT_MAX, mxy = -ORC_FLT_MAX, mxz = -ORC_FLT_MAX;
  for (uint32_t i = 0; i + 2 < nidx; i += 3) {
    v3 a = ld3(&positions[3 * indices[i]]), b = ld3(&positions[3 * indices[i + 1]]), c = ld3(&positions[3 * indices[i + 2]]);
    v3 e1 = sub3(b, a), e2 = sub3(c, a);
    v3 n = rs_cross(e1, e2);
    mnx = fminf(mnx, fminf(a.x, fminf(b.x, c.x))); mny = fminf(mny, fminf(a.y, fminf(b.y, c.y)));
    mnz = fminf(mnz, fminf(a.z, fminf(b.z, c.z)));
    mxx = fmaxf(mxx, fmaxf(a.x, fmaxf(b.x, c.x))); mxy = fmaxf(mxy, fmaxf(a.y, fmaxf(b.y, c.y)));
    mxz = fmaxf(mxz, fmaxf(a.z, fmaxf(b.z, c.z)));
    orc_triangle* t = &tris[i / 3];
    t->a[0] = a.x; t->a[1] = a.y; t->a[2] = a.z; t->a[3] = 1.0f;
    t->edge_one[0] = e1.x; t->edge_one[1] = e1.y; t->edge_one[2] = e1.z; t->edge_one[3] = 1.0f;
    t->edge_two[0] = e2.x; t->edge_two[1] = e2.y; t->edge_two[2] = e2.z; t->edge_two[3] = 1.0f;
    t->normal[0] = n.x; t->normal[1] = n.y; t->normal[2] = n.z; t->normal[3] = 1.0f;
  }
  mn[0] = mnx; mn[1] = mny; mn[2] = mnz; mx[0] = mxx; mx[1] = mxy; mx[2] = mxz;
}

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
