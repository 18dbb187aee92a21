// hrt_math.h -- device-side numerics for the gfx950 path tracer.
//
// The GLSL reference (assets/raytracing.glsl) leaves dot/cross summation order, FMA contraction,
// normalize's form and the transcendental algorithms to the Vulkan driver.  This header pins each
// of them (DESIGN.md "numerics spec" S1-S7) so that a frame is reproducible bit for bit on any IEEE
// binary32 machine; the CPU oracle (oracle/rt_oracle.c) restates the same spec independently.
// The file is compiled with -ffp-contract=off: every fma below is explicit, nothing else fuses.
// gfx950's f32 '/', sqrt, fma, u32->f32 and rint are correctly rounded with denormals kept
// (measured bit-exact against the host over 4M inputs, tools/probe/probe.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hrt {

constexpr float kFltMax = 3.402823466e+38f;  // raytracing.glsl:2

struct f3 {
  float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ f3 adds(f3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }

// S2: dot / cross / mat3*vec with explicit FMA in a fixed order.
__device__ __forceinline__ float dot(f3 a, f3 b) {
  return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return {__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
          __builtin_fmaf(a.x, b.y, -(a.y * b.x))};
}
// S4 at the instruction level.  hipcc lowers a correctly rounded f32 '/' to
//   v_div_scale (den), v_div_scale (num), v_rcp, e = fma(-den, y0, 1), y = fma(e, y0, y0),
//   q = num * y, r = fma(-den, q, num), q1 = fma(r, y, q), r1 = fma(-den, q1, num),
//   v_div_fmas (= fma(r1, y, q1) when no scaling), v_div_fixup
// and a correctly rounded sqrt to a 2^32 pre-scale for tiny inputs, v_sqrt, the two neighbours'
// fma residual tests, the un-scale and a special-value select.  In the range where V_DIV_SCALE_F32
// scales nothing (|num|, |den| in [2^-80, 2^40], nonzero: no exponent gap >= 96, no denormal den,
// 1/den or quotient, num exponent > 23) and V_DIV_FIXUP_F32 passes the finite nonzero quotient
// through, and where the sqrt input needs no pre-scale and is not special (x in [2^-96, 2^80]), the
// sequences below ARE the compiler's instructions minus those identities -- the same bits -- and the
// reciprocal of a common denominator is shared by the three components of a vector.  (Since r02v the
// division also stops after q1: y is then already RN(1/den), so q1 is the correctly rounded quotient
// by Markstein's theorem and the last correction never changes it; see div_core.)
// tests/test_gpu_boundary.py::test_fast_division_and_sqrt_match_ieee checks them on the device.
__device__ __forceinline__ float sqrt_core(float x) {  // x in [2^-96, 2^80]
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) - 1u);
  const float su = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) + 1u);
  float r = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
  r = __builtin_fmaf(-su, s, x) > 0.0f ? su : r;
  return r;
}
__device__ __forceinline__ float rcp_core(float den) {  // the refined reciprocal of the '/' sequence
  const float y0 = __builtin_amdgcn_rcpf(den);
  return __builtin_fmaf(__builtin_fmaf(-den, y0, 1.0f), y0, y0);
}
#ifndef HRT_DIV_MARKSTEIN
#define HRT_DIV_MARKSTEIN 1
#endif
__device__ __forceinline__ float div_core(float num, float den, float y) {
  const float q = num * y;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-den, q, num), y, q);
#if HRT_DIV_MARKSTEIN
  // rcp_core is RN(1/den) on the whole range (every float in [2^-40, 2^40], checked on the device:
  // hrt_debug_math_check_rng), so q = RN(num y) is within 1 ulp of num / den and Markstein's theorem
  // makes the first correction q1 = RN(q + (num - den q) y) the correctly rounded quotient (the
  // residual is exact by the fma); the compiler's sequence's second correction changes nothing
  return q1;
#else
  return __builtin_fmaf(__builtin_fmaf(-den, q1, num), y, q1);
#endif
}
// a / s for s > 0, correctly rounded (the shared-reciprocal path when every lane value is in range)
__device__ __forceinline__ f3 div3(f3 a, float s) {
  const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
  const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
  const float sum = (a.x + a.y) + a.z;  // fmin / fmax skip a NaN component: this does not
  if (s >= 0x1p-40f && s <= 0x1p40f && m >= 0x1p-80f && mx <= 0x1p40f && sum == sum) {
    const float y = rcp_core(s);
    return {div_core(a.x, s, y), div_core(a.y, s, y), div_core(a.z, s, y)};
  }
  return {a.x / s, a.y / s, a.z / s};
}
// S4: normalize = v / sqrt(dot(v, v)), correctly rounded sqrt and divides.
__device__ __forceinline__ f3 normalize(f3 a) {
  const float d2 = dot(a, a);
  const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
  if (d2 >= 0x1p-80f && d2 <= 0x1p78f && m >= 0x1p-80f) {  // then |a.c| <= sqrt(d2) <= 2^39
    const float l = sqrt_core(d2);
    const float y = rcp_core(l);
    return {div_core(a.x, l, y), div_core(a.y, l, y), div_core(a.z, l, y)};
  }
  return a / __builtin_sqrtf(d2);
}
// normalize with the fast path chosen per WAVE: when every active lane is in the fast range (the usual
// case for ray directions) the wave runs it without the per-lane exec-mask split around the IEEE
// fallback (which every lane then skips); otherwise every active lane runs the IEEE spelling, which
// is exact everywhere.  Same bits as normalize either way.
// fast: the wave took the fast path (then every active lane's result has |component| <= 1 + 2^-23:
// |a.c| <= sqrt(RN dot) (1 + 2^-24) and the quotient is correctly rounded)
__device__ __forceinline__ f3 normalize_wu(f3 a, bool& fast_all) {
  const float d2 = dot(a, a);
  const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
  // (a ballot per compare: each is the compare's own lane mask, no VGPR round trip)
  fast_all = (__builtin_amdgcn_ballot_w64(d2 >= 0x1p-80f) & __builtin_amdgcn_ballot_w64(d2 <= 0x1p78f) &
              __builtin_amdgcn_ballot_w64(m >= 0x1p-80f)) == __builtin_amdgcn_read_exec();
  if (__builtin_expect(fast_all, 1)) {
    const float l = sqrt_core(d2);
    const float y = rcp_core(l);
    return {div_core(a.x, l, y), div_core(a.y, l, y), div_core(a.z, l, y)};
  }
  return a / __builtin_sqrtf(d2);
}
__device__ __forceinline__ f3 normalize_wu(f3 a) {
  bool f;
  return normalize_wu(a, f);
}
// The fused loop's and the shading's normalizes (ray generation, adjust_dir, unit_sphere): per wave
// (normalize_wu) or per lane (normalize); the same bits either way.
#ifndef HRT_NORM_UNIFORM_FUSED
#define HRT_NORM_UNIFORM_FUSED 1  // (r04r: island 1.843 -> 1.838, cave 5.625 -> 5.601 ms per frame)
#endif
__device__ __forceinline__ f3 normalize_fl(f3 a) { return HRT_NORM_UNIFORM_FUSED ? normalize_wu(a) : normalize(a); }
// The reference's spelling of both (for the self-check).
__device__ __forceinline__ f3 normalize_ieee(f3 a) { return a / __builtin_sqrtf(dot(a, a)); }
// S6: GLSL 4.60 definitions.
__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }

__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

// S5: natural log.  m in [sqrt(1/2), sqrt(2)), log(1+f) = f - f^2/2 + f^3 P(f), ln2 split in two.
__device__ __forceinline__ float spec_log(float x) {
  uint32_t ix = fbits(x);
  if (x != x) return x;
  if (x == 0.0f) return -__builtin_inff();
  if (ix >> 31) return bitsf(0x7fc00000u);
  if (ix == 0x7f800000u) return x;
  int k = 0;
  if (ix < 0x00800000u) {
    x = x * 8388608.0f;
    ix = fbits(x);
    k = -23;
  }
  ix += 0x3f800000u - 0x3f3504f3u;
  k += (int)(ix >> 23) - 0x7f;
  ix = (ix & 0x007fffffu) + 0x3f3504f3u;
  const float f = bitsf(ix) - 1.0f;
  const float z = f * f;
  float p = 7.0376836292e-2f;
  p = __builtin_fmaf(p, f, -1.1514610310e-1f);
  p = __builtin_fmaf(p, f, 1.1676998740e-1f);
  p = __builtin_fmaf(p, f, -1.2420140846e-1f);
  p = __builtin_fmaf(p, f, 1.4249322787e-1f);
  p = __builtin_fmaf(p, f, -1.6668057665e-1f);
  p = __builtin_fmaf(p, f, 2.0000714765e-1f);
  p = __builtin_fmaf(p, f, -2.4999993993e-1f);
  p = __builtin_fmaf(p, f, 3.3333331174e-1f);
  float y = (p * f) * z;
  const float fk = (float)k;
  y = __builtin_fmaf(fk, -2.12194440e-4f, y);
  y = __builtin_fmaf(z, -0.5f, y);
  const float r = f + y;
  return __builtin_fmaf(fk, 0.693359375f, r);
}

// spec_log on the RNG's values u01(h) = h 2^-32: 0 or in [2^-32, 1] -- never NaN, negative, infinite or
// denormal, so only the zero case remains (checked over all 2^32 states, hrt_debug_math_check_rng).
__device__ __forceinline__ float spec_log_u01(float x) {
  uint32_t ix = fbits(x);
  ix += 0x3f800000u - 0x3f3504f3u;
  const int k = (int)(ix >> 23) - 0x7f;
  ix = (ix & 0x007fffffu) + 0x3f3504f3u;
  const float f = bitsf(ix) - 1.0f;
  const float z = f * f;
  float p = 7.0376836292e-2f;
  p = __builtin_fmaf(p, f, -1.1514610310e-1f);
  p = __builtin_fmaf(p, f, 1.1676998740e-1f);
  p = __builtin_fmaf(p, f, -1.2420140846e-1f);
  p = __builtin_fmaf(p, f, 1.4249322787e-1f);
  p = __builtin_fmaf(p, f, -1.6668057665e-1f);
  p = __builtin_fmaf(p, f, 2.0000714765e-1f);
  p = __builtin_fmaf(p, f, -2.4999993993e-1f);
  p = __builtin_fmaf(p, f, 3.3333331174e-1f);
  float y = (p * f) * z;
  const float fk = (float)k;
  y = __builtin_fmaf(fk, -2.12194440e-4f, y);
  y = __builtin_fmaf(z, -0.5f, y);
  const float r = f + y;
  const float l = __builtin_fmaf(fk, 0.693359375f, r);
  return x == 0.0f ? -__builtin_inff() : l;
}

// S5: sin / cos.  Cody-Waite reduction by pi/2 (3 parts), odd/even polynomials on |r| <= pi/4.
__device__ __forceinline__ float spec_reduce(float x, int& q) {
  const float j = __builtin_rintf(x * 0.636619772367581343f);
  q = (int)j;
  float r = __builtin_fmaf(-j, 1.5703125f, x);
  r = __builtin_fmaf(-j, 4.837512969970703125e-4f, r);
  r = __builtin_fmaf(-j, 7.549789954891882e-8f, r);
  return r;
}
__device__ __forceinline__ float sin_poly(float r) {
  const float z = r * r;
  float p = -1.9515295891e-4f;
  p = __builtin_fmaf(p, z, 8.3321608736e-3f);
  p = __builtin_fmaf(p, z, -1.6666654611e-1f);
  return __builtin_fmaf(p * z, r, r);
}
__device__ __forceinline__ float cos_poly(float r) {
  const float z = r * r;
  float p = 2.443315711809948e-5f;
  p = __builtin_fmaf(p, z, -1.388731625493765e-3f);
  p = __builtin_fmaf(p, z, 4.166664568298827e-2f);
  return __builtin_fmaf(p * z, z, __builtin_fmaf(z, -0.5f, 1.0f));
}
// sin and cos of the same argument (both quadrants from one reduction).
__device__ __forceinline__ void spec_sincos(float x, float& s, float& c) {
  if (!(__builtin_fabsf(x) <= 1.0e5f)) {
    const float nan = (x != x) ? x : bitsf(0x7fc00000u);
    s = nan;
    c = nan;
    return;
  }
  int q;
  const float r = spec_reduce(x, q);
  const float ps = sin_poly(r), pc = cos_poly(r);
  switch (q & 3) {
    case 0: s = ps; c = pc; break;
    case 1: s = pc; c = -ps; break;
    case 2: s = -ps; c = -pc; break;
    default: s = -pc; c = ps; break;
  }
}
__device__ __forceinline__ float spec_cos(float x) {
  float s, c;
  spec_sincos(x, s, c);
  return c;
}
// The same for x in [0, 7] (the RNG's angles u * 2pi): the NaN / range guard always passes there.
// The quadrant as selects and sign flips (no branches): odd q swaps the polynomials, q & 2 negates
// the sine, (q + 1) & 2 the cosine -- the switch above, value for value.
__device__ __forceinline__ void spec_sincos_angle(float x, float& s, float& c) {
  int q;
  const float r = spec_reduce(x, q);
  const float ps = sin_poly(r), pc = cos_poly(r);
  const bool odd = (q & 1) != 0;
  const uint32_t sn = ((uint32_t)q & 2u) << 30, cn = ((uint32_t)(q + 1) & 2u) << 30;
  s = bitsf(fbits(odd ? pc : ps) ^ sn);
  c = bitsf(fbits(odd ? ps : pc) ^ cn);
}

// ---- RNG: assets/raytracing.glsl:13-40 ------------------------------------------------------
__device__ __forceinline__ uint32_t hash(uint32_t& state) {  // :13-21
  uint32_t s = state;
  s ^= 2747636419u;
  s *= 2654435769u;
  s ^= s >> 16;
  s *= 2654435769u;
  s ^= s >> 16;
  s *= 2654435769u;
  state = s;
  return s;
}
// scaleToRange01 :23-25 -- float(4294967295.0) == 2^32, so the divide is an exact power-of-two scale.
__device__ __forceinline__ float u01(uint32_t s) { return (float)s * 2.3283064365386963e-10f; }
// c * u01(s) in one multiply: u01's scaling by 2^-32 is exact (float(s) is 0 or >= 1), so
// RN(c * (float(s) 2^-32)) == RN(float(s) * (c 2^-32)) with c 2^-32 an exact float (c_scaled)
__device__ __forceinline__ float u01_mul(uint32_t s, float c_scaled) { return (float)s * c_scaled; }

// sqrt on the RNG's values: sqrt_core is the correctly rounded sqrt on every u01 value (k * 2^-32, so 0
// or >= 2^-32) and on every -2 log(u01) (0 .. 44.4, -0 at u = 1, +inf at u = 0): checked exhaustively
// over all 2^32 states on the device (hrt_debug_math_check_rng).
__device__ __forceinline__ float sqrt_rng(float x) { return sqrt_core(x); }

__device__ __forceinline__ float normal_dist(uint32_t& state) {  // :28-33
  const float theta = u01_mul(hash(state), 6.2831852f * 0x1p-32f);  // 6.2831852f * u01: 2 * 3.1415926 folded exactly
  const float rho = sqrt_rng(-2.0f * spec_log_u01(u01(hash(state))));
  float s, c;
  spec_sincos_angle(theta, s, c);
  return rho * c;
}
__device__ __forceinline__ f3 unit_sphere(uint32_t& state) {  // :35-40
  const float x = normal_dist(state);
  const float y = normal_dist(state);
  const float z = normal_dist(state);
  return normalize_fl(mk(x, y, z));
}

// S7: R8G8B8A8_UNORM store / load.
__device__ __forceinline__ uint32_t unorm8(float x) {
  if (!(x > 0.0f)) return 0u;
  if (x >= 1.0f) return 255u;
  return (uint32_t)(int)__builtin_rintf(x * 255.0f);
}
__device__ __forceinline__ float unorm8_to_float(uint32_t k) { return (float)k / 255.0f; }

}  // namespace hrt
