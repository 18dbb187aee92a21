// Probe: is hrt_math.h's one-Newton-step reciprocal rcp_core(b) = RN(1/b) for every b of the
// fast-division range, and is then the 3-op quotient q' = RN(q + (a - b q) y), q = RN(a y), equal to
// the IEEE a / b (Markstein's theorem)?  Exhaustive over the mantissas of several binades for the
// reciprocal; hashed pairs for the quotient.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp1(float den) {
  const float y0 = __builtin_amdgcn_rcpf(den);
  return __builtin_fmaf(__builtin_fmaf(-den, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float div3op(float a, float b, float y) {
  const float q = a * y;
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ uint32_t mix(uint32_t s) {
  s ^= 2747636419u; s *= 2654435769u; s ^= s >> 16; s *= 2654435769u; s ^= s >> 16; s *= 2654435769u;
  return s;
}

// thread i: mantissa i of binade e (b = 2^e * (1 + i 2^-23)), e from the launch
__global__ void rcp_exhaustive(int e, unsigned long long* bad) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= (1u << 23)) return;
  const float b = __builtin_bit_cast(float, ((uint32_t)(e + 127) << 23) | i);
  const float y = rcp1(b);
  const float r = 1.0f / b;  // the compiler's correctly rounded division
  if (__builtin_bit_cast(uint32_t, y) != __builtin_bit_cast(uint32_t, r)) atomicAdd(bad, 1ull);
}
// hashed (a, b) with |a|, |b| in [2^-40, 2^40]: 3-op quotient vs IEEE
__global__ void div_hashed(uint32_t seed, unsigned long long* bad) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const uint32_t h1 = mix(seed * 0x9E3779B9u + i), h2 = mix(h1 + 0x7F4A7C15u), h3 = mix(h2);
  const float a = __builtin_ldexpf(__builtin_bit_cast(float, 0x3f800000u | (h1 & 0x7fffffu)), (int)(h3 % 80u) - 40) *
                  ((h3 >> 31) ? -1.0f : 1.0f);
  const float b = __builtin_ldexpf(__builtin_bit_cast(float, 0x3f800000u | (h2 & 0x7fffffu)), (int)((h3 >> 8) % 80u) - 40);
  const float q = div3op(a, b, rcp1(b));
  if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, a / b)) atomicAdd(bad, 1ull);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 8);
  const int exps[] = {-40, -20, -1, 0, 1, 5, 20, 39};
  unsigned long long total = 0;
  for (int e : exps) {
    hipMemset(d, 0, 8);
    rcp_exhaustive<<<(1u << 23) / 256u, 256>>>(e, d);
    unsigned long long h = 0;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("rcp binade 2^%d: %llu of 8388608 mantissas not RN(1/b)\n", e, h);
    total += h;
  }
  unsigned long long dbad = 0;
  for (uint32_t s = 0; s < 64; ++s) {
    hipMemset(d, 0, 8);
    div_hashed<<<(1u << 24) / 256u, 256>>>(s, d);
    unsigned long long h = 0;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    dbad += h;
  }
  printf("3-op quotient: %llu of %llu hashed pairs differ from IEEE a / b\n", dbad, 64ull << 24);
  return (int)(total != 0 || dbad != 0);
}
