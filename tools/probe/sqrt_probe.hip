#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ __forceinline__ float sqrt_core(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) - 1u);
  const float su = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) + 1u);
  float r = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
  r = __builtin_fmaf(-su, s, x) > 0.0f ? su : r;
  return r;
}
__global__ void k(uint32_t base, unsigned long long* bad) {
  const uint32_t i = base + blockIdx.x * 256u + threadIdx.x;
  const float u = (float)i * 2.3283064365386963e-10f;
  if (__builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(u)) != __builtin_bit_cast(uint32_t, sqrt_core(u))) atomicAdd(&bad[0], 1ull);
  const float x = __builtin_bit_cast(float, i);  // every float
  if (x >= 0x1p-96f && x <= 0x1p80f && __builtin_bit_cast(uint32_t, __builtin_amdgcn_sqrtf(x)) != __builtin_bit_cast(uint32_t, sqrt_core(x))) atomicAdd(&bad[1], 1ull);
}
int main() {
  unsigned long long* d; hipMalloc(&d, 16); hipMemset(d, 0, 16);
  for (uint64_t b = 0; b < (1ull << 32); b += (1ull << 28)) k<<<(1u << 28) / 256u, 256>>>((uint32_t)b, d);
  unsigned long long h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("v_sqrt_f32 != correctly rounded: %llu of 2^32 u01 values, %llu of the floats in [2^-96, 2^80]\n", h[0], h[1]);
  return 0;
}
