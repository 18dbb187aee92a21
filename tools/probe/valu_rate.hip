// Issue cost of a few VALU ops on gfx950 (one wave per SIMD and four): 8 independent chains of each
// op inside a timed loop, cycles per instruction from the shader clock.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ void rate(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
  const uint32_t k = seed | 1u;
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if constexpr (OP == 2) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "s"(k));
      if constexpr (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if constexpr (OP == 4) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i]));
      if constexpr (OP == 5) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[i]));
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) out[gridDim.x * blockDim.x + blockIdx.x] = (uint32_t)(t1 - t0);
}

template <int OP>
static void run(const char* name, int waves_per_simd) {
  const int iters = 4096, block = 64 * 4 * waves_per_simd, grid = 256;
  uint32_t* d;
  hipMalloc(&d, (size_t)(grid * block + grid) * 4);
  hipLaunchKernelGGL(rate<OP>, dim3(grid), dim3(block), 0, 0, d, 3u, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(rate<OP>, dim3(grid), dim3(block), 0, 0, d, 3u, iters);
  hipDeviceSynchronize();
  uint32_t cyc[256];
  hipMemcpy(cyc, d + grid * block, grid * 4, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += cyc[i];
  s /= grid;
  // cycles per instruction per SIMD: each SIMD runs waves_per_simd waves of iters * 8 instructions
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.3f}\n", name, waves_per_simd,
         s / ((double)iters * 8 * waves_per_simd));
  hipFree(d);
}

int main() {
  for (int w : {1, 4}) {
    run<0>("v_mul_lo_u32", w);
    run<1>("v_add_u32", w);
    run<2>("v_fma_f32", w);
    run<3>("v_mul_u32_u24", w);
    run<4>("v_sqrt_f32", w);
    run<5>("v_cvt_f32_u32", w);
  }
  return 0;
}
