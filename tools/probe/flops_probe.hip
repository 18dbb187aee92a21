// Does SQ_INSTS_VALU_FLOPS_FP32 weight FP32 VALU instructions by the exec mask?
// Each kernel runs ITERS x 8 instructions of one op per lane on the lanes below `active` (a lane-divergent
// branch: the other lanes are masked off), 1024 waves.  Run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32
//             SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 -- ./flops_probe
// and compare with the expected counts it prints: instructions per wave = ITERS x 8 whatever the mask;
// lane FLOPs = active x ITERS x 8 x (2 for an fma, 1 otherwise) per wave.
// hipcc --offload-arch=gfx950 -O3 -o flops_probe flops_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 1024;
constexpr int kGrid = 256, kBlock = 256;  // 1024 waves

template <int OP>
__global__ void op_kernel(float* out, float seed, int active) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed + (float)(threadIdx.x * 8 + i) * 1e-3f;
  if ((int)(threadIdx.x & 63) < active) {
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "s"(seed));
        if constexpr (OP == 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "s"(seed));
        if constexpr (OP == 2) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "s"(seed));
        if constexpr (OP == 3) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i]));
      }
    }
  }
  float x = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) x += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int OP>
static void run(const char* name, int active, int flops_per_inst, float* d) {
  hipLaunchKernelGGL(op_kernel<OP>, dim3(kGrid), dim3(kBlock), 0, 0, d, 1.0000001f, active);
  hipDeviceSynchronize();
  const double waves = (double)kGrid * kBlock / 64, insts = (double)kIters * 8;
  printf("{\"op\": \"%s\", \"active_lanes\": %d, \"expect_wave_insts\": %.0f, \"expect_lane_flops\": %.0f, "
         "\"expect_64lane_flops\": %.0f}\n",
         name, active, waves * insts, waves * insts * active * flops_per_inst, waves * insts * 64 * flops_per_inst);
}

int main() {
  float* d;
  hipMalloc(&d, (size_t)kGrid * kBlock * 4);
  // dispatch order = the order of the records rocprofv3 writes
  for (int act : {64, 32, 16, 1}) run<0>("v_fma_f32", act, 2, d);
  for (int act : {64, 32}) run<1>("v_mul_f32", act, 1, d);
  for (int act : {64, 32}) run<2>("v_add_f32", act, 1, d);
  for (int act : {64, 32}) run<3>("v_sqrt_f32", act, 1, d);
  hipFree(d);
  return 0;
}
