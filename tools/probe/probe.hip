// Early hardware probe: (1) are gfx950 f32 div / sqrt / fma / u32->f32 / rint bit-identical to the
// host's IEEE results (the parity plan depends on it); (2) v_fma_f32 vs v_pk_fma_f32 throughput.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <random>

__global__ void ops(const float* a, const float* b, const float* c, const uint32_t* u, float* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[6*i+0] = a[i] / b[i];
  o[6*i+1] = __builtin_sqrtf(fabsf(a[i]));
  o[6*i+2] = __builtin_fmaf(a[i], b[i], c[i]);
  o[6*i+3] = (float)u[i];
  o[6*i+4] = __builtin_rintf(a[i] * 1000.0f);
  o[6*i+5] = 1.0f / b[i];
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void fma_scalar(float* out, float x, float y, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0+4, a5=a0+5, a6=a0+6, a7=a0+7;
  for (int k = 0; k < iters; ++k) {
    a0 = __builtin_fmaf(a0, x, y); a1 = __builtin_fmaf(a1, x, y); a2 = __builtin_fmaf(a2, x, y); a3 = __builtin_fmaf(a3, x, y);
    a4 = __builtin_fmaf(a4, x, y); a5 = __builtin_fmaf(a5, x, y); a6 = __builtin_fmaf(a6, x, y); a7 = __builtin_fmaf(a7, x, y);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0+a1+a2+a3+a4+a5+a6+a7;
}
__global__ void fma_packed(float* out, float x, float y, int iters) {
  f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4=a0+4,a5=a0+5,a6=a0+6,a7=a0+7;
  f2 X = {x, x}, Y = {y, y};
  for (int k = 0; k < iters; ++k) {
    a0 = __builtin_elementwise_fma(a0, X, Y); a1 = __builtin_elementwise_fma(a1, X, Y);
    a2 = __builtin_elementwise_fma(a2, X, Y); a3 = __builtin_elementwise_fma(a3, X, Y);
    a4 = __builtin_elementwise_fma(a4, X, Y); a5 = __builtin_elementwise_fma(a5, X, Y);
    a6 = __builtin_elementwise_fma(a6, X, Y); a7 = __builtin_elementwise_fma(a7, X, Y);
  }
  f2 s = a0+a1+a2+a3+a4+a5+a6+a7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main() {
  const int n = 1 << 22;
  std::mt19937 rng(1234);
  std::vector<float> a(n), b(n), c(n); std::vector<uint32_t> u(n);
  for (int i = 0; i < n; ++i) {
    uint32_t r1 = rng(), r2 = rng(), r3 = rng();
    // raw random bit patterns (incl. denormals, excluding NaN/inf) mixed with "nice" values
    auto mk = [](uint32_t r) { uint32_t e = (r >> 23) & 0xff; if (e == 0xff) r ^= 0x40000000u; float f; memcpy(&f, &r, 4); return f; };
    if (i & 1) { a[i] = mk(r1); b[i] = mk(r2); c[i] = mk(r3); }
    else { a[i] = (float)(r1 % 100000) / 977.0f - 50.0f; b[i] = (float)(r2 % 100000) / 331.0f + 1e-3f; c[i] = (float)(r3 % 1000) / 7.0f; }
    u[i] = rng();
  }
  float *da, *db, *dc, *dout; uint32_t* du;
  hipMalloc(&da, n*4); hipMalloc(&db, n*4); hipMalloc(&dc, n*4); hipMalloc(&du, n*4); hipMalloc(&dout, 6*n*4);
  hipMemcpy(da, a.data(), n*4, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), n*4, hipMemcpyHostToDevice);
  hipMemcpy(dc, c.data(), n*4, hipMemcpyHostToDevice); hipMemcpy(du, u.data(), n*4, hipMemcpyHostToDevice);
  ops<<<n/256, 256>>>(da, db, dc, du, dout, n);
  std::vector<float> o(6*n); hipMemcpy(o.data(), dout, 6*n*4, hipMemcpyDeviceToHost);
  long bad[6] = {0};
  for (int i = 0; i < n; ++i) {
    float ref[6] = { a[i] / b[i], sqrtf(fabsf(a[i])), fmaf(a[i], b[i], c[i]), (float)u[i], rintf(a[i] * 1000.0f), 1.0f / b[i] };
    for (int k = 0; k < 6; ++k) {
      bool both_nan = std::isnan(ref[k]) && std::isnan(o[6*i+k]);
      if (!both_nan && fb(ref[k]) != fb(o[6*i+k])) { if (bad[k] < 3) printf("mismatch op%d i=%d a=%a b=%a c=%a host=%a gpu=%a\n", k, i, a[i], b[i], c[i], ref[k], o[6*i+k]); bad[k]++; }
    }
  }
  printf("bit-exact check over %d inputs: div=%ld sqrt=%ld fma=%ld cvt_u32=%ld rint=%ld rcp=%ld mismatches\n", n, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);

  float* dtmp; hipMalloc(&dtmp, 256*1024*4*4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 20000, blocks = 256*16;
  for (int rep = 0; rep < 2; ++rep) {
    fma_scalar<<<blocks, 256>>>(dtmp, 0.999f, 0.001f, iters);
    hipEventRecord(e0); fma_scalar<<<blocks, 256>>>(dtmp, 0.999f, 0.001f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 8 * iters * (double)blocks * 256;
    printf("scalar v_fma_f32: %.2f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    fma_packed<<<blocks, 256>>>(dtmp, 0.999f, 0.001f, iters);
    hipEventRecord(e0); fma_packed<<<blocks, 256>>>(dtmp, 0.999f, 0.001f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("packed v_pk_fma_f32: %.2f ms  %.1f TFLOP/s\n", ms, 2 * fl / ms / 1e9);
  }
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  return 0;
}
