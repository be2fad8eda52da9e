// Probe: issue rate of v_mfma_f32_16x16x4_f32 loops on gfx950 (timing experiment, not product):
// NACC independent accumulators per wave, WPS waves per SIMD, operands in registers.
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int NACC>
__device__ void body(float a, float b, float* out, int iters) {
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a + i, b, acc[i], 0, 0, 0);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(256, 1) void k1(float a, float b, float* out, int iters) { body<NACC>(a, b, out, iters); }
template <int NACC>
__global__ __launch_bounds__(512, 1) void k2(float a, float b, float* out, int iters) { body<NACC>(a, b, out, iters); }
template <int NACC>
__global__ __launch_bounds__(768, 1) void k3(float a, float b, float* out, int iters) { body<NACC>(a, b, out, iters); }

template <typename F>
void run(const char* name, F kern, int threads, int nacc, float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, 1.0f, 0.5f, out, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, 1.0f, 0.5f, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma_per_simd = (double)iters * nacc * (threads / 64) / 4;
  printf("%s threads %d nacc %d: %.1f us, %.2f ns per MFMA per SIMD (32 cyc @2.4GHz = 13.3)\n", name, threads, nacc,
         ms * 1e3, ms * 1e6 / mfma_per_simd);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 768 * sizeof(float));
  const int iters = 4096;
  run("k1", k1<4>, 256, 4, out, iters);
  run("k1", k1<16>, 256, 16, out, iters);
  run("k2", k2<4>, 512, 4, out, iters);
  run("k2", k2<16>, 512, 16, out, iters);
  run("k3", k3<4>, 768, 4, out, iters);
  run("k3", k3<8>, 768, 8, out, iters);
  hipFree(out);
  return 0;
}
