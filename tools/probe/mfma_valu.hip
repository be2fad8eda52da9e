// Probe: v_mfma_f32_16x16x4_f32 throughput with f32 VALU work interleaved (timing experiment).
// One wave per SIMD (256 threads, 1 block per CU), NACC accumulators; each iteration issues NACC
// MFMAs whose A/B operands are produced by NV VALU ops per MFMA of the previous iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int NACC, int NV, int TPB>
__global__ __launch_bounds__(TPB, 1) void k(float a0, float* out, int iters) {
  f32x4 acc[NACC];
  float va[NACC], vb[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    va[i] = a0 + i;
    vb[i] = a0 - i;
  }
  for (int it = 0; it < iters; ++it) {
    float na[NACC], nb[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      na[i] = va[i];
      nb[i] = vb[i];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (v & 1) nb[i] = nb[i] - na[(i + 1) % NACC];
        else na[i] = na[i] + nb[(i + 3) % NACC];
      }
    }
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[i], vb[i], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      va[i] = na[i] * 0.5f;
      vb[i] = nb[i] * 0.25f;
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
void run(const char* name, F kern, int threads, int nacc, float* out, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, 1.0f, out, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, 1.0f, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfma_per_simd = (double)iters * nacc * (threads / 64) / 4;
  printf("%s: %.1f us, %.2f ns per MFMA per SIMD\n", name, ms * 1e3, ms * 1e6 / mfma_per_simd);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 512 * sizeof(float));
  const int iters = 2048;
  run("1w nacc16 valu0", k<16, 0, 256>, 256, 16, out, iters);
  run("1w nacc16 valu2(+2 scale)", k<16, 2, 256>, 256, 16, out, iters);
  run("1w nacc16 valu4(+2 scale)", k<16, 4, 256>, 256, 16, out, iters);
  run("2w nacc16 valu2(+2 scale)", k<16, 2, 512>, 512, 16, out, iters);
  run("2w nacc16 valu4(+2 scale)", k<16, 4, 512>, 512, 16, out, iters);
  (void)hipFree(out);
  return 0;
}
