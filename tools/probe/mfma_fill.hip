// Probe: cost of VALU fillers between v_mfma_f32_16x16x4_f32 (1 wave/SIMD, 16 accumulators,
// A from AGPR via asm, B from registers). NV fillers per MFMA; DEP: one dependent chain vs NV
// independent chains; KIND 0 f32 add, 1 u32 add, 2 v_mov. (timing experiment, not product)
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int NV, int DEP, int KIND, int BATCH = 0>
__global__ __launch_bounds__(256, 1) void k(const float* __restrict__ src, float* out, unsigned long long* clk,
                                            int iters) {
  const int l = threadIdx.x & 63;
  float ua[16], vb[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    ua[i] = src[(i * 64 + l) & 1023];
    vb[i] = src[(i * 64 + l + 512) & 1023];
  }
  f32x4 acc[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  float x[8];
  unsigned u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[i] = src[l + i];
    u[i] = (unsigned)l * (i + 1);
  }
  const float y = src[l + 100];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[p]) : "a"(ua[p]), "v"(vb[p]));
#pragma unroll
      for (int v = 0; v < (BATCH ? (p == 15 ? BATCH : 0) : NV); ++v) {
        const int c = DEP ? 0 : (v & 7);
        if (KIND == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
        else if (KIND == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(l));
        else if (KIND == 2) asm volatile("v_mov_b32 %0, %1" : "=v"(x[c]) : "v"(y));
        else asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*reinterpret_cast<double*>(&x[2 * (c & 3)])) : "v"(*reinterpret_cast<const double*>(&x[0])));
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i] + (float)u[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <typename F>
void run(const char* name, F kern, float* src, float* out, unsigned long long* clk, int iters) {
  for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, src, out, clk, iters);
  (void)hipDeviceSynchronize();
  unsigned long long c;
  (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-26s %.1f cyc/MFMA\n", name, c / ((double)iters * 16));
}

int main() {
  float *src, *out;
  unsigned long long* clk;
  (void)hipMalloc(&src, 2048 * sizeof(float));
  (void)hipMalloc(&out, 256 * 256 * sizeof(float));
  (void)hipMalloc(&clk, 512 * sizeof(unsigned long long));
  float h[2048];
  unsigned s = 12345;
  for (int i = 0; i < 2048; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
  }
  (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  const int it = 2000;
  run("none", k<0, 0, 0>, src, out, clk, it);
  run("1 f32 add", k<1, 0, 0>, src, out, clk, it);
  run("2 f32 add indep", k<2, 0, 0>, src, out, clk, it);
  run("4 f32 add indep", k<4, 0, 0>, src, out, clk, it);
  run("4 f32 add dep", k<4, 1, 0>, src, out, clk, it);
  run("1 u32 add", k<1, 0, 1>, src, out, clk, it);
  run("4 u32 add indep", k<4, 0, 1>, src, out, clk, it);
  run("1 v_mov", k<1, 0, 2>, src, out, clk, it);
  run("4 v_mov", k<4, 0, 2>, src, out, clk, it);
  run("8 f32 add indep", k<8, 0, 0>, src, out, clk, it);
  run("1 pk_add", k<1, 0, 3>, src, out, clk, it);
  run("4 pk_add indep", k<4, 0, 3>, src, out, clk, it);
  run("batch 16 add / 16 MFMA", k<0, 0, 0, 16>, src, out, clk, it);
  run("batch 32 add / 16 MFMA", k<0, 0, 0, 32>, src, out, clk, it);
  run("batch 64 add / 16 MFMA", k<0, 0, 0, 64>, src, out, clk, it);
  run("batch 32 pk_add / 16 MFMA", k<0, 0, 3, 32>, src, out, clk, it);
  return 0;
}
