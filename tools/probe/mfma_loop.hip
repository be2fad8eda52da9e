// Probe: the k_conv3x3_wino2 inner loop shape without global memory (timing experiment, not
// product): 4 waves (1/SIMD), 16 accumulators, A operand from AGPRs (inline asm) or a builtin,
// B operand from LDS (ds_read_b128 one step ahead) or registers, optional VALU op per MFMA.
// Reports ns per MFMA per SIMD and the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

template <int MODE>  // 0 builtin regs, 1 asm AGPR-A regs-B, 2 asm + LDS B, 3 asm + LDS B + VALU, 4 asm + 16 b32 LDS reads/step
__global__ __launch_bounds__(256, 1) void k(const float* __restrict__ src, float* out, unsigned long long* clk,
                                            int iters) {
  __shared__ f32x4 lds[16 * 4 * 64];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16 * 4 * 64; i += 256) lds[i] = f32x4{src[i & 1023], src[(i + 1) & 1023], src[(i + 2) & 1023], src[(i + 3) & 1023]};
  __syncthreads();
  f32x4 ur[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) ur[q] = f32x4{src[(q * 4 + l) & 1023], src[(q * 4 + l + 1) & 1023], src[(q * 4 + l + 2) & 1023], src[(q * 4 + l + 3) & 1023]};
  f32x4 acc[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  float x = src[l], y = src[l + 64];
  f32x2 pk[4] = {{x, y}, {y, x}, {x, x}, {y, y}};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    f32x4 vb[2][4];
    const float* ldsf = reinterpret_cast<const float*>(lds) + (l & 15) * 4 + (l >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) vb[0][j] = MODE >= 2 ? lds[j * 64 + l] : ur[j];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (MODE >= 4 && s + 1 < 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) vb[(s + 1) & 1][j >> 2][j & 3] = ldsf[((s + 1) * 16 + j) * 64];
      } else if (MODE >= 2 && s + 1 < 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vb[(s + 1) & 1][j] = lds[((s + 1) * 4 + j) * 64 + l];
      } else if (s + 1 < 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vb[(s + 1) & 1][j] = ur[(s * 4 + j + 7) & 63];
      }
      if (MODE >= 5 && MODE != 7) {  // 2 ds_write2_b64 (4 x 8 B per lane) into a scratch area
        float* w = reinterpret_cast<float*>(lds) + 16384 - 1024 + (l & 15) * 4 + (l >> 4) * 256;
        f32x2 a = {x, y}, b = {y, x};
        *reinterpret_cast<f32x2*>(w) = a;
        *reinterpret_cast<f32x2*>(w + 64) = b;
        *reinterpret_cast<f32x2*>(w + 128) = a;
        *reinterpret_cast<f32x2*>(w + 192) = b;
      }
      if (MODE == 5 || MODE == 7) {  // 8 packed adds
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(pk[k & 3]) : "v"(pk[(k + 1) & 3]));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const float ua = ur[4 * s + (p >> 2)][p & 3];
        const float vv = vb[s & 1][p >> 2][p & 3];
        if (MODE == 0)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua, vv, acc[p], 0, 0, 0);
        else
          asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[p]) : "a"(ua), "v"(vv));
        if (MODE == 3) x = x - y * (p & 1 ? 1.0f : -1.0f);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = x + pk[0].x + pk[1].y + pk[2].x + pk[3].y;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <typename F>
void run(const char* name, F kern, float* src, float* out, unsigned long long* clk, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, src, out, clk, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, src, out, clk, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c[2];
  (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
  const double mfma = (double)iters * 256;
  printf("%-28s %.1f us, %.2f ns/MFMA/SIMD, %.1f cyc/MFMA, clock %.2f GHz\n", name, ms * 1e3, ms * 1e6 / mfma,
         c[0] / mfma, c[0] / (c[1] / 100e6) / 1e9);
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
  const int iters = 400;
  run("builtin, B regs", k<0>, src, out, clk, iters);
  run("asm A=AGPR, B regs", k<1>, src, out, clk, iters);
  run("asm A=AGPR, B LDS", k<2>, src, out, clk, iters);
  run("asm A=AGPR, B LDS, +VALU", k<3>, src, out, clk, iters);
  run("asm A=AGPR, B LDS b32 x16", k<4>, src, out, clk, iters);
  run("b32 x16 + 8 pk + 4 ds_write_b64", k<5>, src, out, clk, iters);
  run("b32 x16 + 4 ds_write_b64", k<6>, src, out, clk, iters);
  run("b32 x16 + 8 pk", k<7>, src, out, clk, iters);
  return 0;
}
