// Probe: v_mfma_f32_16x16x32_f16 issue rate by accumulation pattern and A-operand register file
// (timing experiment, not product). One wave per SIMD, 4 waves per workgroup, B operands in
// registers. Patterns over 25 accumulators x 27 MFMAs each (one layer's phase B):
//   0: chunk-major  - triples (3 MFMAs on one accumulator) cycling over the 25 accumulators
//   1: group-major  - 9 triples on one accumulator, then the next (27-long dependent chains)
//   2: paired       - group-major over pairs: triples alternate between two accumulators
// AREG: the A operands (weights) come from AGPRs instead of VGPRs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using f32x4 = float __attribute__((ext_vector_type(4)));

template <bool AREG>
__device__ __forceinline__ void mfma3(f32x4& acc, const h16x8& ah, const h16x8& al, const h16x8& b) {
  if (AREG)
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0"
        : "+a"(acc)
        : "a"(ah), "a"(al), "v"(b));
  else
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0"
        : "+a"(acc)
        : "v"(ah), "v"(al), "v"(b));
}

template <int PAT, bool AREG>
__global__ __launch_bounds__(256, 1) void k(const h16x8* __restrict__ w, float* out, unsigned long long* clk) {
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  h16x8 a[9][2], b[4];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    a[j][0] = w[(j * 2) * 64 + l];
    a[j][1] = w[(j * 2 + 1) * 64 + l];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) b[s] = w[(18 + s) * 64 + l];
  f32x4 acc[25];
#pragma unroll
  for (int g = 0; g < 25; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < 10; ++rep) {
    if (PAT == 0) {
#pragma unroll
      for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int g = 0; g < 25; ++g) mfma3<AREG>(acc[g], a[j][0], a[j][1], b[(g + j) & 3]);
    } else if (PAT == 1) {
#pragma unroll
      for (int g = 0; g < 25; ++g)
#pragma unroll
        for (int j = 0; j < 9; ++j) mfma3<AREG>(acc[g], a[j][0], a[j][1], b[(g + j) & 3]);
    } else {
#pragma unroll
      for (int g = 0; g < 24; g += 2)
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          mfma3<AREG>(acc[g], a[j][0], a[j][1], b[(g + j) & 3]);
          mfma3<AREG>(acc[g + 1], a[j][0], a[j][1], b[(g + j + 1) & 3]);
        }
#pragma unroll
      for (int j = 0; j < 9; ++j) mfma3<AREG>(acc[24], a[j][0], a[j][1], b[j & 3]);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < 25; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (l == 0) clk[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int PAT, bool AREG>
void run(const char* name, const h16x8* w, float* out, unsigned long long* clk, int blocks) {
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<PAT, AREG>), dim3(blocks), dim3(256), 0, 0, w, out, clk);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-28s cycles per MFMA %.2f\n", name, (double)h[h.size() / 2] / (10.0 * 675));
}

int main() {
  h16x8* w;
  float* out;
  unsigned long long* clk;
  hipMalloc(&w, 1 << 20);
  hipMemset(w, 0, 1 << 20);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&clk, 256 * 4 * 8);
  run<0, false>("chunk-major, A in VGPR", w, out, clk, 256);
  run<0, true>("chunk-major, A in AGPR", w, out, clk, 256);
  run<1, false>("group-major, A in VGPR", w, out, clk, 256);
  run<1, true>("group-major, A in AGPR", w, out, clk, 256);
  run<2, false>("paired, A in VGPR", w, out, clk, 256);
  run<2, true>("paired, A in AGPR", w, out, clk, 256);
  return 0;
}
