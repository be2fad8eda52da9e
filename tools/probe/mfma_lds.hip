// Probe (timing experiment, not product): cycles per v_mfma_f32_16x16x32_f16 in k_leafnet_x3's
// chunk-major pattern (triples on 25 accumulators, A operands fixed per chunk), one wave per SIMD:
//   DATA 0: all operands zero; 1: random f16 operands (the real kernels' power regime)
//   LDS 0: B operands from 4 registers; 1: B (hi, lo) read from LDS per triple by ds_read_b128,
//          PF triples ahead (the kernel's ring), conflict-free slots
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using f32x4 = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma3(f32x4& acc, const h16x8& ah, const h16x8& al, const h16x8& bh,
                                      const h16x8& bl) {
  asm volatile(
      "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0"
      : "+a"(acc)
      : "v"(ah), "v"(al), "v"(bh), "v"(bl));
}

template <int LDS, int PF>
__global__ __launch_bounds__(256, 1) void k(const h16x8* __restrict__ w, float* out, unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // LDS image: 32 KB of the operands; lane l of triple g reads slot (16 g + (l & 15)) % 512 (+ the
  // k-group's 2 KB block), distinct mod 16 within a 16-lane group
  for (int i = threadIdx.x; i < 2048; i += 256) reinterpret_cast<h16x8*>(lds)[i] = w[i];
  h16x8 a[2], b[4];
  a[0] = w[l];
  a[1] = w[64 + l];
#pragma unroll
  for (int s = 0; s < 4; ++s) b[s] = w[(2 + s) * 64 + l];
  f32x4 acc[25];
#pragma unroll
  for (int g = 0; g < 25; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  auto addr = [&](int g) { return ((16 * g + (l & 15)) % 128) * 16 + (l >> 4) * 2048; };
  h16x8 rb[8][2];
  if (LDS)
#pragma unroll
    for (int g = 0; g < PF; ++g) {
      rb[g][0] = *reinterpret_cast<const h16x8*>(lds + addr(g));
      rb[g][1] = *reinterpret_cast<const h16x8*>(lds + addr(g) + 8192);
    }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < 18; ++rep) {
#pragma unroll
    for (int g = 0; g < 25; ++g) {
      if (LDS) {
        const int gp = g + PF;
        rb[gp % 8][0] = *reinterpret_cast<const h16x8*>(lds + addr(gp));
        rb[gp % 8][1] = *reinterpret_cast<const h16x8*>(lds + addr(gp) + 8192);
        mfma3(acc[g], a[0], a[1], rb[g % 8][0], rb[g % 8][1]);
      } else {
        mfma3(acc[g], a[0], a[1], b[g & 3], b[(g + 1) & 3]);
      }
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

template <int LDS, int PF>
void run(const char* name, const h16x8* w, float* out, unsigned long long* clk) {
  const int blocks = 256;
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<LDS, PF>), dim3(blocks), dim3(256), 32768, 0, w, out, clk);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-34s cycles per MFMA %.2f\n", name, (double)h[h.size() / 2] / (18.0 * 75));
}


// Two output blocks per wave (26 accumulators = 13 pixel groups x 2 blocks of 16 channels): one
// B pair per group read from LDS feeds 6 products (the 2-blocks-per-wave form of k_leafnet_x3)
template <int PF>
__global__ __launch_bounds__(256, 1) void k2(const h16x8* __restrict__ w, float* out, unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 2048; i += 256) reinterpret_cast<h16x8*>(lds)[i] = w[i];
  h16x8 a[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) a[s] = w[s * 64 + l];
  f32x4 acc[26];
#pragma unroll
  for (int g = 0; g < 26; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  auto addr = [&](int g) { return ((16 * g + (l & 15)) % 128) * 16 + (l >> 4) * 2048; };
  h16x8 rb[8][2];
#pragma unroll
  for (int g = 0; g < PF; ++g) {
    rb[g][0] = *reinterpret_cast<const h16x8*>(lds + addr(g));
    rb[g][1] = *reinterpret_cast<const h16x8*>(lds + addr(g) + 8192);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < 18; ++rep) {
#pragma unroll
    for (int g = 0; g < 13; ++g) {
      const int gp = g + PF;
      rb[gp % 8][0] = *reinterpret_cast<const h16x8*>(lds + addr(gp));
      rb[gp % 8][1] = *reinterpret_cast<const h16x8*>(lds + addr(gp) + 8192);
      mfma3(acc[2 * g], a[0], a[1], rb[g % 8][0], rb[g % 8][1]);
      mfma3(acc[2 * g + 1], a[2], a[3], rb[g % 8][0], rb[g % 8][1]);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < 26; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (l == 0) clk[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int PF>
void run2(const char* name, const h16x8* w, float* out, unsigned long long* clk) {
  const int blocks = 256;
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k2<PF>), dim3(blocks), dim3(256), 32768, 0, w, out, clk);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-34s cycles per MFMA %.2f\n", name, (double)h[h.size() / 2] / (18.0 * 13 * 6));
}

int main() {
  h16x8* w;
  float* out;
  unsigned long long* clk;
  const int n = 4096;
  hipMalloc(&w, n * 16);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&clk, 256 * 4 * 8);
  for (int data = 0; data < 2; ++data) {
    std::vector<_Float16> hv(n * 8);
    unsigned s = 12345;
    for (auto& x : hv) {
      s = s * 1664525u + 1013904223u;
      x = data ? (_Float16)(((int)(s >> 9) % 2001 - 1000) / 1000.0f) : (_Float16)0.0f;
    }
    hipMemcpy(w, hv.data(), n * 16, hipMemcpyHostToDevice);
    printf("data %s\n", data ? "random" : "zero");
    run<0, 2>("  B in registers", w, out, clk);
    run<1, 1>("  B from LDS, 1 triple ahead", w, out, clk);
    run<1, 2>("  B from LDS, 2 triples ahead", w, out, clk);
    run<1, 4>("  B from LDS, 4 triples ahead", w, out, clk);
    run<1, 6>("  B from LDS, 6 triples ahead", w, out, clk);
    run2<1>("  2 blocks/wave, B 1 group ahead", w, out, clk);
    run2<2>("  2 blocks/wave, B 2 groups ahead", w, out, clk);
    run2<3>("  2 blocks/wave, B 3 groups ahead", w, out, clk);
  }
  return 0;
}
