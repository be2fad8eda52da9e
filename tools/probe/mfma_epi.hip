// Probe: v_mfma_f32_16x16x32_f16 issue rate with VALU work between the products (timing
// experiment for the leaf net's epilogue placement). One wave per SIMD (256 threads, 1 block per
// CU), 8 accumulators a[0:31], chains of 3 products per accumulator as k_leafnet_x3 issues them.
// Per product, one of:
//   0: nothing                              (the bare rate)
//   NV: NV independent v_add_f32 on VGPRs   (VALU beside the matrix pipe)
//   100 + NR: NR v_accvgpr_read of an accumulator the chain finished 2 accumulators earlier
//   200 + NV: 4 accumulator reads after the first product, NV v_add_f32 after each product
// Cycles per product = s_memtime delta / (iterations x 24), median over blocks.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
using h16x8 = _Float16 __attribute__((ext_vector_type(8)));

#define STR2(x) #x
#define STR(x) STR2(x)
#define MF(acc) "v_mfma_f32_16x16x32_f16 " acc ", v[0:3], v[4:7], " acc "\n\t"
#define ADDS4 "v_add_f32 v20, v21, v20\n\tv_add_f32 v22, v23, v22\n\tv_add_f32 v24, v25, v24\n\tv_add_f32 v26, v27, v26\n\t"
#define RD4(q) "v_accvgpr_read_b32 v30, a[" #q "]\n\tv_accvgpr_read_b32 v31, a[" #q "+1]\n\tv_accvgpr_read_b32 v32, a[" #q "+2]\n\tv_accvgpr_read_b32 v33, a[" #q "+3]\n\t"

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(unsigned long long* out, int iters) {
  asm volatile("v_mov_b32 v0, 0x3c003c00\n\tv_mov_b32 v1, v0\n\tv_mov_b32 v2, v0\n\tv_mov_b32 v3, v0\n\t"
               "v_mov_b32 v4, v0\n\tv_mov_b32 v5, v0\n\tv_mov_b32 v6, v0\n\tv_mov_b32 v7, v0\n\t"
               "v_mov_b32 v20, 1.0\n\tv_mov_b32 v21, 1.0\n\tv_mov_b32 v22, 1.0\n\tv_mov_b32 v23, 1.0\n\t"
               "v_mov_b32 v24, 1.0\n\tv_mov_b32 v25, 1.0\n\tv_mov_b32 v26, 1.0\n\tv_mov_b32 v27, 1.0\n\t"
               "s_nop 7" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v20", "v21", "v22", "v23", "v24",
               "v25", "v26", "v27");
  for (int q = 0; q < 32; ++q) asm volatile("v_accvgpr_write_b32 a0, 0" ::: "a0");
  asm volatile("" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "v30", "v31", "v32", "v33");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define GROUP(acc, rq)                                                              \
  if (MODE == 0) asm volatile(MF(acc) MF(acc) MF(acc) ::: "memory");               \
  else if (MODE == 4) asm volatile(MF(acc) ADDS4 MF(acc) ADDS4 MF(acc) ADDS4 ::: "memory", "v20", "v22", "v24", "v26"); \
  else if (MODE == 8) asm volatile(MF(acc) ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ::: "memory", "v20", "v22", "v24", "v26"); \
  else if (MODE == 12) asm volatile(MF(acc) ADDS4 ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ADDS4 ::: "memory", "v20", "v22", "v24", "v26"); \
  else if (MODE == 104) asm volatile(MF(acc) RD4(rq) MF(acc) MF(acc) ::: "memory", "v30", "v31", "v32", "v33"); \
  else if (MODE == 208) asm volatile(MF(acc) RD4(rq) ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ::: "memory", "v20", "v22", "v24", "v26", "v30", "v31", "v32", "v33"); \
  else if (MODE == 212) asm volatile(MF(acc) RD4(rq) ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ADDS4 MF(acc) ADDS4 ADDS4 ::: "memory", "v20", "v22", "v24", "v26", "v30", "v31", "v32", "v33");
    GROUP("a[0:3]", 24)
    GROUP("a[4:7]", 28)
    GROUP("a[8:11]", 0)
    GROUP("a[12:15]", 4)
    GROUP("a[16:19]", 8)
    GROUP("a[20:23]", 12)
    GROUP("a[24:27]", 16)
    GROUP("a[28:31]", 20)
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x % 64 == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(unsigned long long* d, int iters) {
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, d, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(1024);
  (void)hipMemcpy(h.data(), d, 1024 * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("mode %3d: %.2f cycles per MFMA (median)\n", MODE, (double)h[512] / (iters * 24.0));
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 1024 * 8);
  const int iters = 2000;
  run<0>(d, iters);
  run<4>(d, iters);
  run<8>(d, iters);
  run<12>(d, iters);
  run<104>(d, iters);
  run<208>(d, iters);
  run<212>(d, iters);
  return 0;
}
