// Probe (timing experiment, not product): the sparse policy head's W-row gather as k_leaf_step_ov's
// logit waves run it — 15 waves per workgroup, 4 ids per wave at a time, 16 lanes per 3.2-KB row
// (800 floats), the features in LDS — over NWG workgroups of K random ids each, from a table of
// ROWS rows (30433 = the 97-MB policy Linear, served from the Infinity Cache; 1000 = 3.2 MB,
// L2-resident). Is the gather bound per CU (time flat in NWG) or in aggregate (time grows)?
//   MODE 0: the streaming loop (4 float4 loads per lane in flight)
//   MODE 1: all 13 float4 loads of a lane issued first
// Build: hipcc -O3 --offload-arch=gfx950 -o gather tools/probe/gather.hip; run: ./gather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int F = 800, F4 = F / 4, kQ = 13;

template <int MODE>
__global__ __launch_bounds__(1024) void k_gather(const float* __restrict__ W, const int* __restrict__ ids,
                                                 const float* __restrict__ pf, float* __restrict__ out, int K) {
  __shared__ float4 f4[F4];
  const int b = blockIdx.x, wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < F4; i += 1024) f4[i] = reinterpret_cast<const float4*>(pf + (size_t)b * F)[i];
  __syncthreads();
  if (wave == 0) return;  // wave 0 descends in the real kernel
  const int nw = 15, w = wave - 1, sub = l & 15, quad = l >> 4;
  const int* id = ids + (size_t)b * K;
  for (int j0 = 4 * w; j0 < K; j0 += 4 * nw) {
    const int j = j0 + quad;
    const bool ok = j < K;
    const float4* r = reinterpret_cast<const float4*>(W + (size_t)id[ok ? j : 0] * F);
    float a0 = 0.f, a1 = 0.f;
    if (MODE == 0) {
      int q = sub;
      for (; q + 48 < F4; q += 64) {
        const float4 w0 = r[q], w1 = r[q + 16], w2 = r[q + 32], w3 = r[q + 48];
        const float4 x0 = f4[q], x1 = f4[q + 16], x2 = f4[q + 32], x3 = f4[q + 48];
        a0 += w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w;
        a1 += w1.x * x1.x + w1.y * x1.y + w1.z * x1.z + w1.w * x1.w;
        a0 += w2.x * x2.x + w2.y * x2.y + w2.z * x2.z + w2.w * x2.w;
        a1 += w3.x * x3.x + w3.y * x3.y + w3.z * x3.z + w3.w * x3.w;
      }
      for (; q < F4; q += 16) {
        const float4 w0 = r[q], x0 = f4[q];
        a0 += w0.x * x0.x + w0.y * x0.y + w0.z * x0.z + w0.w * x0.w;
      }
    } else {
      float4 wr[kQ];
#pragma unroll
      for (int k = 0; k < kQ; ++k) wr[k] = r[sub + 16 * k < F4 ? sub + 16 * k : F4 - 1];
#pragma unroll
      for (int k = 0; k < kQ; ++k) {
        const int q = sub + 16 * k;
        if (q < F4) {
          const float4 x = f4[q];
          const float d = wr[k].x * x.x + wr[k].y * x.y + wr[k].z * x.z + wr[k].w * x.w;
          if (k & 1) a1 += d; else a0 += d;
        }
      }
    }
    float a = a0 + a1;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) a += __shfl_xor(a, o, 16);
    if (sub == 0 && ok) out[(size_t)b * K + j] = a;
  }
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

int main() {
  const int maxwg = 256, K = 320, reps = 50;
  const int rows_big = 30433;
  float *W, *pf, *out;
  int* ids;
  CK(hipMalloc(&W, sizeof(float) * (size_t)rows_big * F));
  CK(hipMalloc(&pf, sizeof(float) * maxwg * F));
  CK(hipMalloc(&out, sizeof(float) * maxwg * K));
  CK(hipMalloc(&ids, sizeof(int) * maxwg * K));
  CK(hipMemset(W, 0x3C, sizeof(float) * (size_t)rows_big * F));
  CK(hipMemset(pf, 0x3C, sizeof(float) * maxwg * F));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<int> h(maxwg * K);
  std::printf("{\"K\": %d, \"row_bytes\": %d, \"runs\": [\n", K, F * 4);
  bool first = true;
  for (int rows : {30433, 1000}) {
    srand(7);
    for (auto& x : h) x = rand() % rows;
    CK(hipMemcpy(ids, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice));
    for (int mode = 0; mode < 2; ++mode) {
      for (int nwg : {8, 32, 64, 128, 256}) {
        for (int it = 0; it < 2; ++it) {  // warm-up pass, then the timed pass
          CK(hipEventRecord(e0, 0));
          for (int r = 0; r < reps; ++r) {
            if (mode == 0)
              hipLaunchKernelGGL(k_gather<0>, dim3(nwg), dim3(1024), 0, 0, W, ids, pf, out, K);
            else
              hipLaunchKernelGGL(k_gather<1>, dim3(nwg), dim3(1024), 0, 0, W, ids, pf, out, K);
          }
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
        }
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        const double bytes = (double)nwg * K * F * 4;
        std::printf("%s{\"rows\": %d, \"mode\": %d, \"nwg\": %d, \"us\": %.2f, \"GBps_total\": %.1f, \"GBps_per_wg\": %.1f}",
                    first ? "" : ",\n", rows, mode, nwg, us, bytes / us / 1e3, bytes / us / 1e3 / nwg);
        first = false;
      }
    }
  }
  std::printf("\n]}\n");
  return 0;
}
