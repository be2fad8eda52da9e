// trainfc.hip — the learner's policy Linear (models/blokus_nnet.py:144-146 `policy_out`, 2N^2 -> A,
// 800 -> 30433 at 20x20) evaluated only where the loss reads it. compute_loss
// (neural_network.py:138-157) takes log_softmax(masked_select(logits, mask)): only a row's legal ids
// (K ~ 100-600 of 30433) enter the loss, so the logits, their input gradient and the weight gradient
// are needed only at (row, legal id) pairs. The dense fp32 GEMMs (hipBLASLt, 3 x ~0.45 ms at batch
// 1024) become three gathers over those pairs:
//   k_splin_fwd   xs[b][j] = bias[id] + pf[b] . W[id]                     (id = ids[b][j], j < k[b])
//   k_splin_dx    dpf[b]  = sum_j g[b][j] W[id]
//   k_splin_dw    dW[a]   = sum over the rows b holding id a of g[b][j] pf[b]   (every row of dW
//                 written, zero for ids no row holds; db likewise)
// W rows (3.2 KB) come from the Infinity Cache / L2 (the 97-MB table fits the 256-MB MALL); pf rows
// from L2. Every sum has a fixed order (deterministic): lanes own fixed float4 slices of a row, the
// four waves of a workgroup take fixed residues of j (dx) or fixed quarters of b (dw) and are added
// in wave order. The (id -> rows) index for dw is a counting sort (k_splin_count + an exclusive scan
// + k_splin_fill, atomic cursors) whose within-id order is then fixed by a per-id bitmap of b in LDS.
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

using f32x4 = float __attribute__((ext_vector_type(4)));
constexpr int kFcMaxF4 = 256;  // F <= 1024 floats: 4 float4 slots per lane
constexpr int kFcSlots = kFcMaxF4 / 64;
constexpr int kFcMaxB = 4096;  // rows per launch for k_splin_dw's bitmap

__device__ __forceinline__ int fc_clamp_k(int K, int cap) { return K < 0 ? 0 : (K > cap ? cap : K); }

// lane-sum of a wave -> lane 0 (DPP tree; the same order on every call)
__device__ __forceinline__ float fc_wave_sum(float x) {
  BK_WAVE_SCAN(x, dpp_f, op_add_f);
  return readlane_f(x, kWave - 1);
}

// an id outside [0, A) (not a legal id of the table) contributes nothing: its logit is 0 and it
// enters no gradient (the loads stay inside W)
__device__ __forceinline__ bool fc_id_ok(int a, int A) { return a < A; }

__global__ __launch_bounds__(256) void k_splin_fwd(const float* __restrict__ pf, int F4, const float* __restrict__ W,
                                                   const float* __restrict__ bias, const int16_t* __restrict__ ids,
                                                   const int32_t* __restrict__ kk, int cap, int A, float* __restrict__ xs) {
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = lane_id();
  const int K = fc_clamp_k(kk[b], cap);
  const f32x4* p4 = reinterpret_cast<const f32x4*>(pf) + (size_t)b * F4;
  f32x4 pv[kFcSlots];
#pragma unroll
  for (int s = 0; s < kFcSlots; ++s) {
    const int f = l + 64 * s;
    pv[s] = f < F4 ? p4[f] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int16_t* ir = ids + (size_t)b * cap;
  float* xr = xs + (size_t)b * cap;
  // two ids per wave in flight
  for (int j = w; j < K; j += 8) {
    const int j2 = j + 4;
    const int i0 = (uint16_t)ir[j], i1 = j2 < K ? (uint16_t)ir[j2] : i0;
    const bool ok0 = fc_id_ok(i0, A), ok1 = fc_id_ok(i1, A);
    const int a0 = ok0 ? i0 : 0, a1 = ok1 ? i1 : 0;
    const f32x4* r0 = reinterpret_cast<const f32x4*>(W) + (size_t)a0 * F4;
    const f32x4* r1 = reinterpret_cast<const f32x4*>(W) + (size_t)a1 * F4;
    f32x4 w0[kFcSlots], w1[kFcSlots];
#pragma unroll
    for (int s = 0; s < kFcSlots; ++s) {
      const int f = l + 64 * s;
      w0[s] = f < F4 ? r0[f] : f32x4{0.f, 0.f, 0.f, 0.f};
      w1[s] = f < F4 ? r1[f] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int s = 0; s < kFcSlots; ++s) {
      s0 += ((pv[s].x * w0[s].x + pv[s].y * w0[s].y) + (pv[s].z * w0[s].z + pv[s].w * w0[s].w));
      s1 += ((pv[s].x * w1[s].x + pv[s].y * w1[s].y) + (pv[s].z * w1[s].z + pv[s].w * w1[s].w));
    }
    s0 = fc_wave_sum(s0);
    s1 = fc_wave_sum(s1);
    if (l == 0) {
      xr[j] = ok0 ? s0 + bias[a0] : 0.f;
      if (j2 < K) xr[j2] = ok1 ? s1 + bias[a1] : 0.f;
    }
  }
  for (int j = K + threadIdx.x; j < cap; j += 256) xr[j] = 0.f;
}

__global__ __launch_bounds__(256) void k_splin_dx(const float* __restrict__ g, int F4, const float* __restrict__ W,
                                                  const int16_t* __restrict__ ids, const int32_t* __restrict__ kk,
                                                  int cap, int A, float* __restrict__ dpf) {
  __shared__ f32x4 part[4][kFcMaxF4];
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = lane_id();
  const int K = fc_clamp_k(kk[b], cap);
  const int16_t* ir = ids + (size_t)b * cap;
  const float* gr = g + (size_t)b * cap;
  f32x4 acc[kFcSlots];
#pragma unroll
  for (int s = 0; s < kFcSlots; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j = w; j < K; j += 8) {
    const int j2 = j + 4;
    const int i0 = (uint16_t)ir[j], i1 = j2 < K ? (uint16_t)ir[j2] : i0;
    const bool ok0 = fc_id_ok(i0, A), ok1 = fc_id_ok(i1, A);
    const int a0 = ok0 ? i0 : 0, a1 = ok1 ? i1 : 0;
    const float g0 = ok0 ? gr[j] : 0.f, g1 = (j2 < K && ok1) ? gr[j2] : 0.f;
    const f32x4* r0 = reinterpret_cast<const f32x4*>(W) + (size_t)a0 * F4;
    const f32x4* r1 = reinterpret_cast<const f32x4*>(W) + (size_t)a1 * F4;
    f32x4 w0[kFcSlots], w1[kFcSlots];
#pragma unroll
    for (int s = 0; s < kFcSlots; ++s) {
      const int f = l + 64 * s;
      w0[s] = f < F4 ? r0[f] : f32x4{0.f, 0.f, 0.f, 0.f};
      w1[s] = f < F4 ? r1[f] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < kFcSlots; ++s) {
      acc[s] += g0 * w0[s];
      acc[s] += g1 * w1[s];
    }
  }
#pragma unroll
  for (int s = 0; s < kFcSlots; ++s) part[w][l + 64 * s] = acc[s];
  __syncthreads();
  f32x4* out = reinterpret_cast<f32x4*>(dpf) + (size_t)b * F4;
  for (int f = threadIdx.x; f < F4; f += 256) out[f] = ((part[0][f] + part[1][f]) + part[2][f]) + part[3][f];
}

// the (id -> pairs) index: count[a] (atomics), then slots via an exclusive scan on the host side
// (torch.cumsum) and k_splin_fill's atomic cursors; the order inside an id is fixed in k_splin_dw
__global__ __launch_bounds__(256) void k_splin_count(const int16_t* __restrict__ ids, const int32_t* __restrict__ kk,
                                                     int cap, int B, int A, int32_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * cap) return;
  const int b = (int)(i / cap), j = (int)(i - (int64_t)b * cap);
  const int a = (uint16_t)ids[i];
  if (j < fc_clamp_k(kk[b], cap) && fc_id_ok(a, A)) atomicAdd(count + a, 1);
}

__global__ __launch_bounds__(256) void k_splin_fill(const int16_t* __restrict__ ids, const int32_t* __restrict__ kk,
                                                    int cap, int B, int A, const int32_t* __restrict__ start,
                                                    int32_t* __restrict__ cursor, int32_t* __restrict__ pairs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * cap) return;
  const int b = (int)(i / cap), j = (int)(i - (int64_t)b * cap);
  const int a = (uint16_t)ids[i];
  if (j < fc_clamp_k(kk[b], cap) && fc_id_ok(a, A)) {
    pairs[start[a] + atomicAdd(cursor + a, 1)] = (int32_t)i;
  }
}

// one workgroup per id a: its pairs' rows b as a bitmap (+ j per b) in LDS, then the four waves
// take b in [q B/4, (q+1) B/4) in ascending order: dW[a] = sum g[b][j] pf[b], db[a] = sum g[b][j]
__global__ __launch_bounds__(256) void k_splin_dw(const float* __restrict__ g, const float* __restrict__ pf, int F4,
                                                  int cap, int B, const int32_t* __restrict__ start,
                                                  const int32_t* __restrict__ pairs, float* __restrict__ dW,
                                                  float* __restrict__ db) {
  __shared__ uint32_t bits[kFcMaxB / 32];
  __shared__ uint16_t jmap[kFcMaxB];
  __shared__ f32x4 part[4][kFcMaxF4];
  __shared__ float gpart[4];
  const int a = blockIdx.x, w = threadIdx.x >> 6, l = lane_id();
  const int s0 = start[a], n = start[a + 1] - s0;
  f32x4* out = reinterpret_cast<f32x4*>(dW) + (size_t)a * F4;
  if (n == 0) {  // workgroup-uniform
    for (int f = threadIdx.x; f < F4; f += 256) out[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (threadIdx.x == 0) db[a] = 0.f;
    return;
  }
  const int nw = (B + 31) / 32;
  for (int i = threadIdx.x; i < nw; i += 256) bits[i] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const int p = pairs[s0 + i];
    const int b = p / cap;
    jmap[b] = (uint16_t)(p - b * cap);
    atomicOr(&bits[b >> 5], 1u << (b & 31));
  }
  __syncthreads();
  f32x4 acc[kFcSlots];
#pragma unroll
  for (int s = 0; s < kFcSlots; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gs = 0.f;
  const int wq = (nw + 3) / 4;
  for (int i = w * wq; i < (w + 1) * wq && i < nw; ++i) {
    uint32_t m = bits[i];
    while (m) {  // wave-uniform
      const int b = 32 * i + __ffs(m) - 1;
      m &= m - 1u;
      const float gv = g[(size_t)b * cap + jmap[b]];
      const f32x4* pr = reinterpret_cast<const f32x4*>(pf) + (size_t)b * F4;
#pragma unroll
      for (int s = 0; s < kFcSlots; ++s) {
        const int f = l + 64 * s;
        if (f < F4) acc[s] += gv * pr[f];
      }
      gs += gv;
    }
  }
#pragma unroll
  for (int s = 0; s < kFcSlots; ++s) part[w][l + 64 * s] = acc[s];
  if (l == 0) gpart[w] = gs;
  __syncthreads();
  for (int f = threadIdx.x; f < F4; f += 256) out[f] = ((part[0][f] + part[1][f]) + part[2][f]) + part[3][f];
  if (threadIdx.x == 0) db[a] = ((gpart[0] + gpart[1]) + gpart[2]) + gpart[3];
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_sparse_linear_fwd(const float* pf, int B, int F, const float* W, const float* bias, int A, const int16_t* ids,
                         const int32_t* k, int cap, float* xs, void* stream) {
  BK_REQUIRE(pf && W && bias && ids && k && xs && B >= 0 && cap > 0 && A > 0, "bad argument");
  BK_REQUIRE(F > 0 && F % 4 == 0 && F / 4 <= kFcMaxF4, "bk_sparse_linear: F a multiple of 4, <= 1024");
  BK_REQUIRE(((uintptr_t)pf & 15u) == 0 && ((uintptr_t)W & 15u) == 0, "bk_sparse_linear: 16-byte aligned pf / W");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_splin_fwd, dim3(B), dim3(256), 0, (hipStream_t)stream, pf, F / 4, W, bias, ids, k, cap, A, xs);
  return launch_check("k_splin_fwd");
}

int bk_sparse_linear_dx(const float* g, int B, int F, const float* W, int A, const int16_t* ids, const int32_t* k,
                        int cap, float* dpf, void* stream) {
  BK_REQUIRE(g && W && ids && k && dpf && B >= 0 && cap > 0 && A > 0, "bad argument");
  BK_REQUIRE(F > 0 && F % 4 == 0 && F / 4 <= kFcMaxF4, "bk_sparse_linear: F a multiple of 4, <= 1024");
  BK_REQUIRE(((uintptr_t)dpf & 15u) == 0 && ((uintptr_t)W & 15u) == 0, "bk_sparse_linear: 16-byte aligned dpf / W");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_splin_dx, dim3(B), dim3(256), 0, (hipStream_t)stream, g, F / 4, W, ids, k, cap, A, dpf);
  return launch_check("k_splin_dx");
}

int bk_sparse_linear_index(const int16_t* ids, const int32_t* k, int cap, int B, int A, int32_t* count,
                           int32_t* start, int32_t* cursor, int32_t* pairs, void* stream) {
  BK_REQUIRE(ids && k && count && B >= 0 && cap > 0 && A > 0, "bad argument");
  BK_REQUIRE(!start || (cursor && pairs), "bk_sparse_linear_index: phase 2 needs cursor and pairs");
  if (B == 0) return BK_OK;
  const int64_t n = (int64_t)B * cap;
  const int grid = (int)((n + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (start == nullptr) {  // phase 1 (the caller zeroed count): per-id counts
    hipLaunchKernelGGL(k_splin_count, dim3(grid), dim3(256), 0, s, ids, k, cap, B, A, count);
    return launch_check("k_splin_count");
  }
  // phase 2 (start = exclusive scan of count, cursor zeroed): the pairs by id
  hipLaunchKernelGGL(k_splin_fill, dim3(grid), dim3(256), 0, s, ids, k, cap, B, A, start, cursor, pairs);
  return launch_check("k_splin_fill");
}

int bk_sparse_linear_dw(const float* g, const float* pf, int B, int F, int cap, int A, const int32_t* start,
                        const int32_t* pairs, float* dW, float* db, void* stream) {
  BK_REQUIRE(g && pf && start && pairs && dW && db && B >= 0 && cap > 0 && A > 0, "bad argument");
  BK_REQUIRE(F > 0 && F % 4 == 0 && F / 4 <= kFcMaxF4, "bk_sparse_linear: F a multiple of 4, <= 1024");
  BK_REQUIRE(B <= kFcMaxB, "bk_sparse_linear_dw: <= 4096 rows per call");
  BK_REQUIRE(((uintptr_t)pf & 15u) == 0 && ((uintptr_t)dW & 15u) == 0, "bk_sparse_linear: 16-byte aligned pf / dW");
  hipLaunchKernelGGL(k_splin_dw, dim3(A), dim3(256), 0, (hipStream_t)stream, g, pf, F / 4, cap, B, start, pairs, dW,
                     db);
  return launch_check("k_splin_dw");
}

}  // extern "C"
