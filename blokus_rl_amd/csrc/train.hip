// train.hip — the learner side of the loop: the replay-batch loader and the
// AlphaZero policy loss over sparse search policies.
//
// * k_replay_batch — the native data loader. Decodes packed replay rows (blokus_rl_amd/replay.py:
//   state 384 B | k i32 | player i32 | z f32[4] | ids i16[cap] | pi f32[cap]) picked by an index
//   vector straight into the training batch: the observation planes (Board.canonical_board,
//   blokus_wrapper.py:134-146, the same planes bk_observe writes), the search policy (ids, pi, K)
//   and the outcome z. Replaces AlphaZeroDataset.__getitem__ + collate_dataset_fn
//   (alphazero/dataset.py:38-54) and the host->device copy of train_step (neural_network.py:64).
// * k_policy_loss / k_policy_loss_grad — the policy term of compute_loss (neural_network.py:
//   138-157) with get_valid_dist(log_softmax=True) (:159-173): per row b,
//     loss_b = -sum_j pi_bj * log_softmax(x_b[legal])_j,
//   over the row's legal ids only. The reference gathers the legal logits with masked_select and
//   pads pi to the batch's longest K; the search policy already lists exactly the legal ids in
//   ascending order (the order of masked_select), so the kernel reads the K logits those ids
//   name and never touches the other A-K entries. The gradient w.r.t. x is
//     d loss_b / d x_bi = S_b * softmax_i - pi_bi   (i legal, S_b = sum_j pi_bj), 0 otherwise.
//   Bound: latency/HBM — K (<= ~650) gathered floats + K pi + K ids per row.
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

constexpr int kRowState = kStateBytes;               // 384
constexpr int kRowK = kRowState;                     // int32 K
constexpr int kRowZ = kRowState + 8;                 // f32[4]
constexpr int kRowHeader = kRowState + 4 + 4 + 16;   // 408

__host__ __device__ inline size_t replay_stride(int cap) {
  const size_t s = (size_t)kRowHeader + (size_t)cap * 6;
  return (s + 15) / 16 * 16;
}

// One 256-thread block per batch row.
__global__ __launch_bounds__(256) void k_replay_batch(DevPreset dp, const uint8_t* __restrict__ rows, int cap,
                                                      const int64_t* __restrict__ index, int B,
                                                      float* __restrict__ obs, int16_t* __restrict__ ids,
                                                      float* __restrict__ pi, int32_t* __restrict__ kout,
                                                      float* __restrict__ z, uint8_t* __restrict__ states) {
  __shared__ uint32_t s[kStateWords];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const size_t stride = replay_stride(cap);
  const uint8_t* src = rows + (size_t)index[b] * stride;
  const uint32_t* src32 = reinterpret_cast<const uint32_t*>(src);
  if (t < kStateWords) {
    const uint32_t w = src32[t];
    s[t] = w;
    if (states) reinterpret_cast<uint32_t*>(states + (size_t)b * kStateBytes)[t] = w;
  }
  if (t == kStateWords) kout[b] = *reinterpret_cast<const int32_t*>(src + kRowK);
  if (t > kStateWords && t <= kStateWords + dp.P)
    z[(size_t)b * dp.P + (t - kStateWords - 1)] =
        reinterpret_cast<const float*>(src + kRowZ)[t - kStateWords - 1];
  // ids (2 B each) and pi (4 B each): 8-byte aligned (row base 16-aligned, header 408, cap % 64 == 0)
  const uint2* ids_src = reinterpret_cast<const uint2*>(src + kRowHeader);
  uint2* ids_dst = reinterpret_cast<uint2*>(ids + (size_t)b * cap);
  for (int i = t; i < cap / 4; i += blockDim.x) ids_dst[i] = ids_src[i];
  const uint2* pi_src = reinterpret_cast<const uint2*>(src + kRowHeader + 2 * (size_t)cap);
  uint2* pi_dst = reinterpret_cast<uint2*>(pi + (size_t)b * cap);
  for (int i = t; i < cap / 2; i += blockDim.x) pi_dst[i] = pi_src[i];
  __syncthreads();
  // observation planes: P occupancy planes, then the P to-move one-hot planes
  const int NN = dp.N * dp.N;
  const int total = 2 * dp.P * NN;
  const int tm = (int)s[kWToMove];
  float* o = obs + (size_t)b * total;
  for (int i = t; i < total; i += blockDim.x) {
    const int plane = i / NN, cell = i - plane * NN;
    float v;
    if (plane < dp.P) {
      const int r = cell / dp.N, c = cell - r * dp.N;
      v = (float)((s[plane * kMaxN + r] >> c) & 1u);
    } else {
      v = (plane - dp.P) == tm ? 1.0f : 0.0f;
    }
    o[i] = v;
  }
}

__device__ __forceinline__ int clamp_k(int K, int cap) { return K < 0 ? 0 : (K > cap ? cap : K); }

// One wave per row, 4 rows per block.
__global__ __launch_bounds__(256) void k_policy_loss(const float* __restrict__ x, int64_t ldx,
                                                     const int16_t* __restrict__ ids, const float* __restrict__ pi,
                                                     const int32_t* __restrict__ kk, int cap, int B,
                                                     float* __restrict__ loss, float* __restrict__ lse_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;  // wave-uniform
  const int l = lane_id();
  const int K = clamp_k(kk[row], cap);
  const float* xr = x + (size_t)row * ldx;
  const int16_t* ir = ids + (size_t)row * cap;
  const float* pr = pi + (size_t)row * cap;
  float m = -INFINITY;
  for (int j = l; j < K; j += kWave) m = fmaxf(m, xr[(uint16_t)ir[j]]);
  m = wave_max_f(m);
  float se = 0.0f, sp = 0.0f, dot = 0.0f;
  for (int j = l; j < K; j += kWave) {
    const float d = xr[(uint16_t)ir[j]] - m;
    const float p = pr[j];
    se += expf(d);
    sp += p;
    dot += p * d;
  }
  se = wave_sum_f(se);
  sp = wave_sum_f(sp);
  dot = wave_sum_f(dot);
  if (l == 0) {
    const float lz = K > 0 ? logf(se) : 0.0f;  // log-partition relative to the max
    loss[row] = K > 0 ? sp * lz - dot : 0.0f;
    lse_out[row] = K > 0 ? m + lz : 0.0f;
  }
}

__global__ __launch_bounds__(256) void k_policy_loss_grad(const float* __restrict__ x, int64_t ldx,
                                                          const int16_t* __restrict__ ids,
                                                          const float* __restrict__ pi,
                                                          const int32_t* __restrict__ kk, int cap, int B,
                                                          const float* __restrict__ lse, float scale,
                                                          const float* __restrict__ gscale,
                                                          float* __restrict__ g, int64_t ldg) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  if (gscale) scale *= *gscale;  // the upstream gradient, read on the device (no host sync)
  const int l = lane_id();
  const int K = clamp_k(kk[row], cap);
  const float* xr = x + (size_t)row * ldx;
  const int16_t* ir = ids + (size_t)row * cap;
  const float* pr = pi + (size_t)row * cap;
  float sp = 0.0f;
  for (int j = l; j < K; j += kWave) sp += pr[j];
  sp = wave_sum_f(sp);
  const float z = lse[row];
  float* gr = g + (size_t)row * ldg;
  for (int j = l; j < K; j += kWave) {
    const int id = (uint16_t)ir[j];
    gr[id] = scale * (sp * expf(xr[id] - z) - pr[j]);
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

size_t bk_replay_stride(int cap) { return cap > 0 ? replay_stride(cap) : 0; }

int bk_replay_batch(bk_ctx* c, const void* rows, int cap, const int64_t* index, int B, float* obs, int16_t* ids,
                    float* pi, int32_t* k, float* z, void* states, void* stream) {
  BK_REQUIRE(c && rows && index && obs && ids && pi && k && z && B >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  BK_REQUIRE(cap > 0 && cap % 64 == 0, "replay cap must be a positive multiple of 64");
  BK_REQUIRE(((uintptr_t)rows & 15u) == 0, "replay rows must be 16-byte aligned");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_replay_batch, dim3(B), dim3(256), 0, (hipStream_t)stream, c->dp, (const uint8_t*)rows, cap,
                     index, B, obs, ids, pi, k, z, (uint8_t*)states);
  return launch_check("k_replay_batch");
}

int bk_policy_loss(const float* x, int64_t ldx, const int16_t* ids, const float* pi, const int32_t* k, int cap,
                   int B, float* loss, float* lse, void* stream) {
  BK_REQUIRE(x && ids && pi && k && loss && lse && cap > 0 && B >= 0 && ldx > 0, "bad argument");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_policy_loss, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, ldx, ids, pi, k, cap,
                     B, loss, lse);
  return launch_check("k_policy_loss");
}

int bk_policy_loss_grad(const float* x, int64_t ldx, const int16_t* ids, const float* pi, const int32_t* k,
                        int cap, int B, const float* lse, float scale, const float* gscale, float* grad, int64_t ldg,
                        void* stream) {
  BK_REQUIRE(x && ids && pi && k && lse && grad && cap > 0 && B >= 0 && ldx > 0 && ldg > 0, "bad argument");
  if (B == 0) return BK_OK;
  hipLaunchKernelGGL(k_policy_loss_grad, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, ldx, ids, pi,
                     k, cap, B, lse, scale, gscale, grad, ldg);
  return launch_check("k_policy_loss_grad");
}

}  // extern "C"
