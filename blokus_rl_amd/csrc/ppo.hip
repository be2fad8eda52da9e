// ppo.hip — the PPO trainer's device kernels around the config-5 vector env.
//
// * k_gae — PPOTrainer._compute_gae (ppo/trainer.py:177-211): the backward recursion over the
//   rollout's T steps, one lane per env, in the reference's float32 operation order
//     nnt   = 1 - done[t+1]        (next_done at t = T-1)
//     delta = (r[t] + (g * v[t+1]) * nnt) - v[t]     (next_value at t = T-1)
//     adv   = delta + (gl * nnt) * last               (gl = float32(gamma * gae_lambda), the
//                                                      Python-double product rounded once)
//   and returns = adv + v (trainer.py:83). Built with -ffp-contract=off: bit-exact with the
//   reference's torch ops. Bound: HBM (reads 3 x T x E f32 + 2E, writes 2 x T x E f32).
// * k_filter_legal — FilterLegalMoves (ppo/agent.py:27-42) from the env's bitmask instead of a
//   Python loop over `ai_possible_indexes`: v = x * m (m = 0/1), v == 0 -> -1e9 — including its
//   quirk that a legal logit that is exactly 0 is masked too. Bound: HBM (E x A f32 in + out).
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

__global__ __launch_bounds__(256) void k_gae(int T, int E, const float* __restrict__ rewards,
                                             const float* __restrict__ values, const float* __restrict__ dones,
                                             const float* __restrict__ next_value,
                                             const float* __restrict__ next_done, float g, float gl,
                                             float* __restrict__ adv, float* __restrict__ ret) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  float last = 0.0f;
  float nv = next_value[e];
  float nnt = 1.0f - next_done[e];
  for (int t = T - 1; t >= 0; --t) {
    const size_t i = (size_t)t * E + e;
    const float v = values[i];
    const float delta = (rewards[i] + (g * nv) * nnt) - v;
    last = delta + (gl * nnt) * last;
    adv[i] = last;
    ret[i] = last + v;
    nv = v;
    nnt = 1.0f - dones[i];
  }
}

__global__ __launch_bounds__(256) void k_filter_legal(const float* __restrict__ x, int E, int A,
                                                      const uint64_t* __restrict__ mask, int W,
                                                      float* __restrict__ out) {
  const size_t n = (size_t)E * A;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int e = (int)(i / A), a = (int)(i - (size_t)e * A);
    const float m = (float)((mask[(size_t)e * W + (a >> 6)] >> (a & 63)) & 1ull);
    const float v = x[i] * m;
    out[i] = v == 0.0f ? -1e9f : v;
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_ppo_gae(int T, int E, const float* rewards, const float* values, const float* dones, const float* next_value,
               const float* next_done, float gamma, float gamma_lambda, float* advantages, float* returns,
               void* stream) {
  BK_REQUIRE(T >= 0 && E >= 0 && rewards && values && dones && next_value && next_done && advantages && returns,
             "bad argument");
  if (T == 0 || E == 0) return BK_OK;
  hipLaunchKernelGGL(k_gae, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, T, E, rewards, values, dones,
                     next_value, next_done, gamma, gamma_lambda, advantages, returns);
  return launch_check("k_gae");
}

int bk_filter_legal(const float* x, int E, int A, const uint64_t* mask, int mask_words, float* out, void* stream) {
  BK_REQUIRE(x && mask && out && E >= 0 && A > 0 && mask_words * 64 >= A, "bad argument");
  if (E == 0) return BK_OK;
  const size_t n = (size_t)E * A;
  const int blocks = (int)((n + 255) / 256 < 16384 ? (n + 255) / 256 : 16384);
  hipLaunchKernelGGL(k_filter_legal, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, E, A, mask, mask_words,
                     out);
  return launch_check("k_filter_legal");
}

}  // extern "C"
