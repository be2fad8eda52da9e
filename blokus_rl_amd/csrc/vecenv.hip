// vecenv.hip — config 5: the PPO vector env on the device (bk_vec_reset / bk_vec_step).
//
// Restates the blokus_gym `blokus-simple-v0` env as the reference's PPO path drives it
// (ppo/trainer.py:128-175 `_play_env`, :380-386 `ai_possible_indexes`; docs/README.md:47-51):
// 7x7, two colours, the agent is colour 0 and plays against a built-in uniform-random opponent
// (colour 1); reward at the end of an episode is +1 win / 0 draw / -1 loss (most squares
// placed); episodes auto-reset like gymnasium's SyncVectorEnv. One 64-lane wave per env runs the
// whole step: the agent's placement, every opponent placement until the agent is to move again
// (the skip rule may give either side several moves in a row), the reward, the reset, and the
// agent's next observation + legal mask — one launch per vector step, no host round trip.
//
// Randomness: per-env 64-bit counter state, splitmix64 output, index = (hi32 * K) >> 32 — the
// same function in oracle/vecenv_oracle.py, so trajectories compare bit for bit.
#include "../../include/blokus_engine.h"
#include "ctx.h"

namespace bk {
namespace {

__device__ __forceinline__ uint32_t rng_index(uint64_t* st, int K) {
  *st += 0x9E3779B97F4A7C15ull;
  uint64_t z = *st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(((z >> 32) * (uint64_t)(uint32_t)K) >> 32);
}

// id of the k-th set bit (0-based) of the LDS mask (wave-cooperative).
__device__ __forceinline__ int kth_legal(const DevPreset& dp, const uint32_t* m32, int k) {
  const int l = lane_id();
  int before = 0;
  for (int w0 = 0; w0 < dp.W32; w0 += kWave) {
    const int w = w0 + l;
    const uint32_t bits = w < dp.W32 ? m32[w] : 0u;
    const int cnt = __popc(bits);
    const int incl = wave_incl_scan(cnt);
    const int total = readlane_i(incl, kWave - 1);
    if (k < before + total) {  // wave-uniform
      const int excl = before + incl - cnt;
      int found = -1;
      if (k >= excl && k < excl + cnt) {
        uint32_t b = bits;
        for (int i = 0; i < k - excl; ++i) b &= b - 1u;
        found = w * 32 + __ffs(b) - 1;
      }
      const uint64_t who = __ballot(found >= 0);
      return readlane_i(found, __ffsll((unsigned long long)who) - 1);
    }
    before += total;
  }
  return -1;
}

__device__ __forceinline__ void init_state_lds(const DevPreset& dp, uint32_t* s) {
  const int l = lane_id();
  for (int w = l; w < kStateWords; w += kWave) {
    uint32_t v = 0u;
    if (w >= kWPieces && w < kWPieces + kMaxP) v = (w - kWPieces) < dp.P ? dp.full_pieces : 0u;
    if (w == kWHash) v = 0x7F4A7C15u;
    if (w == kWHash + 1) v = 0x9E3779B9u;
    s[w] = v;
  }
  __syncthreads();
}

// Agent-view outputs: obs [N*N] u8 (0 empty, 1 agent, 2 opponent) and the agent's legal mask.
__device__ __forceinline__ void write_agent_view(const DevPreset& dp, const uint32_t* s, uint64_t* fa,
                                                 uint32_t* m32, uint8_t* obs, uint64_t* mask) {
  const int l = lane_id();
  const int NN = dp.N * dp.N;
  for (int i = l; i < NN; i += kWave) {
    const int r = i / dp.N, c = i - r * dp.N;
    obs[i] = ((s[r] >> c) & 1u) ? 1 : (((s[kMaxN + r] >> c) & 1u) ? 2 : 0);
  }
  if (s[kWFlags] & kFlagOver) {  // cannot happen after auto-reset; keep the mask defined
    for (int j = l; j < dp.W64; j += kWave) mask[j] = 0ull;
    return;
  }
  build_mask(dp, s, 0, fa, m32);
  for (int j = l; j < dp.W64; j += kWave) mask[j] = (uint64_t)m32[2 * j] | ((uint64_t)m32[2 * j + 1] << 32);
}

__global__ __launch_bounds__(64) void k_vec_reset(DevPreset dp, uint32_t* states, uint64_t* rng,
                                                  const uint64_t* seeds, uint8_t* obs, uint64_t* mask) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* s = lds;
  uint64_t* fa = reinterpret_cast<uint64_t*>(lds + kStateWords);
  uint32_t* m32 = lds + kStateWords + 2 * kMaxN;
  const int e = blockIdx.x;
  init_state_lds(dp, s);
  store_state(states + (size_t)e * kStateWords, s);
  if (lane_id() == 0 && seeds) rng[e] = seeds[e];
  write_agent_view(dp, s, fa, m32, obs + (size_t)e * dp.N * dp.N, mask + (size_t)e * dp.W64);
}

__global__ __launch_bounds__(64) void k_vec_step(DevPreset dp, uint32_t* states, uint64_t* rng,
                                                 const int32_t* actions, uint8_t* obs, uint64_t* mask,
                                                 float* reward, int32_t* done) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* s = lds;
  uint64_t* fa = reinterpret_cast<uint64_t*>(lds + kStateWords);
  uint32_t* m32 = lds + kStateWords + 2 * kMaxN;
  const int e = blockIdx.x;
  const int l = lane_id();
  load_state(s, states + (size_t)e * kStateWords);
  uint64_t st = rng[e];
  __syncthreads();
  float rew = 0.0f;
  int fin = 0;
  // the agent's move (actions < 0: a uniformly random legal move, the benchmark's policy stand-in)
  int a = actions ? actions[e] : -1;
  if (a < 0) {
    build_mask(dp, s, 0, fa, m32);
    int K = 0;
    for (int w = l; w < dp.W32; w += kWave) K += __popc(m32[w]);
    K = wave_sum(K);
    a = K > 0 ? kth_legal(dp, m32, (int)rng_index(&st, K)) : -1;
  }
  bool illegal = a < 0 || apply_action(dp, s, a, fa) != 0;
  if (illegal) {  // an illegal agent action ends the episode as a loss
    rew = -1.0f;
    fin = 1;
  } else {
    // the built-in random opponent moves while it is colour 1's turn
    while (!(s[kWFlags] & kFlagOver) && s[kWToMove] == 1u) {
      build_mask(dp, s, 1, fa, m32);
      int K = 0;
      for (int w = l; w < dp.W32; w += kWave) K += __popc(m32[w]);
      K = wave_sum(K);
      const int b = kth_legal(dp, m32, (int)rng_index(&st, K));
      apply_action(dp, s, b, fa);
    }
    if (s[kWFlags] & kFlagOver) {
      const int a0 = squares_of(dp, s, 0), a1 = squares_of(dp, s, 1);
      rew = a0 > a1 ? 1.0f : (a0 < a1 ? -1.0f : 0.0f);
      fin = 1;
    }
  }
  if (fin) init_state_lds(dp, s);  // auto-reset (gymnasium vector-env semantics)
  store_state(states + (size_t)e * kStateWords, s);
  write_agent_view(dp, s, fa, m32, obs + (size_t)e * dp.N * dp.N, mask + (size_t)e * dp.W64);
  if (l == 0) {
    rng[e] = st;
    reward[e] = rew;
    done[e] = fin;
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

static size_t vec_lds(const DevPreset& dp) {
  return sizeof(uint32_t) * (size_t)(kStateWords + 2 * kMaxN + dp.W32pad);
}

extern "C" {

int bk_vec_reset(bk_ctx* c, void* states, uint64_t* rng, const uint64_t* seeds, int E, uint8_t* obs,
                 uint64_t* mask, void* stream) {
  BK_REQUIRE(c && states && rng && obs && mask && E >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  BK_REQUIRE(c->dp.P == 2, "the vector env is the 2-player preset");
  if (E == 0) return BK_OK;
  hipLaunchKernelGGL(k_vec_reset, dim3(E), dim3(kWave), vec_lds(c->dp), (hipStream_t)stream, c->dp,
                     (uint32_t*)states, rng, seeds, obs, mask);
  return launch_check("k_vec_reset");
}

int bk_vec_step(bk_ctx* c, void* states, uint64_t* rng, const int32_t* actions, int E, uint8_t* obs,
                uint64_t* mask, float* reward, int32_t* done, void* stream) {
  BK_REQUIRE(c && states && rng && obs && mask && reward && done && E >= 0, "bad argument");
  BK_REQUIRE(c->d_items, "host-only context (created with device < 0)");
  BK_REQUIRE(c->dp.P == 2, "the vector env is the 2-player preset");
  if (E == 0) return BK_OK;
  hipLaunchKernelGGL(k_vec_step, dim3(E), dim3(kWave), vec_lds(c->dp), (hipStream_t)stream, c->dp,
                     (uint32_t*)states, rng, actions, obs, mask, reward, done);
  return launch_check("k_vec_step");
}

}  // extern "C"
