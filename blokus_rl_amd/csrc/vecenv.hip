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
#include "orient_table.h"

#include <cstdlib>

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

// ---------------------------------------------------------------------------------------------
// k_vec_step7: the same step for the 7x7 presets (config 5), G = 16 (or 8) lanes per env instead
// of a wave. A 7x7 colour is one u64 bitboard with rows at stride 8 (bit 8 r + c; column 7 is a guard
// that absorbs the +-1 column shifts), so a colour's forbidden / anchor cells are a handful of
// 64-bit shifts and the legal origins of a fixed orientation are
//   L_o = VALID_o & ~OR_k (F >> off_k) & OR_k (A >> off_k)      (off_k = 8 dr_k + dc_k)
// (compute_fa + eval_item of common.h on whole boards). The orientations are dealt round robin
// to the G lanes of an env (orientation G i + j to lane j: 2 per lane for the 919-id preset, 6
// for the 2522-id one at G = 16), each lane holding its orientations' cells / valid origins / id base in
// registers. Counting, the k-th legal id (ascending id = ascending orientation, then origin bit
// r*8 + c, as the bitmask order), the board hash (recomputed from the final board, one row key per lane) and the legal-move mask are per-lane work met by
// 3- or 4-step DPP butterflies inside the env's lanes; obs and mask are staged in LDS and leave as coalesced
// rows. Only the state words a 2-colour 7x7 game uses are read and written (occupancy rows 0..6
// of colours 0 and 1, pieces, hash, to-move, ply, flags); the rest of the 384-B state stays as
// bk_vec_reset wrote it (zero). Bitwise the trajectories of k_vec_step (tests/test_vecenv_gpu.py).
constexpr uint64_t kBoard7 = 0x007F7F7F7F7F7F7Full;  // rows 0..6 x columns 0..6 at stride 8
constexpr int kVecThreads = 256;

template <int MC, int G>
struct Vec7 {
  static constexpr int NO = MC == 4 ? 28 : 91;     // fixed orientations of the <= MC-cell pieces
  static constexpr int NP = MC == 4 ? 9 : 21;      // pieces
  static constexpr int NL = (NO + G - 1) / G;      // orientations per lane (G lanes per env)
  static constexpr int EPB = kVecThreads / G;      // envs per workgroup
  static constexpr int A = MC == 4 ? 919 : 2522;   // action ids
  static constexpr int W64 = (A + 63) / 64, W32 = (A + 31) / 32;
};
// per orientation: cells at stride 8 packed 6 bits each (unused cells repeat cell 0), valid
// origins, first id | piece << 12 | origin columns W << 17 | height h << 20 | ceil(256 / W) << 23
// (rel / W = (rel * ceil(256 / W)) >> 8 for every rel < 64, W <= 7)
struct Or7 {
  uint32_t offs, meta;
  uint64_t valid;
};
template <int MC>
struct Or7Table {
  Or7 o[Vec7<MC, 8>::NO];
  constexpr Or7Table() : o() {
    int id = 0;
    for (int k = 0; k < Vec7<MC, 8>::NO; ++k) {
      const OrientC& q = kOrient[k];
      uint32_t offs = 0;
      for (int i = 0; i < 5; ++i) offs |= (uint32_t)(q.dr[i] * 8 + q.dc[i]) << (6 * i);
      const int R = 8 - q.h, W = 8 - q.w;
      uint64_t valid = 0;
      for (int r = 0; r < R; ++r)
        for (int c = 0; c < W; ++c) valid |= 1ull << (r * 8 + c);
      o[k] = Or7{offs,
                 (uint32_t)id | ((uint32_t)q.piece << 12) | ((uint32_t)W << 17) | ((uint32_t)q.h << 20) |
                     ((uint32_t)((256 + W - 1) / W) << 23),
                 valid};
      id += R * W;
    }
  }
};
template <int MC>
__device__ constexpr Or7Table<MC> kOr7{};

// collectives over the G (8 or 16) lanes of an env, on DPP: quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror (8 lanes), then row_mirror (16 lanes)
template <int CTRL>
__device__ __forceinline__ uint32_t dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int G>
__device__ __forceinline__ int grp_sum(int x) {
  x += (int)dppu<0xB1>((uint32_t)x);
  x += (int)dppu<0x4E>((uint32_t)x);
  x += (int)dppu<0x141>((uint32_t)x);
  if (G == 16) x += (int)dppu<0x140>((uint32_t)x);
  return x;
}
template <int G, typename OP>
__device__ __forceinline__ uint64_t grp_red64(uint64_t x, OP op) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  lo = op(lo, dppu<0xB1>(lo));
  hi = op(hi, dppu<0xB1>(hi));
  lo = op(lo, dppu<0x4E>(lo));
  hi = op(hi, dppu<0x4E>(hi));
  lo = op(lo, dppu<0x141>(lo));
  hi = op(hi, dppu<0x141>(hi));
  if (G == 16) {
    lo = op(lo, dppu<0x140>(lo));
    hi = op(hi, dppu<0x140>(hi));
  }
  return ((uint64_t)hi << 32) | lo;
}
template <int G>
__device__ __forceinline__ uint32_t grp_or32(uint32_t x) {
  x |= dppu<0xB1>(x);
  x |= dppu<0x4E>(x);
  x |= dppu<0x141>(x);
  if (G == 16) x |= dppu<0x140>(x);
  return x;
}
template <int G>
__device__ __forceinline__ uint64_t grp_or64(uint64_t x) {
  return grp_red64<G>(x, [](uint32_t a, uint32_t b) { return a | b; });
}
template <int G>
__device__ __forceinline__ uint64_t grp_xor64(uint64_t x) {
  return grp_red64<G>(x, [](uint32_t a, uint32_t b) { return a ^ b; });
}
// inclusive prefix sum over lanes 0..j of the env's group (row_shr 1, 2, 4 (, 8) inside it)
template <int G>
__device__ __forceinline__ int grp_incl(int x, int j) {
  int t = (int)dppu<0x111>((uint32_t)x);
  if (j >= 1) x += t;
  t = (int)dppu<0x112>((uint32_t)x);
  if (j >= 2) x += t;
  t = (int)dppu<0x114>((uint32_t)x);
  if (j >= 4) x += t;
  if (G == 16) {
    t = (int)dppu<0x118>((uint32_t)x);
    if (j >= 8) x += t;
  }
  return x;
}
// bit index of the k-th (0-based) set bit of x (k < popcount(x)): binary search on popcounts
__device__ __forceinline__ int kth_bit64(uint64_t x64, int k) {
  const int c0 = __popc((uint32_t)x64);
  const bool up = k >= c0;
  uint32_t x = up ? (uint32_t)(x64 >> 32) : (uint32_t)x64;  // 32-bit ops from here
  int pos = up ? 32 : 0;
  k = up ? k - c0 : k;
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    const uint32_t lo = x & ((1u << w) - 1u);
    const int c = __popc(lo);
    const bool u = k >= c;
    k = u ? k - c : k;
    x = u ? x >> w : lo;
    pos += u ? w : 0;
  }
  return pos;
}

// ---------------------------------------------------------------------------------------------
// The agent's move drawn from its policy, as the reference's PPO rollout draws it
// (ppo/trainer.py:144-155 -> CnnAgent.get_action_and_value, ppo/agent.py:148-156: the actor's
// logits through FilterLegalMoves, :27-42, then Categorical(logits).sample() and .log_prob()), by
// the 16 lanes of an env: fused into the env step (k_vec_step7<.., POL>, which has the agent's
// legal mask in registers at the step's start) and standalone (k_vec_policy, mask words from HBM).
// Lane j owns mask words w = j, j + 16, ... (< W64); its candidates are those words' set bits
// (ids ascending), minus ids whose logit is exactly 0 under the reference filter's quirk; with no
// candidate in the env, every id in [0, A) at logit -1e9 (the reference's all -1e9 row: uniform).
// Only the candidates' logits are read (~22 of 919 per env on config-5 boards). The draw is an
// inverse CDF with a fixed, restatable arithmetic (oracle/vecenv_oracle.py policy_sample):
//   m = max candidate logit (16-lane butterfly); p = bk_expf(x - m); s_j = lane j's sum, ids
//   ascending; incl = 16-lane Hillis-Steele scan (DPP row_shr 1, 2, 4, 8); S = incl_15;
//   u = (z >> 40) 2^-24 from the env's splitmix64 stream (one draw, before the opponent's);
//   target = S u; lane = first with incl > target (else the last with s > 0); inside it, walking
//   from incl_{lane-1}: the first candidate whose running sum passes the target (else its last
//   p > 0); logp = x_a - (m + bk_logf(S))  (torch's logsumexp form: the all -1e9 row gives 0).
// exp / log from + - * / only (-ffp-contract=off): bitwise reproducible by numpy float32.
__device__ __forceinline__ float bk_expf(float x) {  // x <= 0; below -80 (e^-80 < 2^-115): 0
  if (!(x >= -80.0f)) return 0.0f;
  const float n = __builtin_rintf(x * 1.44269502f);
  const float r = (x - n * 0.693145752f) - n * 1.42860677e-6f;
  float p = 1.38888892e-3f;
  p = p * r + 8.33333377e-3f;
  p = p * r + 4.16666679e-2f;
  p = p * r + 0.166666672f;
  p = p * r + 0.5f;
  p = p * r + 1.0f;
  p = p * r + 1.0f;
  return p * __int_as_float(((int)n + 127) << 23);
}
__device__ __forceinline__ float bk_logf(float x) {  // x >= 1, finite
  const int bits = __float_as_int(x);
  int e = ((bits >> 23) & 255) - 127;
  float f = __int_as_float((bits & 0x7FFFFF) | 0x3F800000);  // [1, 2)
  if (f > 1.41421354f) {
    f = f * 0.5f;
    e += 1;
  }
  const float s = (f - 1.0f) / (f + 1.0f);
  const float s2 = s * s;
  float q = 0.111111112f;
  q = q * s2 + 0.142857149f;
  q = q * s2 + 0.200000003f;
  q = q * s2 + 0.333333343f;
  q = q * s2 + 1.0f;
  return (float)e * 0.693147182f + (2.0f * s) * q;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// -> the drawn id (the same in the env's 16 lanes; A when every logit was non-finite: the env then
// takes it as an illegal move), logp in every lane; st advanced by one draw. wd: lane j's words.
template <int W64, int A, bool ZQ>
__device__ __forceinline__ int policy_draw16(const float* __restrict__ row, const uint64_t (&wd)[(W64 + 15) / 16],
                                             uint64_t& st, float& logp) {
  constexpr int NW = (W64 + 15) / 16;
  constexpr int CAPW = NW == 1 ? 8 : 4;  // candidates per word whose logits load up front
  const int l = lane_id(), j = l & 15, gb = l & ~15;
  float xr[NW][CAPW];
  int idr[NW][CAPW], nr[NW];
  uint64_t rem[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    uint64_t b = (j + 16 * i < W64) ? wd[i] : 0ull;
    nr[i] = 0;
#pragma unroll
    for (int c = 0; c < CAPW; ++c) {
      const int pos = b ? __ffsll((unsigned long long)b) - 1 : 0;
      idr[i][c] = 64 * (j + 16 * i) + pos;
      nr[i] += b ? 1 : 0;
      b &= b - 1ull;
    }
    rem[i] = b;
#pragma unroll
    for (int c = 0; c < CAPW; ++c) xr[i][c] = c < nr[i] ? row[idr[i][c]] : 0.0f;
  }
  // every candidate in order: f(x, id) (the register ones, then the rest of the word: rare)
  auto each = [&](auto&& f) {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
#pragma unroll
      for (int c = 0; c < CAPW; ++c)
        if (c < nr[i] && (!ZQ || xr[i][c] != 0.0f)) f(xr[i][c], idr[i][c]);
      uint64_t b = rem[i];
      while (b) {
        const int id = 64 * (j + 16 * i) + __ffsll((unsigned long long)b) - 1;
        b &= b - 1ull;
        const float x = row[id];
        if (!ZQ || x != 0.0f) f(x, id);
      }
    }
  };
  float m = -INFINITY;
  bool has = false;
  each([&](float x, int) {
    m = fmaxf(m, x);
    has = true;
  });
  const bool none = ((__ballot(has) >> gb) & 0xFFFFull) == 0ull;  // group-uniform
  m = fmaxf(m, dppf<0xB1>(m));
  m = fmaxf(m, dppf<0x4E>(m));
  m = fmaxf(m, dppf<0x141>(m));
  m = fmaxf(m, dppf<0x140>(m));
  if (none) m = -1e9f;
  // valid ids of the lane's words (the no-candidate row)
  int nvalid = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int w = j + 16 * i, lim = A - 64 * w;
    nvalid += w < W64 ? (lim >= 64 ? 64 : lim) : 0;
  }
  float s = 0.0f;
  if (none) {
    for (int c = 0; c < nvalid; ++c) s = s + 1.0f;
  } else {
    each([&](float x, int) { s = s + bk_expf(x - m); });
  }
  float incl = s, t = dppf<0x111>(incl);
  if (j >= 1) incl = t + incl;
  t = dppf<0x112>(incl);
  if (j >= 2) incl = t + incl;
  t = dppf<0x114>(incl);
  if (j >= 4) incl = t + incl;
  t = dppf<0x118>(incl);
  if (j >= 8) incl = t + incl;
  const float S = __shfl(incl, gb + 15);
  const uint64_t z = mix64(st);  // = the env's splitmix64 output (rng_index's draw)
  st += 0x9E3779B97F4A7C15ull;
  const float target = S * ((float)(uint32_t)(z >> 40) * 0x1p-24f);
  const uint32_t over = (uint32_t)((__ballot(incl > target) >> gb) & 0xFFFFull);
  const uint32_t pos = (uint32_t)((__ballot(s > 0.0f) >> gb) & 0xFFFFull);
  const int sel = over ? __ffs(over) - 1 : (pos ? 31 - __clz(pos) : 0);
  const float excl = __shfl(incl, gb + (sel > 0 ? sel - 1 : 0));
  int pick = -1;
  float xp = 0.0f;
  if (j == sel) {
    float acc = sel > 0 ? excl : 0.0f;
    if (none) {
      for (int c = 0; c < nvalid; ++c) {
        acc = acc + 1.0f;
        if (acc > target) {
          pick = 64 * (j + 16 * (c >> 6)) + (c & 63);
          break;
        }
      }
      if (pick < 0 && nvalid > 0) pick = 64 * (j + 16 * ((nvalid - 1) >> 6)) + ((nvalid - 1) & 63);
      xp = -1e9f;
    } else {
      int last = -1;
      float xl = 0.0f;
      each([&](float x, int id) {
        if (pick >= 0) return;
        const float p = bk_expf(x - m);
        if (p > 0.0f) {
          acc = acc + p;
          last = id;
          xl = x;
          if (acc > target) {
            pick = id;
            xp = x;
          }
        }
      });
      if (pick < 0) {
        pick = last;
        xp = xl;
      }
    }
  }
  pick = __shfl(pick, gb + sel);
  xp = __shfl(xp, gb + sel);
  logp = pick >= 0 ? xp - (m + bk_logf(S)) : __int_as_float(0x7FC00000);
  return pick >= 0 ? pick : A;
}

#ifdef BK_VEC_STAMP
// diagnostic build only: per wave (lane 0), s_memtime at the phases of k_vec_step7 (bk_vec_stamps)
__device__ unsigned long long g_vec_stamps[4096][8];
#define VSTAMP(i)                                                                   \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0) {                                                  \
      const int w_ = blockIdx.x * (kVecThreads / 64) + (threadIdx.x >> 6);          \
      if (w_ < 4096) g_vec_stamps[w_][i] = __builtin_amdgcn_s_memtime();            \
    }                                                                               \
  } while (0)
#else
#define VSTAMP(i) \
  do {            \
  } while (0)
#endif

// POL (G = 16 only): 0 = the agent's id given (actions) or drawn uniformly; 1 / 2 = drawn from
// its policy logits by policy_draw16 (2: with the reference filter's zero-logit quirk), the id and
// its log-prob written to act_out / logp_out
template <int MC, int G, int POL = 0>
__global__ __launch_bounds__(kVecThreads) void k_vec_step7(uint32_t* states, uint64_t* rng,
                                                          const int32_t* __restrict__ actions, int E,
                                                          uint8_t* __restrict__ obs, uint64_t* __restrict__ mask,
                                                          float* __restrict__ reward, int32_t* __restrict__ done,
                                                          const float* __restrict__ logits = nullptr,
                                                          int32_t* __restrict__ act_out = nullptr,
                                                          float* __restrict__ logp_out = nullptr) {
  static_assert(POL == 0 || G == 16, "the policy draw runs on 16 lanes per env");
  using V = Vec7<MC, G>;
  constexpr int NL = V::NL, kVecEnvsPerBlock = V::EPB;
  __shared__ uint32_t m32[kVecEnvsPerBlock][V::W32 + 1];
  __shared__ __attribute__((aligned(16))) uint8_t ob[kVecEnvsPerBlock * 49 + 16];
  const int tid = threadIdx.x, j = tid & (G - 1), le = tid / G;
  const int e0 = blockIdx.x * kVecEnvsPerBlock;
  VSTAMP(0);
  const int e = e0 + le;
  const bool live = e < E;
  const int es = live ? e : E - 1;  // a spare lane group mirrors the last env and stores nothing
  for (int w = j; w < V::W32 + 1; w += G) m32[le][w] = 0u;  // the env's mask words (its own lanes)

  // this lane's orientations (8 i + j): cells, valid origins, meta
  uint32_t offs[NL], meta[NL], off[NL][MC];
  uint64_t valid[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int k = G * i + j;
    const Or7 q = kOr7<MC>.o[k < V::NO ? k : 0];
    offs[i] = q.offs;
    meta[i] = q.meta;
    valid[i] = k < V::NO ? q.valid : 0ull;
#pragma unroll
    for (int c = 0; c < MC; ++c) off[i][c] = (q.offs >> (6 * c)) & 63u;  // cells past the piece repeat cell 0
  }
  // the state words of a 7x7 / 2-colour game
  const uint32_t* g = states + (size_t)es * kStateWords;
  uint64_t occ[2];
  {
    const uint4 a0 = *reinterpret_cast<const uint4*>(g), a1 = *reinterpret_cast<const uint4*>(g + 4);
    const uint4 b0 = *reinterpret_cast<const uint4*>(g + kMaxN), b1 = *reinterpret_cast<const uint4*>(g + kMaxN + 4);
    occ[0] = (uint64_t)a0.x | (uint64_t)a0.y << 8 | (uint64_t)a0.z << 16 | (uint64_t)a0.w << 24 |
             (uint64_t)a1.x << 32 | (uint64_t)a1.y << 40 | (uint64_t)a1.z << 48;
    occ[1] = (uint64_t)b0.x | (uint64_t)b0.y << 8 | (uint64_t)b0.z << 16 | (uint64_t)b0.w << 24 |
             (uint64_t)b1.x << 32 | (uint64_t)b1.y << 40 | (uint64_t)b1.z << 48;
  }
  const uint4 w80 = *reinterpret_cast<const uint4*>(g + kWPieces);  // pieces of colours 0..3
  const uint4 w84 = *reinterpret_cast<const uint4*>(g + kWHash);    // hash lo, hi, to-move, ply
  uint32_t pieces[2] = {w80.x, w80.y};
  int to_move = (int)w84.z;
  uint32_t ply = w84.w, flags = g[kWFlags];
  uint64_t st = rng[es];

  // legal origins of colour q for this lane's orientations into L; returns the env's legal-move
  // count (also kept in lastK)
  uint64_t L[NL];
  int lastK = 0;
  auto legal = [&](int q) {
    const uint64_t own = occ[q], all = occ[0] | occ[1];
    const uint64_t F = all | own << 1 | own >> 1 | own << 8 | own >> 8;
    const uint64_t A = own ? ((own << 9 | own << 7 | own >> 7 | own >> 9) & kBoard7) : (q == 0 ? 1ull : 1ull << 54);
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      uint64_t fo = 0, ao = 0;
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        fo |= F >> off[i][k];
        ao |= A >> off[i][k];
      }
      const bool have = (pieces[q] >> ((meta[i] >> 12) & 31u)) & 1u;
      L[i] = have ? (valid[i] & ~fo & ao) : 0ull;
      cnt += __popcll(L[i]);
    }
    lastK = grp_sum<G>(cnt);
    return lastK;
  };
  // the k-th legal id in ascending order -> (id, the orientation's offs, meta, origin bit), the
  // same in every lane of the env's group
  struct Pick {
    int id;
    uint32_t offs, meta;
    int org;
  };
  auto kth = [&](int k) {
    int before = 0;
    uint32_t sel = 0;  // id | org << 12 | 1 << 31 from the owning lane
    uint32_t so = 0, sm = 0;
    // orientations i, i + 1 scanned together: counts (<= 49 each, <= 784 per group) in 16-bit halves
    int inclp[(NL + 1) / 2], totp[(NL + 1) / 2];
#pragma unroll
    for (int h = 0; h < (NL + 1) / 2; ++h) {
      const int x = __popcll(L[2 * h]) | (2 * h + 1 < NL ? __popcll(L[2 * h + 1]) << 16 : 0);
      inclp[h] = grp_incl<G>(x, j);
      totp[h] = grp_sum<G>(x);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = __popcll(L[i]);
      const int sh = 16 * (i & 1);
      const int incl = (inclp[i / 2] >> sh) & 0xFFFF, tot = (totp[i / 2] >> sh) & 0xFFFF;
      const int kk = k - before - (incl - c);
      if (kk >= 0 && kk < c) {
        const int pos = kth_bit64(L[i], kk);
        const int W = (int)((meta[i] >> 17) & 7u);
        const int id = (int)(meta[i] & 0xFFFu) + (pos >> 3) * W + (pos & 7);
        sel = (uint32_t)id | ((uint32_t)pos << 12) | (1u << 31);
        so = offs[i];
        sm = meta[i];
      }
      before += tot;
    }
    sel = grp_or32<G>(sel);
    const uint64_t om = grp_or64<G>(((uint64_t)sm << 32) | so);
    return Pick{(int)(sel & 0xFFFu), (uint32_t)om, (uint32_t)(om >> 32), (int)((sel >> 12) & 63u)};
  };
  // decode a given id -> the same Pick; id -1 when it is out of range or not a legal origin of the
  // colour whose origins L holds (the owning lane tests its bit)
  auto decode = [&](int a) {
    uint32_t sel = 0;
    uint32_t so = 0, sm = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int base = (int)(meta[i] & 0xFFFu), W = (int)((meta[i] >> 17) & 7u), h = (int)((meta[i] >> 20) & 7u);
      const int rel = a - base;
      if (valid[i] && rel >= 0 && rel < (8 - h) * W) {
        const int r = (rel * (int)(meta[i] >> 23)) >> 8, c = rel - r * W;
        if ((L[i] >> (r * 8 + c)) & 1ull) {
          sel = (uint32_t)a | ((uint32_t)(r * 8 + c) << 12) | (1u << 31);
          so = offs[i];
          sm = meta[i];
        }
      }
    }
    sel = grp_or32<G>(sel);
    const uint64_t om = grp_or64<G>(((uint64_t)sm << 32) | so);
    return Pick{(sel >> 31) ? (int)(sel & 0xFFFu) : -1, (uint32_t)om, (uint32_t)(om >> 32), (int)((sel >> 12) & 63u)};
  };
  // place pick p for colour q: cells, pieces, ply (the board hash is recomputed once at the end)
  auto place = [&](int q, const Pick& p) {
    uint64_t cells = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) cells |= 1ull << ((p.offs >> (6 * k)) & 63u);
    occ[q] |= cells << p.org;
    pieces[q] &= ~(1u << ((p.meta >> 12) & 31u));
    ply += 1u;
  };
  // advance_turn (common.h) after colour p placed; last_q: the colour whose L the last legal()
  // call left (-1 none): the next mover's origins stay in L for the caller
  int last_q = -1;
  auto advance = [&](int p) {
    int next = -1;
    for (int d = 1; d <= 2; ++d) {
      const int q = (p + d) & 1;
      if ((flags >> (kFlagDeadShift + q)) & 1u) continue;
      const int K = legal(q);
      last_q = q;
      if (K > 0) {
        next = q;
        break;
      }
      flags |= 1u << (kFlagDeadShift + q);
    }
    if (next < 0) {
      flags |= kFlagOver;
      next = (p + 1) & 1;
      last_q = -1;
    }
    to_move = next;
  };

  // each orientation's legal origins compacted from stride-8 rows to its (R x W)-bit field
  // (<= 49 bits), ORed into the env's LDS words at the orientation's first id (<= 3 words)
  auto assemble = [&]() {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int base = (int)(meta[i] & 0xFFFu), W = (int)((meta[i] >> 17) & 7u);
      uint64_t f = 0;
#pragma unroll
      for (int r = 0; r < 7; ++r) f |= (uint64_t)((uint32_t)(L[i] >> (8 * r)) & 0x7Fu) << (r * W);
      if (f) {
        const int w = base >> 5, sh = base & 31;
        const uint64_t x = f << sh;
        const uint32_t x2 = sh ? (uint32_t)(f >> (64 - sh)) : 0u;
        if ((uint32_t)x) atomicOr(&m32[le][w], (uint32_t)x);
        if ((uint32_t)(x >> 32)) atomicOr(&m32[le][w + 1], (uint32_t)(x >> 32));
        if (x2) atomicOr(&m32[le][w + 2], x2);
      }
    }
  };

  float rew = 0.0f;
  int fin = 0;
  int a = actions ? actions[es] : -1;
  const int K0 = legal(0);  // the agent (colour 0) is to move at every step start
  VSTAMP(1);
  if (POL) {  // the agent's id drawn from its policy over its legal mask (assembled in LDS)
    wave_lds_sync();  // the group's zeroing of its words (kernel start) is done
    assemble();
    wave_lds_sync();
    constexpr int NW = (V::W64 + 15) / 16;
    uint64_t wd[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int w = j + 16 * i;
      wd[i] = w < V::W64 ? ((uint64_t)m32[le][2 * w] | ((uint64_t)m32[le][2 * w + 1] << 32)) : 0ull;
    }
    float lp;
    a = policy_draw16<V::W64, V::A, POL == 2>(logits + (size_t)es * V::A, wd, st, lp);
    if (live && j == 4) {
      act_out[e] = a;
      logp_out[e] = lp;
    }
    wave_lds_sync();  // every lane has read the words
    for (int w = j; w < V::W32 + 1; w += G) m32[le][w] = 0u;  // re-zeroed for the output mask
  }
  // the agent's move: the given id if it is legal, else (a < 0) a uniformly random legal one
  Pick pk = a >= 0 ? decode(a) : (K0 > 0 ? kth((int)rng_index(&st, K0)) : Pick{-1, 0u, 0u, 0});
  if (pk.id < 0) {  // an illegal agent action (or no legal move) ends the episode as a loss
    rew = -1.0f;
    fin = 1;
  } else {
    place(0, pk);
    advance(0);
    VSTAMP(2);
    // the built-in random opponent moves while it is colour 1's turn (advance left its origins in L)
    while (!(flags & kFlagOver) && to_move == 1) {
      const Pick pb = kth((int)rng_index(&st, lastK));
      place(1, pb);
      advance(1);
    }
    if (flags & kFlagOver) {
      const int a0 = __popcll(occ[0]), a1 = __popcll(occ[1]);
      rew = a0 > a1 ? 1.0f : (a0 < a1 ? -1.0f : 0.0f);
      fin = 1;
    }
  }
  VSTAMP(3);
  if (fin) {  // auto-reset (gymnasium vector-env semantics): init_state_lds's words
    occ[0] = occ[1] = 0ull;
    pieces[0] = pieces[1] = (1u << V::NP) - 1u;
    to_move = 0;
    ply = 0u;
    flags = 0u;
    last_q = -1;
  }
  if (last_q != 0) legal(0);  // the agent's legal origins for its mask
  // the board hash (a board-only key: the seed ^ the row keys of the non-empty colour rows, as
  // bk_vec_reset / k_next_state keep it) from the final board, one row per lane
  uint64_t hash;
  {
    uint64_t hx = 0;
#pragma unroll
    for (int k0 = 0; k0 < 14; k0 += G) {
      const int k = k0 + j, q = k >= 7 ? 1 : 0, row = k - 7 * q;
      const uint32_t bits = k < 14 ? (uint32_t)(occ[q] >> (8 * row)) & 0x7Fu : 0u;
      if (bits) hx ^= row_key(q, row, bits);
    }
    hash = 0x9E3779B97F4A7C15ull ^ grp_xor64<G>(hx);
  }
  VSTAMP(4);

  // ---- outputs: the state words, rng, reward, done (lanes 0..3 of the env's group); obs and mask via LDS
  if (live) {
    uint32_t* gs = states + (size_t)e * kStateWords;
    if (j == 0) {
      *reinterpret_cast<uint4*>(gs) = make_uint4((uint32_t)occ[0] & 0x7Fu, (uint32_t)(occ[0] >> 8) & 0x7Fu,
                                                 (uint32_t)(occ[0] >> 16) & 0x7Fu, (uint32_t)(occ[0] >> 24) & 0x7Fu);
      *reinterpret_cast<uint4*>(gs + 4) = make_uint4((uint32_t)(occ[0] >> 32) & 0x7Fu, (uint32_t)(occ[0] >> 40) & 0x7Fu,
                                                     (uint32_t)(occ[0] >> 48) & 0x7Fu, 0u);
    } else if (j == 1) {
      *reinterpret_cast<uint4*>(gs + kMaxN) = make_uint4((uint32_t)occ[1] & 0x7Fu, (uint32_t)(occ[1] >> 8) & 0x7Fu,
                                                         (uint32_t)(occ[1] >> 16) & 0x7Fu,
                                                         (uint32_t)(occ[1] >> 24) & 0x7Fu);
      *reinterpret_cast<uint4*>(gs + kMaxN + 4) =
          make_uint4((uint32_t)(occ[1] >> 32) & 0x7Fu, (uint32_t)(occ[1] >> 40) & 0x7Fu,
                     (uint32_t)(occ[1] >> 48) & 0x7Fu, 0u);
    } else if (j == 2) {
      *reinterpret_cast<uint4*>(gs + kWPieces) = make_uint4(pieces[0], pieces[1], 0u, 0u);
      *reinterpret_cast<uint4*>(gs + kWHash) = make_uint4((uint32_t)hash, (uint32_t)(hash >> 32), (uint32_t)to_move, ply);
      gs[kWFlags] = flags;
    } else if (j == 3) {
      rng[e] = st;
      reward[e] = rew;
      done[e] = fin;
    }
    // obs: lane j < 7 writes row j (0 empty, 1 colour 0, 2 colour 1)
    if (j < 7) {
      const uint32_t r0 = (uint32_t)(occ[0] >> (8 * j)) & 0x7Fu, r1 = (uint32_t)(occ[1] >> (8 * j)) & 0x7Fu;
#pragma unroll
      for (int c = 0; c < 7; ++c) ob[le * 49 + j * 7 + c] = ((r0 >> c) & 1u) ? 1 : (((r1 >> c) & 1u) ? 2 : 0);
    }
    // mask: the agent's legal origins as the env's LDS words
    wave_lds_sync();  // the group's zeroing of its words is done
    assemble();
  }
  VSTAMP(5);
  __syncthreads();
  VSTAMP(6);
  // the block's envs are contiguous: obs rows as dwords, mask rows as u64 (coalesced)
  const int nenv = min(kVecEnvsPerBlock, E - e0);
  {
    uint8_t* o = obs + (size_t)e0 * 49;  // 16-B aligned: e0 * 49 is a multiple of 32 * 49 = 98 x 16
    if (nenv == kVecEnvsPerBlock) {
      if (tid < kVecEnvsPerBlock * 49 / 16)
        reinterpret_cast<uint4*>(o)[tid] = reinterpret_cast<const uint4*>(ob)[tid];
    } else {
      for (int i = tid; i < nenv * 49; i += kVecThreads) o[i] = ob[i];
    }
  }
  for (int i = tid; i < nenv * V::W64; i += kVecThreads) {
    const int le2 = i / V::W64, w = i - le2 * V::W64;
    mask[(size_t)(e0 + le2) * V::W64 + w] = (uint64_t)m32[le2][2 * w] | ((uint64_t)m32[le2][2 * w + 1] << 32);
  }
  VSTAMP(7);
}

// k_vec_policy: policy_draw16 alone (the rollout's draw without the step: the agent's legal mask
// words from HBM, as bk_vec_reset / bk_vec_step leave them); 16 lanes per env, 16 envs per block.
template <int MC, bool ZQ>
__global__ __launch_bounds__(kVecThreads) void k_vec_policy(const float* __restrict__ logits,
                                                            const uint64_t* __restrict__ mask,
                                                            uint64_t* __restrict__ rng, int E,
                                                            int32_t* __restrict__ act, float* __restrict__ logp) {
  using V = Vec7<MC, 16>;
  constexpr int NW = (V::W64 + 15) / 16;
  const int j = threadIdx.x & 15, e = blockIdx.x * (kVecThreads / 16) + (threadIdx.x >> 4);
  const int es = e < E ? e : E - 1;  // a spare lane group mirrors the last env and stores nothing
  uint64_t wd[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int w = j + 16 * i;
    wd[i] = w < V::W64 ? mask[(size_t)es * V::W64 + w] : 0ull;
  }
  uint64_t st = rng[es];
  float lp;
  const int a = policy_draw16<V::W64, V::A, ZQ>(logits + (size_t)es * V::A, wd, st, lp);
  if (e < E && j == 0) {
    act[e] = a;
    logp[e] = lp;
    rng[e] = st;
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

static size_t vec_lds(const DevPreset& dp) {
  return sizeof(uint32_t) * (size_t)(kStateWords + 2 * kMaxN + dp.W32pad);
}

extern "C" {

#ifdef BK_VEC_STAMP
int bk_vec_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vec_stamps), sizeof(g_vec_stamps)) == hipSuccess ? 0 : -1;
}
#endif

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
  const char* g = getenv("BK_VEC_WAVE");  // A/B: the one-wave-per-env kernel on 7x7 too
  if (c->dp.N == 7 && (c->dp.num_pieces == 9 || c->dp.num_pieces == 21) && !(g && atoi(g))) {
    const char* gl = getenv("BK_VEC_LANES");  // A/B: lanes per env (8 or 16)
    const int G = gl && atoi(gl) == 8 ? 8 : 16;
    const dim3 grid((E + kVecThreads / G - 1) / (kVecThreads / G));
    hipStream_t st = (hipStream_t)stream;
    uint32_t* sp = (uint32_t*)states;
    if (c->dp.num_pieces == 9 && G == 16)
      hipLaunchKernelGGL((k_vec_step7<4, 16>), grid, dim3(kVecThreads), 0, st, sp, rng, actions, E, obs, mask, reward, done);
    else if (c->dp.num_pieces == 9)
      hipLaunchKernelGGL((k_vec_step7<4, 8>), grid, dim3(kVecThreads), 0, st, sp, rng, actions, E, obs, mask, reward, done);
    else if (G == 16)
      hipLaunchKernelGGL((k_vec_step7<5, 16>), grid, dim3(kVecThreads), 0, st, sp, rng, actions, E, obs, mask, reward, done);
    else
      hipLaunchKernelGGL((k_vec_step7<5, 8>), grid, dim3(kVecThreads), 0, st, sp, rng, actions, E, obs, mask, reward, done);
    return launch_check("k_vec_step7");
  }
  hipLaunchKernelGGL(k_vec_step, dim3(E), dim3(kWave), vec_lds(c->dp), (hipStream_t)stream, c->dp,
                     (uint32_t*)states, rng, actions, obs, mask, reward, done);
  return launch_check("k_vec_step");
}

int bk_vec_policy(bk_ctx* c, const float* logits, const uint64_t* mask, uint64_t* rng, int E, int zero_masked,
                  int32_t* actions, float* logp, void* stream) {
  BK_REQUIRE(c && logits && mask && rng && actions && logp && E >= 0, "bad argument");
  BK_REQUIRE(c->dp.P == 2 && c->dp.N == 7 && (c->dp.num_pieces == 9 || c->dp.num_pieces == 21),
             "policy sampling: the 2-player 7x7 presets (919 / 2522 ids)");
  if (E == 0) return BK_OK;
  const dim3 grid((E + 15) / 16), block(kVecThreads);
  hipStream_t st = (hipStream_t)stream;
  if (c->dp.num_pieces == 9) {
    if (zero_masked)
      hipLaunchKernelGGL((k_vec_policy<4, true>), grid, block, 0, st, logits, mask, rng, E, actions, logp);
    else
      hipLaunchKernelGGL((k_vec_policy<4, false>), grid, block, 0, st, logits, mask, rng, E, actions, logp);
  } else {
    if (zero_masked)
      hipLaunchKernelGGL((k_vec_policy<5, true>), grid, block, 0, st, logits, mask, rng, E, actions, logp);
    else
      hipLaunchKernelGGL((k_vec_policy<5, false>), grid, block, 0, st, logits, mask, rng, E, actions, logp);
  }
  return launch_check("k_vec_policy");
}

int bk_vec_step_policy(bk_ctx* c, void* states, uint64_t* rng, const float* logits, int zero_masked, int E,
                       uint8_t* obs, uint64_t* mask, float* reward, int32_t* done, int32_t* actions, float* logp,
                       void* stream) {
  BK_REQUIRE(c && states && rng && logits && obs && mask && reward && done && actions && logp && E >= 0,
             "bad argument");
  BK_REQUIRE(c->dp.P == 2 && c->dp.N == 7 && (c->dp.num_pieces == 9 || c->dp.num_pieces == 21),
             "the fused policy step: the 2-player 7x7 presets (919 / 2522 ids)");
  if (E == 0) return BK_OK;
  const dim3 grid((E + kVecThreads / 16 - 1) / (kVecThreads / 16));
  hipStream_t st = (hipStream_t)stream;
  uint32_t* sp = (uint32_t*)states;
#define BK_SP(MC, P)                                                                                              \
  hipLaunchKernelGGL((k_vec_step7<MC, 16, P>), grid, dim3(kVecThreads), 0, st, sp, rng, (const int32_t*)nullptr, E, \
                     obs, mask, reward, done, logits, actions, logp)
  if (c->dp.num_pieces == 9) {
    if (zero_masked) BK_SP(4, 2); else BK_SP(4, 1);
  } else {
    if (zero_masked) BK_SP(5, 2); else BK_SP(5, 1);
  }
#undef BK_SP
  return launch_check("k_vec_step7<policy>");
}

}  // extern "C"
