// ply.hip — the batched self-play ply's tail after the search: what
// trainer.py:108-137 does per game between two searches, for every game of the batch in two
// launches instead of ~90 small PyTorch kernels.
//
// * k_ply_policy — one workgroup per game: root-only Dirichlet noise on the game's first ply
//   (trainer.py:110-116: pi = (1 - w) pi + w Dir(alpha) over the legal ids, in float64), the
//   float32 pi the episode records (trainer.py:124-126), a draw of the action from it
//   (np.random.choice(len(pi), p=pi), trainer.py:125) by inverse CDF over the float32
//   probabilities, and the per-ply record fields (int16 ids, float32 pi, mover, active flag).
//   Random numbers: counter-based (splitmix64 of seed, ply, game, draw index), so a ply's draws do
//   not depend on launch order; the law is pinned statistically
//   (tests/test_selfplay_gpu.py::test_play_ply_sampling_statistics). Gamma(alpha) by
//   Marsaglia-Tsang (alpha = 1: an exact exponential draw), bounded retries.
// * k_ply_finish — one workgroup for the batch: the games that ended this ply record z (the
//   final scores, trainer.py:134-135) under their game id, count as finished, flag their tree for
//   reset (a new MCTS per episode, trainer.py:95); in continuous mode their slot restarts from the
//   empty board with the next game ids (an exclusive prefix count over the batch), otherwise it
//   goes inactive. Also the first-ply flags, the simulation counter and the root-overflow latch.
// Bound: latency (a few KB per game); the point is the launch count.
#include "../../include/blokus_engine.h"
#include "common.h"
#include "ctx.h"

namespace bk {
namespace {

constexpr int kPlyThreads = 256;
constexpr int kPlyMaxCap = 4096;  // LDS: cap doubles of noise + cap floats of pi

__device__ __forceinline__ uint64_t ply_rng(uint64_t seed, uint64_t ply, int game, int draw) {
  return mix64(mix64(seed ^ mix64(ply)) + ((uint64_t)(uint32_t)game << 24) + (uint64_t)(uint32_t)draw);
}
// uniform in (0, 1]: 53 random bits
__device__ __forceinline__ double u01(uint64_t x) { return ((double)(x >> 11) + 1.0) * 0x1.0p-53; }

// Gamma(alpha, 1): alpha = 1 -> -log(u); else Marsaglia-Tsang (alpha < 1 boosted by u^(1/alpha)),
// normals by Box-Muller; at most 32 rounds (the acceptance rate is > 95% per round for alpha >= 1)
constexpr int kGammaSlots = 128;  // draw slots per entry: the boost + 3 per round x 32 rounds = 97 <= 128
__device__ double gamma_draw(double alpha, uint64_t seed, uint64_t ply, int game, int idx) {
  int k = idx * kGammaSlots;
  if (alpha == 1.0) return -log(u01(ply_rng(seed, ply, game, k)));
  double boost = 1.0, a = alpha;
  if (a < 1.0) {
    boost = pow(u01(ply_rng(seed, ply, game, k++)), 1.0 / a);
    a += 1.0;
  }
  const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int round = 0; round < 32; ++round) {
    const double u1 = u01(ply_rng(seed, ply, game, k++)), u2 = u01(ply_rng(seed, ply, game, k++));
    const double x = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = u01(ply_rng(seed, ply, game, k++));
    if (u < 1.0 - 0.0331 * x * x * x * x || log(u) < 0.5 * x * x + d * (1.0 - v + log(v))) return d * v * boost;
  }
  return d * boost;  // (not reached in practice: 32 rejections in a row)
}

// sum over the workgroup (kPlyThreads = 4 waves); sh: 4 doubles of LDS; barriers inside
__device__ __forceinline__ double block_sum_d(double x, double* sh) {
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane_id() == 0) sh[w] = x;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__global__ __launch_bounds__(kPlyThreads) void k_ply_policy(const int32_t* __restrict__ ids,
                                                           const double* __restrict__ pi,
                                                           const int32_t* __restrict__ counts,
                                                           const int32_t* __restrict__ active,
                                                           const uint8_t* __restrict__ first_ply, int cap,
                                                           double weight, double alpha, uint64_t seed, uint64_t ply,
                                                           const uint32_t* __restrict__ roots,
                                                           int32_t* __restrict__ action, int16_t* __restrict__ ids16,
                                                           float* __restrict__ pi32, uint8_t* __restrict__ act_mask,
                                                           int32_t* __restrict__ player) {
  __shared__ double noise[kPlyMaxCap];
  __shared__ float p32[kPlyMaxCap];
  __shared__ double red[4];
  __shared__ double scan[kPlyThreads];
  __shared__ int pick;
  const int g = blockIdx.x, tid = threadIdx.x;
  const int Kraw = counts[g];
  const bool act = active[g] != 0 && Kraw > 0;
  const int K = Kraw > 0 ? Kraw : 0;  // counts < 0: the root had more than cap children (latched by k_ply_finish)
  const bool mix = act && first_ply[g] != 0;
  const int32_t* id_row = ids + (size_t)g * cap;
  const double* pi_row = pi + (size_t)g * cap;
  if (tid == 0) {
    player[g] = (int32_t)roots[(size_t)g * kStateWords + kWToMove];
    act_mask[g] = act ? 1 : 0;
    pick = -1;
  }
  // Dirichlet(alpha) over the K legal ids: Gamma draws normalised by their sum
  double gs = 0.0;
  if (mix) {
    for (int i = tid; i < K; i += kPlyThreads) {
      const double x = gamma_draw(alpha, seed, ply, g, i);
      noise[i] = x;
      gs += x;
    }
  }
  gs = mix ? block_sum_d(gs, red) : 0.0;
  for (int i = tid; i < cap; i += kPlyThreads) {
    float p = 0.0f;
    if (i < K) {
      double v = pi_row[i];
      if (mix) v = v * (1.0 - weight) + (noise[i] / (gs > 1e-300 ? gs : 1e-300)) * weight;
      p = (float)v;
    }
    p32[i] = p;
    pi32[(size_t)g * cap + i] = p;
    ids16[(size_t)g * cap + i] = (int16_t)(i < K ? id_row[i] : 0);
  }
  if (!act) {
    if (tid == 0) action[g] = -1;
    return;
  }
  __syncthreads();
  // inverse CDF: contiguous chunks per thread, an exclusive scan of the chunk sums, then the
  // thread whose chunk holds the target walks it
  const int C = (K + kPlyThreads - 1) / kPlyThreads, lo = tid * C, hi = lo + C < K ? lo + C : K;
  double cs = 0.0;
  for (int i = lo; i < hi; ++i) cs += (double)p32[i];
  scan[tid] = cs;
  __syncthreads();
  if (tid < 64) {  // wave 0 scans the 256 chunk sums (4 per lane)
    const double a0 = scan[4 * tid], a1 = scan[4 * tid + 1], a2 = scan[4 * tid + 2], a3 = scan[4 * tid + 3];
    const double s4 = ((a0 + a1) + a2) + a3;
    double inc = s4;
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(inc, o, 64);
      if (tid >= o) inc += y;
    }
    const double ex = inc - s4;
    scan[4 * tid] = ex;
    scan[4 * tid + 1] = ex + a0;
    scan[4 * tid + 2] = (ex + a0) + a1;
    scan[4 * tid + 3] = ((ex + a0) + a1) + a2;
    if (tid == 63) red[0] = inc;
  }
  __syncthreads();
  const double total = red[0];
  const double target = (1.0 - u01(ply_rng(seed, ply, g, 0x7fffffff))) * total;  // [0, total)
  const double base = scan[tid];
  if (hi > lo && target >= base && target < base + cs) {
    // the chunk claims the target: its first entry whose running sum passes it, or — when the walk
    // (base + p0 + p1 + ...) rounds below the chunk test's base + cs — its last positive entry
    double acc = base;
    int last = -1, at = -1;
    for (int i = lo; i < hi; ++i) {
      acc += (double)p32[i];
      if (p32[i] > 0.0f) {
        last = i;
        if (acc > target) {
          at = i;
          break;
        }
      }
    }
    if (at < 0) at = last;
    if (at >= 0) atomicMax(&pick, at);
  }
  __syncthreads();
  if (tid == 0) {
    int i = pick;
    if (i < 0) {  // no chunk claimed the target (rounding at the very end): the last positive entry
      for (i = K - 1; i > 0 && !(p32[i] > 0.0f); --i) {
      }
    }
    action[g] = id_row[i];
  }
}

constexpr int kFinThreads = 1024;

__global__ __launch_bounds__(kFinThreads) void k_ply_finish(int G, int P, const int32_t* __restrict__ ended,
                                                            const double* __restrict__ scores,
                                                            const int32_t* __restrict__ counts,
                                                            const uint8_t* __restrict__ act_mask,
                                                            const int64_t* __restrict__ game_id,
                                                            const uint32_t* __restrict__ roots,
                                                            const uint32_t* __restrict__ init_state, int continuous,
                                                            int num_sims, int32_t* __restrict__ active,
                                                            uint8_t* __restrict__ first_ply,
                                                            int32_t* __restrict__ reset_flags,
                                                            int64_t* __restrict__ game_id_out,
                                                            uint32_t* __restrict__ roots_out,
                                                            float* __restrict__ z_table, uint8_t* __restrict__ z_known,
                                                            int64_t zcap, int64_t* __restrict__ next_gid,
                                                            int64_t* __restrict__ fin_count,
                                                            int64_t* __restrict__ sims_count,
                                                            int32_t* __restrict__ cap_overflow) {
  __shared__ int wsum[kFinThreads / 64];
  __shared__ int base_sh, over_sh, acts_sh;
  const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
  if (tid == 0) {
    base_sh = 0;
    over_sh = 0;
    acts_sh = 0;
  }
  __syncthreads();
  const int64_t gid0 = *next_gid;
  for (int c0 = 0; c0 < G; c0 += kFinThreads) {
    const int g = c0 + tid;
    const bool in = g < G;
    const bool act = in && active[g] != 0;
    const bool done = act && ended[g] != 0;
    if (in && act && counts[g] < 0) atomicOr(&over_sh, 1);
    if (in && act_mask[g]) atomicAdd(&acts_sh, 1);
    // the position of this game among the batch's finished games: ballot prefix + wave offsets
    const uint64_t bal = __ballot(done);
    const int below = __popcll(bal & ((1ull << l) - 1ull));
    if (l == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base_sh;
    for (int i = 0; i < w; ++i) off += wsum[i];
    int chunk = 0;
    for (int i = 0; i < kFinThreads / 64; ++i) chunk += wsum[i];
    if (in) {
      const int64_t gid = game_id[g];
      if (done && gid >= 0 && gid < zcap) {
        for (int q = 0; q < P; ++q) z_table[gid * P + q] = (float)scores[(size_t)g * P + q];
        z_known[gid] = 1;
      }
      reset_flags[g] = done ? 1 : 0;
      const uint8_t fp = (uint8_t)((first_ply[g] && !act_mask[g]) || (continuous && done));
      first_ply[g] = fp;
      const uint4* src = reinterpret_cast<const uint4*>((continuous && done) ? init_state : roots + (size_t)g * kStateWords);
      uint4* dst = reinterpret_cast<uint4*>(roots_out + (size_t)g * kStateWords);
#pragma unroll
      for (int k = 0; k < kStateWords / 4; ++k) dst[k] = src[k];
      if (continuous)
        game_id_out[g] = done ? gid0 + off + below : gid;
      else {
        game_id_out[g] = gid;
        if (done) active[g] = 0;
      }
    }
    __syncthreads();
    if (tid == 0) base_sh += chunk;
    __syncthreads();
  }
  if (tid == 0) {
    *fin_count += base_sh;
    if (continuous) *next_gid = gid0 + base_sh;
    *sims_count += (int64_t)num_sims * acts_sh;
    if (over_sh) *cap_overflow = 1;
  }
}

}  // namespace
}  // namespace bk

using namespace bk;

extern "C" {

int bk_ply_policy(const int32_t* ids, const double* pi, const int32_t* counts, const int32_t* active,
                  const uint8_t* first_ply, int G, int cap, double dirichlet_weight, double dirichlet_alpha,
                  uint64_t seed, uint64_t ply, const void* roots, int32_t* action, int16_t* ids16, float* pi32,
                  uint8_t* act_mask, int32_t* player, void* stream) {
  BK_REQUIRE(ids && pi && counts && active && first_ply && roots && action && ids16 && pi32 && act_mask && player,
             "bad argument");
  BK_REQUIRE(G >= 0 && cap > 0 && cap <= kPlyMaxCap, "bk_ply_policy: 0 < cap <= 4096");
  BK_REQUIRE(dirichlet_alpha > 0.0 && dirichlet_weight >= 0.0 && dirichlet_weight <= 1.0,
             "bk_ply_policy: alpha > 0, 0 <= weight <= 1");
  if (G == 0) return BK_OK;
  hipLaunchKernelGGL(k_ply_policy, dim3(G), dim3(kPlyThreads), 0, (hipStream_t)stream, ids, pi, counts, active,
                     first_ply, cap, dirichlet_weight, dirichlet_alpha, seed, ply, (const uint32_t*)roots, action,
                     ids16, pi32, act_mask, player);
  return launch_check("k_ply_policy");
}

int bk_ply_finish(int G, int P, const int32_t* ended, const double* scores, const int32_t* counts,
                  const uint8_t* act_mask, const int64_t* game_id, const void* roots, const void* init_state,
                  int continuous, int num_sims, int32_t* active, uint8_t* first_ply, int32_t* reset_flags,
                  int64_t* game_id_out, void* roots_out, float* z_table, uint8_t* z_known, int64_t zcap,
                  int64_t* next_gid, int64_t* fin_count, int64_t* sims_count, int32_t* cap_overflow, void* stream) {
  BK_REQUIRE(ended && scores && counts && act_mask && game_id && roots && init_state && active && first_ply &&
                 reset_flags && game_id_out && roots_out && z_table && z_known && next_gid && fin_count &&
                 sims_count && cap_overflow,
             "bad argument");
  BK_REQUIRE(G >= 0 && P > 0 && zcap >= 0 && roots_out != roots, "bk_ply_finish: bad sizes (roots_out != roots)");
  BK_REQUIRE((((uintptr_t)roots | (uintptr_t)roots_out | (uintptr_t)init_state) & 15u) == 0,
             "bk_ply_finish: 16-byte aligned states");
  if (G == 0) return BK_OK;
  hipLaunchKernelGGL(k_ply_finish, dim3(1), dim3(kFinThreads), 0, (hipStream_t)stream, G, P, ended, scores, counts,
                     act_mask, game_id, (const uint32_t*)roots, (const uint32_t*)init_state, continuous, num_sims,
                     active, first_ply, reset_flags, game_id_out, (uint32_t*)roots_out, z_table, z_known, zcap,
                     next_gid, fin_count, sims_count, cap_overflow);
  return launch_check("k_ply_finish");
}

}  // extern "C"
